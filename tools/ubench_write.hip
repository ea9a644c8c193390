// ubench_write.hip -- HBM ceilings on gfx950 for share-gen's read/write mix (packed_gen.hip): per batch a
// lane reads K i64 secrets + T i64 draws and writes N i64 shares, one to each clerk row of the ABI's
// [N][B] output (batched.rs:25-28), rows B*8 bytes apart.  No arithmetic: the loads are folded by XOR
// into every store, so this is the memory-only ceiling of an access pattern.  Variants:
//   rows<BPL>   [N][B] output; a 256-lane block handles 256*BPL batches, so each clerk row receives
//               BPL consecutive 2 KiB pieces from one block (BPL = 1 is share-gen's pattern)
//   batchmajor  [B][N] output (not the ABI's layout): every lane writes N*8 contiguous bytes
//   writeonly   [N][B] stores only (no reads)
//   copy        flat 16-byte nt load -> nt store (1:1)
//   read        flat 16-byte nt loads only
// Prints algorithmic bytes / kernel time (TB/s) per variant, best of REPS.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_write.hip -o tools/ubench_write && ./tools/ubench_write
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int K = 8, T = 7, N = 26;
constexpr uint64_t B = 8000000;   // 64 vectors x 125,000 batches = bench.py's 64 x 1M launch

template <int BPL>
__global__ __launch_bounds__(256) void rows(const int64_t* __restrict__ sec, const int64_t* __restrict__ dr,
                                            int64_t* __restrict__ out) {
#pragma unroll
    for (int q = 0; q < BPL; ++q) {
        const uint64_t b = ((uint64_t)blockIdx.x * BPL + q) * 256 + threadIdx.x;
        if (b >= B) return;
        int64_t acc = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) acc ^= __builtin_nontemporal_load(sec + b * K + i);
#pragma unroll
        for (int i = 0; i < T; ++i) acc ^= __builtin_nontemporal_load(dr + b * T + i);
#pragma unroll
        for (int c = 0; c < N; ++c) __builtin_nontemporal_store(acc + c, out + (uint64_t)c * B + b);
    }
}

// rows<1> with share-gen's coalesced read: the block's 256 x (K + T) input words arrive as 16-byte loads
// and are regrouped per batch in LDS.  PIPE = persistent blocks that issue the next tile's loads before
// the current tile's stores (register double buffer).
constexpr int SV = 256 * K / 2, DV = 256 * T / 2;   // v2 loads per tile: 1024 secrets, 896 draws
constexpr int LPL = (SV + DV + 255) / 256;           // 8 per lane
typedef int64_t v2 __attribute__((ext_vector_type(2)));

template <bool PIPE>
__global__ __launch_bounds__(256) void rows_lds(const v2* __restrict__ sec, const v2* __restrict__ dr,
                                                int64_t* __restrict__ out) {
    __shared__ v2 tile[SV + DV];
    const uint64_t ntiles = B / 256;   // B is a multiple of 256
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    v2 r[LPL];
    auto fetch = [&](uint64_t tt) {
#pragma unroll
        for (int j = 0; j < LPL; ++j) {
            const int i = j * 256 + threadIdx.x;
            if (i < SV) r[j] = __builtin_nontemporal_load(sec + tt * SV + i);
            else if (i < SV + DV) r[j] = __builtin_nontemporal_load(dr + tt * DV + (i - SV));
        }
    };
    fetch(t);
    for (;;) {
#pragma unroll
        for (int j = 0; j < LPL; ++j) {
            const int i = j * 256 + threadIdx.x;
            if (i < SV + DV) tile[i] = r[j];
        }
        __syncthreads();
        const uint64_t next = t + gridDim.x;
        if (PIPE && next < ntiles) fetch(next);
        const int64_t* ts = (const int64_t*)tile;
        int64_t acc = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) acc ^= ts[threadIdx.x * K + i];
#pragma unroll
        for (int i = 0; i < T; ++i) acc ^= ts[2 * SV + threadIdx.x * T + i];
        const uint64_t b = t * 256 + threadIdx.x;
#pragma unroll
        for (int c = 0; c < N; ++c) __builtin_nontemporal_store(acc + c, out + (uint64_t)c * B + b);
        if (!PIPE || next >= ntiles) return;
        __syncthreads();
        t = next;
    }
}

__global__ __launch_bounds__(256) void batchmajor(const int64_t* __restrict__ sec, const int64_t* __restrict__ dr,
                                                  int64_t* __restrict__ out) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) acc ^= __builtin_nontemporal_load(sec + b * K + i);
#pragma unroll
    for (int i = 0; i < T; ++i) acc ^= __builtin_nontemporal_load(dr + b * T + i);
#pragma unroll
    for (int c = 0; c < N; ++c) __builtin_nontemporal_store(acc + c, out + b * N + c);
}

__global__ __launch_bounds__(256) void writeonly(int64_t* __restrict__ out) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
#pragma unroll
    for (int c = 0; c < N; ++c) __builtin_nontemporal_store((int64_t)(b ^ c), out + (uint64_t)c * B + b);
}

__global__ __launch_bounds__(256) void copy(const v2* __restrict__ src, v2* __restrict__ dst, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ __launch_bounds__(256) void readonly(const v2* __restrict__ src, uint64_t n, int64_t* __restrict__ sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    int64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const v2 v = __builtin_nontemporal_load(src + i);
        acc ^= v[0] + v[1];
    }
    if (acc == 0x123456789) sink[0] = acc;
}

#define CHECK(x)                                                                   \
    do {                                                                           \
        if ((x) != hipSuccess) {                                                   \
            fprintf(stderr, "%s failed at line %d\n", #x, __LINE__);               \
            return 1;                                                              \
        }                                                                          \
    } while (0)

template <class F>
static float best_ms(F launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();   // warm
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(a, 0);
        launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return best;
}

int main() {
    const int reps = 20;
    int64_t *sec, *dr, *out, *sink;
    CHECK(hipMalloc(&sec, B * K * 8));
    CHECK(hipMalloc(&dr, B * T * 8));
    CHECK(hipMalloc(&out, B * N * 8));
    CHECK(hipMalloc(&sink, 8));
    CHECK(hipMemset(sec, 1, B * K * 8));
    CHECK(hipMemset(dr, 2, B * T * 8));
    const double gen_bytes = (double)B * (K + T + N) * 8, w_bytes = (double)B * N * 8;
    const unsigned g1 = (unsigned)((B + 255) / 256);
    struct {
        const char* name;
        float ms;
        double bytes;
    } res[16];
    int nr = 0;
    res[nr++] = {"rows<1> (share-gen pattern)",
                 best_ms([&] { hipLaunchKernelGGL(rows<1>, dim3(g1), dim3(256), 0, 0, sec, dr, out); }, reps), gen_bytes};
    res[nr++] = {"rows<2>", best_ms([&] { hipLaunchKernelGGL(rows<2>, dim3((g1 + 1) / 2), dim3(256), 0, 0, sec, dr, out); }, reps),
                 gen_bytes};
    res[nr++] = {"rows<4>", best_ms([&] { hipLaunchKernelGGL(rows<4>, dim3((g1 + 3) / 4), dim3(256), 0, 0, sec, dr, out); }, reps),
                 gen_bytes};
    res[nr++] = {"rows_lds (coalesced reads via LDS)",
                 best_ms([&] { hipLaunchKernelGGL(rows_lds<false>, dim3(g1), dim3(256), 0, 0, (const v2*)sec, (const v2*)dr, out); }, reps),
                 gen_bytes};
    for (int per_cu : {2, 4, 8}) {
        static char names[3][48];
        char* nm = names[per_cu == 2 ? 0 : per_cu == 4 ? 1 : 2];
        snprintf(nm, 48, "rows_lds pipelined, %d blocks/CU", per_cu);
        res[nr++] = {nm, best_ms([&] { hipLaunchKernelGGL(rows_lds<true>, dim3(256 * per_cu), dim3(256), 0, 0, (const v2*)sec, (const v2*)dr, out); }, reps),
                     gen_bytes};
    }
    res[nr++] = {"batchmajor", best_ms([&] { hipLaunchKernelGGL(batchmajor, dim3(g1), dim3(256), 0, 0, sec, dr, out); }, reps),
                 gen_bytes};
    res[nr++] = {"writeonly [N][B]", best_ms([&] { hipLaunchKernelGGL(writeonly, dim3(g1), dim3(256), 0, 0, out); }, reps), w_bytes};
    const uint64_t n16 = B * N * 8 / 16 / 2;   // copy half the output buffer into the other half
    res[nr++] = {"copy 1:1 (bytes = read + write)",
                 best_ms([&] { hipLaunchKernelGGL(copy, dim3(8192), dim3(256), 0, 0, (const v2*)out, (v2*)out + n16, n16); }, reps),
                 (double)n16 * 32};
    res[nr++] = {"read only", best_ms([&] { hipLaunchKernelGGL(readonly, dim3(8192), dim3(256), 0, 0, (const v2*)out, 2 * n16, sink); }, reps),
                 (double)n16 * 32};
    CHECK(hipDeviceSynchronize());
    printf("B = %llu batches, K = %d, T = %d, N = %d; share-gen bytes per launch %.3f GB (%.0f %% writes)\n",
           (unsigned long long)B, K, T, N, gen_bytes / 1e9, 100.0 * w_bytes / gen_bytes);
    for (int i = 0; i < nr; ++i)
        printf("%-34s %8.4f ms  %6.3f TB/s\n", res[i].name, res[i].ms, res[i].bytes / (res[i].ms * 1e-3) / 1e12);
    return 0;
}
