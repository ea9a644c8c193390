// ubench_gen.hip -- memory-only model of packed-Shamir share-gen (packed_gen.hip) at the bench's full
// launch: V = 1,000 vectors x 1M-dim, k = 8, t = 7, n = 26 -> B = 125,000 batches per vector;
//   secrets [V][D] i64, draws [V][B][t] i64, shares [V][n][B] i64 (batched.rs:25-28: clerk-major rows).
// 41 GB per launch, 63 % of it writes.  No arithmetic: a lane folds its batch's 15 input words by XOR and
// stores (fold + row) sign-extended, so every byte the real kernel moves is moved here, in the real
// layout, by the real tile (256 batches per 256-lane workgroup, inputs staged through LDS).
//
// Knobs (template): LD  input staging   0 = 8-byte loads per lane -> LDS (packed_gen.hip today)
//                                       1 = 16-byte loads per lane -> LDS
//                                       2 = global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip)
//                   ST  share stores    0 = v_permlane32_swap pairs, dwordx4: lanes 0-31 row j, 32-63 row j+1
//                                           (packed_gen.hip today; 512 B per row per wave-instruction)
//                                       1 = LDS transpose, then 1 KiB of ONE row per wave-instruction
//                                       2 = one batch per lane, dwordx2 (512 B per row per instruction)
//                   POL store policy    0 = nt, 1 = plain, 2 = sc1 (buffer store, aux 16), 3 = sc0 sc1 nt
//                   runtime: remap of the workgroup id (0 = natural, 1 = XCD-chunked), rows rotated per wave.
// Reference streams at the same size: flat copy, flat read, write-only rows.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_gen.hip -o tools/ubench_gen && ./tools/ubench_gen [V]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

constexpr int K = 8, T = 7, NR = 26, BS = 256;
constexpr uint64_t D = 1000000, B = D / K;   // 125,000 batches per vector
typedef int32_t v4i __attribute__((ext_vector_type(4)));
typedef int64_t v2l __attribute__((ext_vector_type(2)));

template <int POL>
__device__ __forceinline__ void store16(v4i v, int64_t* rowbase, uint32_t byte_off, __amdgpu_buffer_rsrc_t rs) {
    if constexpr (POL == 0) __builtin_nontemporal_store(v, reinterpret_cast<v4i*>((char*)rowbase + byte_off));
    else if constexpr (POL == 1) *reinterpret_cast<v4i*>((char*)rowbase + byte_off) = v;
    else if constexpr (POL == 2) __builtin_amdgcn_raw_buffer_store_b128(v, rs, byte_off, 0, 16);
    else __builtin_amdgcn_raw_buffer_store_b128(v, rs, byte_off, 0, 16 | 2 | 1);
}

template <int LD, int ST, int POL>
__global__ __launch_bounds__(BS) void gen_mem(const int64_t* __restrict__ sec, const int64_t* __restrict__ dr,
                                              int64_t* __restrict__ out, uint32_t V, int remap, int rotate) {
    __shared__ __attribute__((aligned(16))) int64_t lds[BS * (K + T)];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t gx = gridDim.x;
    uint32_t L = blockIdx.x + blockIdx.y * gx;
    if (remap == 1) {   // XCD-chunked: XCD x (= L % 8, dispatch round-robin) walks a contiguous 1/8 of the tiles
        const uint32_t total = gx * gridDim.y, per = (total + 7) / 8;
        const uint32_t nl = (L % 8) * per + L / 8;
        if (nl >= total) return;
        L = nl;
    } else if (remap >= 2) {   // XCD super-tiles of S = remap consecutive tiles, the 8 XCDs on adjacent super-tiles
        const uint32_t S = (uint32_t)remap, total = gx * gridDim.y, round = total / (8 * S) * (8 * S);
        if (L < round) {
            const uint32_t x = L % 8, j = L / 8;
            L = ((j / S) * 8 + x) * S + j % S;
        }
    }
    const uint32_t vec = L / gx, tile = L % gx;
    const uint64_t b0 = (uint64_t)tile * BS;
    const uint32_t nb = (uint32_t)std::min<uint64_t>(BS, B - b0);
    const int64_t* ssrc = sec + (uint64_t)vec * D + b0 * K;
    const int64_t* dsrc = dr + ((uint64_t)vec * B + b0) * T;
    // ---- inputs -> LDS ----
    const uint32_t ns = nb * K, nd = nb * T;
    if constexpr (LD == 0) {
        for (uint32_t base = 0; base < ns; base += 8 * BS) {
            int64_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) { const uint32_t e = base + u * BS + tid; v[u] = __builtin_nontemporal_load(ssrc + (e < ns ? e : 0)); }
#pragma unroll
            for (int u = 0; u < 8; ++u) { const uint32_t e = base + u * BS + tid; if (e < ns) lds[e] = v[u]; }
        }
        for (uint32_t base = 0; base < nd; base += 8 * BS) {
            int64_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) { const uint32_t e = base + u * BS + tid; v[u] = __builtin_nontemporal_load(dsrc + (e < nd ? e : 0)); }
#pragma unroll
            for (int u = 0; u < 8; ++u) { const uint32_t e = base + u * BS + tid; if (e < nd) lds[BS * K + e] = v[u]; }
        }
    } else if constexpr (LD == 1) {
        const v2l* s2 = reinterpret_cast<const v2l*>(ssrc);
        const v2l* d2 = reinterpret_cast<const v2l*>(dsrc);   // b0 * T even (BS even)
        v2l* l2 = reinterpret_cast<v2l*>(lds);
        const uint32_t ns2 = ns / 2, nd2 = (nd + 1) / 2;
        v2l v[8];
#pragma unroll
        for (int u = 0; u < 4; ++u) { const uint32_t e = u * BS + tid; v[u] = __builtin_nontemporal_load(s2 + (e < ns2 ? e : 0)); }
#pragma unroll
        for (int u = 0; u < 4; ++u) { const uint32_t e = u * BS + tid; v[4 + u] = __builtin_nontemporal_load(d2 + (e < nd2 ? e : 0)); }
#pragma unroll
        for (int u = 0; u < 4; ++u) { const uint32_t e = u * BS + tid; if (e < ns2) l2[e] = v[u]; }
#pragma unroll
        for (int u = 0; u < 4; ++u) { const uint32_t e = u * BS + tid; if (e < nd2) l2[BS * K / 2 + e] = v[4 + u]; }
    } else {
        // LDS-DMA: each wave-instruction moves 1 KiB; wave w takes KiB pieces w, w + 4, ...
        const uint32_t spieces = (ns * 8 + 1023) / 1024, dpieces = (nd * 8 + 1023) / 1024;
        for (uint32_t pc = wave; pc < spieces + dpieces; pc += 4) {
            const bool isd = pc >= spieces;
            const uint32_t q = isd ? pc - spieces : pc;
            const char* g = isd ? (const char*)dsrc + q * 1024 : (const char*)ssrc + q * 1024;
            char* l = (char*)lds + (isd ? BS * K * 8 : 0) + q * 1024;
            __builtin_amdgcn_global_load_lds((const void*)(g + lane * 16), (__attribute__((address_space(3))) void*)l, 16, 0, 2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // ---- per-lane fold (the transform's stand-in) ----
    const uint32_t half = lane >> 5;
    const uint32_t lb = (ST == 0) ? (tid & ~63u) + 2 * (lane & 31) + half : tid;
    int32_t acc = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) acc ^= (int32_t)lds[lb * K + i];
#pragma unroll
    for (int i = 0; i < T; ++i) acc ^= (int32_t)lds[BS * K + lb * T + i];
    acc &= 0x7fffffff;
    if (acc == 0x7fffffff) acc = -1;   // keep the sign path live
    int64_t* vbase = out + (uint64_t)vec * NR * B;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(vbase, 0, (int)(NR * B * 8), 0x00020000);
    const uint32_t rot = rotate ? (wave * 7 + tile) % (NR / 2) : 0;
    if constexpr (ST == 0) {
        const uint32_t pb_off = (tid & ~63u) + 2 * (lane & 31);
        const uint64_t pb = b0 + pb_off;
        const bool st = pb < b0 + nb;
#pragma unroll
        for (int qq = 0; qq < NR / 2; ++qq) {
            const int q = rotate ? (int)((qq + rot) % (NR / 2)) : qq;
            const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)(acc + 1 + 2 * q), (uint32_t)(acc + 2 + 2 * q), false, false);
            const int32_t lo = (int32_t)r[0], hi = (int32_t)r[1];
            const v4i val = {lo, lo >> 31, hi, hi >> 31};
            const uint32_t row = 2 * q + half;
            if (st) store16<POL>(val, vbase, (uint32_t)((row * B + pb) * 8), rs);
        }
    } else if constexpr (ST == 1) {
        __syncthreads();                                     // every lane has read its inputs
        int32_t* l32 = reinterpret_cast<int32_t*>(lds);       // [NR][BS] int32 (26 KiB <= 30 KiB)
#pragma unroll
        for (int j = 0; j < NR; ++j) l32[j * BS + tid] = acc + 1 + j;
        __syncthreads();
        // 52 (row, half) pieces of 1 KiB; wave w takes pieces w, w + 4, ...
#pragma unroll
        for (int i = 0; i < 13; ++i) {
            const uint32_t pc0 = wave + 4 * i;
            const uint32_t pc = rotate ? (pc0 + 4 * rot) % (2 * NR) : pc0;
            const uint32_t row = pc >> 1, h = pc & 1;
            const uint32_t bl = h * 128 + 2 * lane;
            const int2 w = *reinterpret_cast<const int2*>(l32 + row * BS + bl);
            const v4i val = {w.x, w.x >> 31, w.y, w.y >> 31};
            if (bl < nb) store16<POL>(val, vbase, (uint32_t)((row * B + b0 + bl) * 8), rs);
        }
    } else {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            int64_t* p = vbase + (uint64_t)j * B + b0 + tid;
            if (tid < nb) {
                if constexpr (POL == 1) *p = (int64_t)(acc + 1 + j);
                else __builtin_nontemporal_store((int64_t)(acc + 1 + j), p);
            }
        }
    }
}

// Memory-only model of the reveal (packed_reveal.hip): a lane reads its batch's NI shares from the
// [V][NI][B] clerk rows (1 MB apart) and writes the batch's K secrets; the workgroup's 256 x K results go
// through LDS so the [V][D] output is written with coalesced 16-byte stores (the reveal's STAGED flush).
constexpr int NI = 15;
template <bool NT_LOAD, bool XCD>
__global__ __launch_bounds__(BS) void reveal_mem(const int64_t* __restrict__ sh, int64_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) int64_t lds[BS * K];
    const uint32_t tid = threadIdx.x;
    const uint64_t total = (uint64_t)gridDim.x * gridDim.y;
    uint64_t L = blockIdx.x + (uint64_t)blockIdx.y * gridDim.x;
    if (XCD) {
        const uint64_t q = total / 8, r = total % 8, x = L % 8;
        L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + L / 8;
    }
    const uint64_t vec = L / gridDim.x, tile = L % gridDim.x;
    const uint64_t b0 = tile * BS, b = b0 + tid;
    const uint64_t nb = std::min<uint64_t>(BS, B - b0);
    const int64_t* src = sh + vec * NI * B + (b < B ? b : B - 1);
    int64_t v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) v[i] = NT_LOAD ? __builtin_nontemporal_load(src + (uint64_t)i * B) : src[(uint64_t)i * B];
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < NI; ++i) acc ^= v[i];
#pragma unroll
    for (int e = 0; e < K; ++e) lds[tid * K + e] = acc + e;
    __syncthreads();
    v2l* o = reinterpret_cast<v2l*>(out + vec * D + b0 * K);
    const v2l* l2 = reinterpret_cast<const v2l*>(lds);
    for (uint32_t j = tid; j < nb * K / 2; j += BS) __builtin_nontemporal_store(l2[j], o + j);
}

__global__ __launch_bounds__(256) void copy_flat(const v2l* __restrict__ src, v2l* __restrict__ dst, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ __launch_bounds__(256) void read_flat(const v2l* __restrict__ src, uint64_t n, int64_t* __restrict__ sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    int64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const v2l v = __builtin_nontemporal_load(src + i);
        acc ^= v[0] + v[1];
    }
    if (acc == 0x123456789) sink[0] = acc;
}

// the share rows alone, same grid and store shape as ST = 0 (no reads)
__global__ __launch_bounds__(BS) void write_rows(int64_t* __restrict__ out) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, half = lane >> 5;
    const uint32_t vec = blockIdx.y, tile = blockIdx.x;
    const uint64_t pb = (uint64_t)tile * BS + (tid & ~63u) + 2 * (lane & 31);
    if (pb >= B) return;
    int64_t* vbase = out + (uint64_t)vec * NR * B;
#pragma unroll
    for (int q = 0; q < NR / 2; ++q) {
        const int32_t x = (int32_t)(pb ^ q);
        const v4i val = {x, 0, x + 1, 0};
        __builtin_nontemporal_store(val, reinterpret_cast<v4i*>(vbase + (uint64_t)(2 * q + half) * B + pb));
    }
}

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s failed at line %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

struct Res { char name[64]; float best, med; double bytes; };

template <class F>
static Res timeit(const char* name, double bytes, F launch, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a, 0));
        launch();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float t = 0;
        CHECK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t);
    }
    CHECK(hipGetLastError());
    std::sort(ms.begin(), ms.end());
    Res r;
    snprintf(r.name, sizeof r.name, "%s", name);
    r.best = ms[0];
    r.med = ms[ms.size() / 2];
    r.bytes = bytes;
    printf("%-44s best %8.3f ms  %6.3f TB/s   median %8.3f ms  %6.3f TB/s\n", name, r.best, bytes / (r.best * 1e-3) / 1e12,
           r.med, bytes / (r.med * 1e-3) / 1e12);
    fflush(stdout);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return r;
}

// A share buffer of `bytes` built from physical chunks of `chunk` bytes (hipMemCreate), mapped into one
// virtual range in order (shuffle = 0) or in a random order (shuffle = 1), so the buffer is physically
// contiguous at most at the chunk's granularity.
struct VmmBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    std::vector<hipMemGenericAllocationHandle_t> h;
};
static VmmBuf vmm_alloc(size_t bytes, size_t chunk, int shuffle) {
    VmmBuf b;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    chunk = (chunk + gran - 1) / gran * gran;
    const size_t n = (bytes + chunk - 1) / chunk;
    b.bytes = n * chunk;
    CHECK(hipMemAddressReserve(&b.ptr, b.bytes, chunk, nullptr, 0));
    b.h.resize(n);
    for (size_t i = 0; i < n; ++i) CHECK(hipMemCreate(&b.h[i], chunk, &prop, 0));
    std::vector<size_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = i;
    if (shuffle) {
        uint64_t s = 0x9e3779b97f4a7c15ull;
        for (size_t i = n - 1; i > 0; --i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            std::swap(order[i], order[s % (i + 1)]);
        }
    }
    for (size_t i = 0; i < n; ++i) CHECK(hipMemMap((char*)b.ptr + i * chunk, chunk, 0, b.h[order[i]], 0));
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CHECK(hipMemSetAccess(b.ptr, b.bytes, &acc, 1));
    return b;
}
static void vmm_free(VmmBuf& b) {
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemUnmap(b.ptr, b.bytes));
    for (auto& h : b.h) CHECK(hipMemRelease(h));
    CHECK(hipMemAddressFree(b.ptr, b.bytes));
}

int main(int argc, char** argv) {
    const uint32_t V = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    int64_t *sec, *dr, *out, *sink;
    const size_t sb = (size_t)V * D * 8, db = (size_t)V * B * T * 8, ob = (size_t)V * NR * B * 8;
    if (argc > 3 && argv[3][0] == 'p') {     // placement mode: share-gen (XCD-chunked) into differently built share buffers
        CHECK(hipMalloc(&sec, sb + 4096));
        CHECK(hipMalloc(&dr, db + 4096));
        CHECK(hipMemset(sec, 1, sb));
        CHECK(hipMemset(dr, 2, db));
        const double gen_bytes = (double)(sb + db + ob);
        const dim3 grid((unsigned)((B + BS - 1) / BS), V), blk(BS);
        printf("V = %u: share-gen memory model, XCD-chunked, %.3f GB per launch\n", V, gen_bytes / 1e9);
        auto run = [&](const char* nm, int64_t* o) {
            CHECK(hipMemset(o, 0, ob));
            timeit(nm, gen_bytes, [&] { hipLaunchKernelGGL((gen_mem<0, 0, 0>), grid, blk, 0, 0, sec, dr, o, V, 1, 0); }, reps);
        };
        for (int i = 0; i < 3; ++i) {
            CHECK(hipMalloc(&out, ob));
            char nm[64];
            snprintf(nm, sizeof nm, "hipMalloc share buffer %d", i);
            run(nm, out);
            CHECK(hipFree(out));
        }
        const size_t MB = 1 << 20;
        for (size_t chunk : {2 * MB, 64 * MB, 1024 * MB}) {
            for (int shuffle : {0, 1}) {
                VmmBuf b = vmm_alloc(ob, chunk, shuffle);
                char nm[64];
                snprintf(nm, sizeof nm, "VMM %5zu MiB chunks, %s", chunk / MB, shuffle ? "shuffled" : "in order");
                run(nm, (int64_t*)b.ptr);
                vmm_free(b);
            }
        }
        return 0;
    }
    CHECK(hipMalloc(&sec, sb + 4096));
    CHECK(hipMalloc(&dr, db + 4096));
    CHECK(hipMalloc(&out, ob));
    CHECK(hipMalloc(&sink, 8));
    CHECK(hipMemset(sec, 1, sb));
    CHECK(hipMemset(dr, 2, db));
    CHECK(hipMemset(out, 0, ob));
    const double gen_bytes = (double)(sb + db + ob);
    printf("V = %u vectors x 1M-dim, k = %d t = %d n = %d: %.3f GB per launch (%.0f %% writes)\n", V, K, T, NR,
           gen_bytes / 1e9, 100.0 * ob / gen_bytes);
    const dim3 grid((unsigned)((B + BS - 1) / BS), V), blk(BS);
#define GEN(LD, ST, POL, RM, ROT, NAME)                                                                         \
    timeit(NAME, gen_bytes, [&] { hipLaunchKernelGGL((gen_mem<LD, ST, POL>), grid, blk, 0, 0, sec, dr, out, V, RM, ROT); }, reps)
    if (argc > 3) {     // quick mode: the XCD order variants only
        GEN(0, 0, 0, 0, 0, "natural order");
        GEN(0, 0, 0, 1, 0, "XCD-chunked (eighths of the grid)");
        for (int S : {4, 16, 64, 256, 1024}) {
            char nm[64];
            snprintf(nm, sizeof nm, "XCD super-tiles of %d tiles", S);
            timeit(nm, gen_bytes, [&] { hipLaunchKernelGGL((gen_mem<0, 0, 0>), grid, blk, 0, 0, sec, dr, out, V, S, 0); }, reps);
        }
        return 0;
    }
    GEN(0, 0, 0, 0, 0, "today: ld8 -> LDS, permlane x4 nt");
    GEN(1, 0, 0, 0, 0, "ld16 -> LDS, permlane x4 nt");
    GEN(2, 0, 0, 0, 0, "LDS-DMA, permlane x4 nt");
    GEN(0, 1, 0, 0, 0, "ld8, LDS-transposed 1 KiB rows nt");
    GEN(1, 1, 0, 0, 0, "ld16, LDS-transposed 1 KiB rows nt");
    GEN(2, 1, 0, 0, 0, "LDS-DMA, LDS-transposed 1 KiB rows nt");
    GEN(0, 2, 0, 0, 0, "ld8, dwordx2 per lane nt");
    GEN(0, 0, 1, 0, 0, "ld8, permlane x4 plain");
    GEN(0, 0, 2, 0, 0, "ld8, permlane x4 sc1");
    GEN(0, 0, 3, 0, 0, "ld8, permlane x4 sc0 sc1 nt");
    GEN(0, 0, 0, 1, 0, "ld8, permlane x4 nt, XCD-chunked");
    GEN(1, 0, 0, 1, 0, "ld16, permlane x4 nt, XCD-chunked");
    GEN(0, 1, 0, 1, 0, "ld8, 1 KiB rows nt, XCD-chunked");
    GEN(2, 0, 0, 1, 0, "LDS-DMA, permlane x4 nt, XCD-chunked");
    GEN(0, 0, 1, 1, 0, "ld8, permlane x4 plain, XCD-chunked");
    GEN(0, 0, 0, 0, 1, "ld8, permlane x4 nt, rows rotated");
    GEN(1, 1, 0, 0, 1, "ld16, 1 KiB rows nt, rows rotated");
    GEN(1, 1, 2, 0, 0, "ld16, 1 KiB rows sc1");
    GEN(1, 1, 1, 0, 0, "ld16, 1 KiB rows plain");
    {   // reveal pattern: V x 15 share rows in, V x D secrets out (reuses the share-gen buffers)
        const double rbytes = (double)V * NI * B * 8 + (double)V * D * 8;
        int64_t* rsh = out;           // [V][NI][B] fits in [V][NR][B]
        int64_t* rout = sec;          // [V][D]
        timeit("reveal mem: nt loads, natural order", rbytes,
               [&] { hipLaunchKernelGGL((reveal_mem<true, false>), grid, blk, 0, 0, rsh, rout); }, reps);
        timeit("reveal mem: nt loads, XCD-chunked", rbytes,
               [&] { hipLaunchKernelGGL((reveal_mem<true, true>), grid, blk, 0, 0, rsh, rout); }, reps);
        timeit("reveal mem: plain loads, XCD-chunked", rbytes,
               [&] { hipLaunchKernelGGL((reveal_mem<false, true>), grid, blk, 0, 0, rsh, rout); }, reps);
    }
    timeit("write-only rows (no reads)", (double)ob, [&] { hipLaunchKernelGGL(write_rows, grid, blk, 0, 0, out); }, reps);
    const uint64_t n16 = ob / 16 / 2;
    timeit("copy 1:1 flat (read + write bytes)", (double)n16 * 32,
           [&] { hipLaunchKernelGGL(copy_flat, dim3(8192), dim3(256), 0, 0, (const v2l*)out, (v2l*)out + n16, n16); }, reps);
    timeit("read-only flat", (double)ob,
           [&] { hipLaunchKernelGGL(read_flat, dim3(8192), dim3(256), 0, 0, (const v2l*)out, ob / 16, sink); }, reps);
    CHECK(hipDeviceSynchronize());
    return 0;
}
