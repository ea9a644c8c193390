// ubench_mix.hip -- HBM ceiling of a streaming kernel at a given read:write byte mix on gfx950.
// Each lane of a grid-stride loop reads NR 16-byte words of one buffer and writes NW 16-byte words of
// another per step (coalesced, non-temporal both ways, NR loads in flight before the stores).  The
// mixes are those of the packed-Shamir kernels: share-gen reads 15 and writes 26 i64 per 8 secrets
// (k + t in, n out), reveal reads 15 and writes 8 (|I| in, k out); plus pure read, pure write, copy.
// Prints TB/s = (read + written bytes) / median kernel time over 7 launches of ~40 GB.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_mix.hip -o tools/ubench_mix && ./tools/ubench_mix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef int64_t v2 __attribute__((ext_vector_type(2)));

template <int NR, int NW>
__global__ __launch_bounds__(256) void mix(const v2* __restrict__ in, v2* __restrict__ out, uint64_t steps,
                                           uint64_t* __restrict__ sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    int64_t acc = 0;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < steps; s += stride) {
        v2 v[NR > 0 ? NR : 1];
#pragma unroll
        for (int u = 0; u < NR; ++u) v[u] = __builtin_nontemporal_load(in + s * NR + u);
        // fold the loads into the stored words so neither side is dead code
        v2 x = {0, 0};
#pragma unroll
        for (int u = 0; u < NR; ++u) x += v[u];
        // the word layout of each step is [step][NR] / [step][NW]: a wave's lanes own adjacent steps, so a
        // wave instruction touches 64 words NR (NW) apart -- as strided as the kernels' row streams, which
        // the L2 merges into full lines within the step range a wave covers
#pragma unroll
        for (int u = 0; u < NW; ++u) {
            v2 y = x;
            y[0] += u;
            __builtin_nontemporal_store(y, out + s * NW + u);
        }
        acc ^= x[0];
    }
    if (acc == 0x123456789abcdefll) sink[0] = acc;
}

// the same mix with coalesced rows: word u of a step lives at u * steps + s (lane-adjacent addresses
// for every instruction), the layout of [row][batch] streams
template <int NR, int NW>
__global__ __launch_bounds__(256) void mix_rows(const v2* __restrict__ in, v2* __restrict__ out, uint64_t steps,
                                                uint64_t* __restrict__ sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    int64_t acc = 0;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < steps; s += stride) {
        v2 v[NR > 0 ? NR : 1];
#pragma unroll
        for (int u = 0; u < NR; ++u) v[u] = __builtin_nontemporal_load(in + (uint64_t)u * steps + s);
        v2 x = {0, 0};
#pragma unroll
        for (int u = 0; u < NR; ++u) x += v[u];
#pragma unroll
        for (int u = 0; u < NW; ++u) {
            v2 y = x;
            y[0] += u;
            __builtin_nontemporal_store(y, out + (uint64_t)u * steps + s);
        }
        acc ^= x[0];
    }
    if (acc == 0x123456789abcdefll) sink[0] = acc;
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                              \
        }                                                                          \
    } while (0)

template <int NR, int NW, bool ROWS>
static int run(const char* name, v2* in, v2* out, uint64_t* sink, int cus) {
    const uint64_t total = 40ull << 30;                       // ~40 GB moved per launch
    const uint64_t steps = total / (16ull * (NR + NW));
    const dim3 grid((unsigned)(cus * 16)), block(256);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ms;
    for (int r = 0; r < 8; ++r) {
        CK(hipEventRecord(a));
        if (ROWS) hipLaunchKernelGGL((mix_rows<NR, NW>), grid, block, 0, 0, in, out, steps, sink);
        else hipLaunchKernelGGL((mix<NR, NW>), grid, block, 0, 0, in, out, steps, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float t = 0;
        CK(hipEventElapsedTime(&t, a, b));
        if (r) ms.push_back(t);                                // first launch: warm-up
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    const double bytes = 16.0 * (NR + NW) * (double)steps;
    printf("%-34s read:write %2d:%-2d  %8.3f ms  %6.3f TB/s  (%.1f GB)\n", name, NR, NW, med,
           bytes / (med * 1e-3) / 1e12, bytes / 1e9);
    return 0;
}

int main() {
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t bytes = 41ull << 30;
    v2 *in = nullptr, *out = nullptr;
    uint64_t* sink = nullptr;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(in, 1, bytes));
    CK(hipMemset(out, 0, bytes));
    int rc = 0;
    rc |= run<1, 0, true>("read only", in, out, sink, cus);
    rc |= run<0, 1, true>("write only", in, out, sink, cus);
    rc |= run<1, 1, true>("copy", in, out, sink, cus);
    rc |= run<15, 26, true>("share-gen mix (rows)", in, out, sink, cus);
    rc |= run<15, 8, true>("reveal mix (rows)", in, out, sink, cus);
    rc |= run<15, 26, false>("share-gen mix (step-major)", in, out, sink, cus);
    rc |= run<15, 8, false>("reveal mix (step-major)", in, out, sink, cus);
    return rc;
}
