// ubench_mall.hip -- can the clerk's decode -> combine keep its int32 slots in the 256 MiB Infinity Cache?
// Memory-only model of codec.hip's slot path (1,000 payloads x 1M field shares: 4.94 GB of payload, 4 B of
// slot per share): kernel A streams a payload slice in and writes the group's slots, kernel B reads the slots
// back (and would combine them).  Variants:
//   whole job   : A over all 1,000 blobs into a 4 GB slot buffer, then B over it (today's two passes)
//   groups of G : A then B per group of G blobs through ONE reused G x 4 MB slot buffer (stays in the MALL if
//                 G x (payload + slots) fits), with default-policy or non-temporal slot stores
// Prints ms per 1,000-blob job and the payload rate.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_mall.hip -o tools/ubench_mall && ./tools/ubench_mall
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

constexpr uint64_t NB = 1000;                 // blobs
constexpr uint64_t PAY = 4937000;             // payload bytes per blob (4.94 B per share)
constexpr uint64_t SLOTB = 4000000;           // slot bytes per blob (1M int32)
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// A: each lane reads 16 B of payload and writes 16 B of slots (payload is 1.23x the slots: the first
// SLOTB/PAY of the lanes write), standing in for decode pass C's read/write mix.
template <bool NT_STORE>
__global__ __launch_bounds__(256) void decode_mem(const v4u* __restrict__ pay, v4u* __restrict__ slots, uint64_t n_pay16,
                                                  uint64_t n_slot16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n_pay16; i += stride) {
        const v4u v = __builtin_nontemporal_load(pay + i);
        const uint64_t j = i * n_slot16 / n_pay16;
        if (NT_STORE) __builtin_nontemporal_store(v + 1u, slots + j);
        else slots[j] = v + 1u;
    }
}

// B: read the slots back (16 B per lane), fold into a per-lane sum so the loads stay live.
__global__ __launch_bounds__(256) void combine_mem(const v4u* __restrict__ slots, uint64_t n16, uint32_t* __restrict__ sink) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        const v4u v = slots[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            fprintf(stderr, "%s failed at line %d: %s\n", #x, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

template <class F>
static float time_ms(F job, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    job();
    CHECK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a, 0));
        job();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float t;
        CHECK(hipEventElapsedTime(&t, a, b));
        v.push_back(t);
    }
    std::sort(v.begin(), v.end());
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return v[v.size() / 2];
}

int main() {
    v4u *pay, *slots;
    uint32_t* sink;
    CHECK(hipMalloc(&pay, NB * PAY + 4096));
    CHECK(hipMalloc(&slots, NB * SLOTB + 4096));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(pay, 3, NB * PAY));
    const unsigned grid = 256 * 16;
    auto job = [&](uint64_t G, bool nt) {
        for (uint64_t g0 = 0; g0 < NB; g0 += G) {
            const uint64_t n = std::min(G, NB - g0);
            const v4u* p = pay + g0 * PAY / 16;
            v4u* s = G >= NB ? slots : slots;      // groups reuse the buffer's first n blobs
            if (nt) hipLaunchKernelGGL((decode_mem<true>), dim3(grid), dim3(256), 0, 0, p, s, n * PAY / 16, n * SLOTB / 16);
            else hipLaunchKernelGGL((decode_mem<false>), dim3(grid), dim3(256), 0, 0, p, s, n * PAY / 16, n * SLOTB / 16);
            hipLaunchKernelGGL(combine_mem, dim3(grid), dim3(256), 0, 0, s, n * SLOTB / 16, sink);
        }
    };
    printf("1,000 blobs: %.2f GB payload, %.2f GB slots\n", NB * PAY / 1e9, NB * SLOTB / 1e9);
    for (bool nt : {true, false}) {
        for (uint64_t G : {1000ull, 100ull, 40ull, 20ull, 10ull, 5ull}) {
            const float ms = time_ms([&] { job(G, nt); }, 5);
            printf("%-10s stores, groups of %4llu blobs (%3llu launches): %7.3f ms  payload %5.2f TB/s\n",
                   nt ? "nt" : "default", (unsigned long long)G, (unsigned long long)(2 * ((NB + G - 1) / G)), ms,
                   NB * PAY / (ms * 1e-3) / 1e12);
        }
    }
    const float rd = time_ms([&] { hipLaunchKernelGGL(combine_mem, dim3(grid), dim3(256), 0, 0, pay, NB * PAY / 16, sink); }, 5);
    printf("payload read alone: %.3f ms (%.2f TB/s)\n", rd, NB * PAY / (rd * 1e-3) / 1e12);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    return 0;
}
