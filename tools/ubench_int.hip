// ubench_int.hip -- issue rates of the integer VALU ops the sharing kernels are built from (gfx950).
// Each lane runs 8 independent dependency chains of one op; we report lane-ops/s across the chip.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_int.hip -o tools/ubench_int && ./tools/ubench_int
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHAINS 8
#define ITERS 4096

template <int OP>
__global__ __launch_bounds__(256) void ubench(uint32_t seed, uint64_t* sink) {
    uint32_t a[CHAINS];
    uint64_t w[CHAINS];
    const uint32_t b = seed * 2654435761u + threadIdx.x;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) { a[c] = seed + c * 977 + threadIdx.x; w[c] = a[c]; }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if constexpr (OP == 0) a[c] = a[c] + b;                                   // v_add_u32
            if constexpr (OP == 1) a[c] = a[c] * b;                                   // v_mul_lo_u32
            if constexpr (OP == 2) a[c] = __umulhi(a[c], b) ^ c;                      // v_mul_hi_u32 (+xor)
            if constexpr (OP == 3) w[c] = (uint64_t)(uint32_t)w[c] * b + w[c];        // v_mad_u64_u32
            if constexpr (OP == 4) w[c] = (uint64_t)((int64_t)(int32_t)w[c] * (int32_t)b + (int64_t)w[c]);  // v_mad_i64_i32
            if constexpr (OP == 5) a[c] = __builtin_amdgcn_alignbit(a[c], a[c], 7) ^ b;   // rotate + xor
            if constexpr (OP == 6) w[c] = w[c] + (uint64_t)b;                        // 64-bit add (2 ops)
            if constexpr (OP == 7) { double d = (double)a[c]; a[c] = (uint32_t)(d * 1.0000001 + 3.0); } // f64 fma + cvts
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += a[c] + w[c];
    if (s == 0x12345) sink[threadIdx.x] = s;
}

template <int OP>
double run(const char* name, uint64_t* sink) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 256 * 8;
    hipLaunchKernelGGL(ubench<OP>, dim3(blocks), dim3(256), 0, 0, 1u, sink);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ubench<OP>, dim3(blocks), dim3(256), 0, 0, (uint32_t)r + 2, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = 5.0 * blocks * 256.0 * ITERS * CHAINS;
    const double rate = ops / (ms * 1e-3);
    printf("%-28s %8.2f T lane-ops/s  (%.3f ms/launch)\n", name, rate / 1e12, ms / 5);
    return rate;
}

int main() {
    uint64_t* sink;
    hipMalloc(&sink, 4096);
    run<0>("v_add_u32", sink);
    run<1>("v_mul_lo_u32", sink);
    run<2>("v_mul_hi_u32 + xor", sink);
    run<3>("v_mad_u64_u32", sink);
    run<4>("v_mad_i64_i32", sink);
    run<5>("v_alignbit + xor", sink);
    run<6>("u64 add (2 ops)", sink);
    run<7>("f64 cvt+fma+cvt", sink);
    hipFree(sink);
    return 0;
}
