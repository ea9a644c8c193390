// ubench_bank.hip -- does a VALU instruction whose two VGPR sources sit in the same register bank (index mod 4)
// issue slower on gfx950?  ChaCha's quarter-round as the test pattern: four independent chains per wave, each
// a += b; b ^= a; b = rotl(b, r) on a (a, b) register pair, written in inline asm with fixed registers so the
// pairing is ours, not the register allocator's:
//   same bank : (v40, v44) (v41, v45) (v42, v46) (v43, v47)   -- every add / xor reads one bank twice
//   diff bank : (v40, v45) (v41, v46) (v42, v47) (v43, v44)
// plus the add / xor pairs alone (no rotate), and the rotate as three VOP2 ops (all or half of them).  Prints
// T lane-ops/s per variant, counting a QR step as its 12 ChaCha operations whatever the rotate's encoding.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_bank.hip -o tools/ubench_bank && ./tools/ubench_bank
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                                                 \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s failed at line %d: %s\n", #x, __LINE__, hipGetErrorString(e_));  \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

#define QR4(A0, B0, A1, B1, A2, B2, A3, B3, R)                                 \
    "v_add_u32 " A0 ", " A0 ", " B0 "\n v_add_u32 " A1 ", " A1 ", " B1 "\n"    \
    "v_add_u32 " A2 ", " A2 ", " B2 "\n v_add_u32 " A3 ", " A3 ", " B3 "\n"    \
    "v_xor_b32 " B0 ", " B0 ", " A0 "\n v_xor_b32 " B1 ", " B1 ", " A1 "\n"    \
    "v_xor_b32 " B2 ", " B2 ", " A2 "\n v_xor_b32 " B3 ", " B3 ", " A3 "\n"    \
    "v_alignbit_b32 " B0 ", " B0 ", " B0 ", " R "\n v_alignbit_b32 " B1 ", " B1 ", " B1 ", " R "\n" \
    "v_alignbit_b32 " B2 ", " B2 ", " B2 ", " R "\n v_alignbit_b32 " B3 ", " B3 ", " B3 ", " R "\n"
#define AX4(A0, B0, A1, B1, A2, B2, A3, B3)                                    \
    "v_add_u32 " A0 ", " A0 ", " B0 "\n v_add_u32 " A1 ", " A1 ", " B1 "\n"    \
    "v_add_u32 " A2 ", " A2 ", " B2 "\n v_add_u32 " A3 ", " A3 ", " B3 "\n"    \
    "v_xor_b32 " B0 ", " B0 ", " A0 "\n v_xor_b32 " B1 ", " B1 ", " A1 "\n"    \
    "v_xor_b32 " B2 ", " B2 ", " A2 "\n v_xor_b32 " B3 ", " B3 ", " A3 "\n"

// the rotate as three full-rate VOP2 ops (v58..v61 scratch): b = (b << r) | (b >> (32 - r))
#define ROT3(B, T, R, RR) "v_lshlrev_b32 " T ", " R ", " B "\n v_lshrrev_b32 " B ", " RR ", " B "\n v_or_b32 " B ", " B ", " T "\n"
#define QS4(A0, B0, A1, B1, A2, B2, A3, B3)                                    \
    "v_add_u32 " A0 ", " A0 ", " B0 "\n v_add_u32 " A1 ", " A1 ", " B1 "\n"    \
    "v_add_u32 " A2 ", " A2 ", " B2 "\n v_add_u32 " A3 ", " A3 ", " B3 "\n"    \
    "v_xor_b32 " B0 ", " B0 ", " A0 "\n v_xor_b32 " B1 ", " B1 ", " A1 "\n"    \
    "v_xor_b32 " B2 ", " B2 ", " A2 "\n v_xor_b32 " B3 ", " B3 ", " A3 "\n"    \
    ROT3(B0, "v58", "16", "16") ROT3(B1, "v59", "16", "16") ROT3(B2, "v60", "16", "16") ROT3(B3, "v61", "16", "16")
// half the rotates as alignbit, half as the VOP2 triple
#define QH4(A0, B0, A1, B1, A2, B2, A3, B3)                                    \
    "v_add_u32 " A0 ", " A0 ", " B0 "\n v_add_u32 " A1 ", " A1 ", " B1 "\n"    \
    "v_add_u32 " A2 ", " A2 ", " B2 "\n v_add_u32 " A3 ", " A3 ", " B3 "\n"    \
    "v_xor_b32 " B0 ", " B0 ", " A0 "\n v_xor_b32 " B1 ", " B1 ", " A1 "\n"    \
    "v_xor_b32 " B2 ", " B2 ", " A2 "\n v_xor_b32 " B3 ", " B3 ", " A3 "\n"    \
    "v_alignbit_b32 " B0 ", " B0 ", " B0 ", 16\n" ROT3(B1, "v59", "16", "16")     \
    "v_alignbit_b32 " B2 ", " B2 ", " B2 ", 16\n" ROT3(B3, "v61", "16", "16")
#define QS4X(...) QS4(__VA_ARGS__)
#define QH4X(...) QH4(__VA_ARGS__)
#define QR4X(...) QR4(__VA_ARGS__)
#define AX4X(...) AX4(__VA_ARGS__)
#define SAME "v40", "v44", "v41", "v45", "v42", "v46", "v43", "v47"
#define DIFF "v40", "v45", "v41", "v46", "v42", "v47", "v43", "v44"
#define X4(M) M M M M

// 12 (QR) or 8 (AX) instructions per macro; each body below is 16 macros
template <int MODE>
__global__ __launch_bounds__(256) void bank_kernel(int iters, uint32_t* __restrict__ sink) {
    uint32_t seed = threadIdx.x * 2654435761u + blockIdx.x;
    uint32_t out;
    asm volatile(
        "v_mov_b32 v40, %1\n v_add_u32 v41, 1, %1\n v_add_u32 v42, 2, %1\n v_add_u32 v43, 3, %1\n"
        "v_add_u32 v44, 4, %1\n v_add_u32 v45, 5, %1\n v_add_u32 v46, 6, %1\n v_add_u32 v47, 7, %1\n"
        "v_mov_b32 %0, v40\n"
        : "=v"(out) : "v"(seed) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) asm volatile(X4(X4(QR4X(SAME, "16"))) ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (MODE == 1) asm volatile(X4(X4(QR4X(DIFF, "16"))) ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (MODE == 2) asm volatile(X4(X4(AX4X(SAME))) ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (MODE == 3) asm volatile(X4(X4(AX4X(DIFF))) ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (MODE == 4) asm volatile(X4(X4(QS4X(DIFF))) ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v58", "v59", "v60", "v61");
        if constexpr (MODE == 5) asm volatile(X4(X4(QH4X(DIFF))) ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v58", "v59", "v60", "v61");
    }
    asm volatile("v_xor_b32 %0, %0, v40\n v_xor_b32 %0, %0, v45" : "+v"(out) :: "v40", "v45");
    if (out == 0x12345678u) sink[0] = out;
}

template <int MODE>
static void run(const char* name, int waves_per_simd, uint32_t* sink) {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * waves_per_simd;          // 256-lane blocks: 4 waves = one per SIMD
    const int iters = 2000;
    // lane-ops counted as the QR's own 12 (add, xor, rotate x 4 chains), whatever the rotate costs
    const double per_macro = (MODE < 2 || MODE >= 4) ? 12 : 8;
    const double insts = per_macro * 16 * iters;      // per lane
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(bank_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, 10, sink);
    CHECK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(bank_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, iters, sink);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    const double lane_ops = insts * blocks * 256.0;
    printf("%-34s %d waves/SIMD  %8.3f ms  %6.2f T lane-ops/s\n", name, waves_per_simd, v[2],
           lane_ops / (v[2] * 1e-3) / 1e12);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

int main() {
    uint32_t* sink;
    CHECK(hipMalloc(&sink, 64));
    for (int w : {4, 6, 8}) {
        run<0>("QR chains, same-bank pairs", w, sink);
        run<1>("QR chains, different-bank pairs", w, sink);
        run<2>("add/xor chains, same-bank pairs", w, sink);
        run<3>("add/xor chains, different-bank pairs", w, sink);
        run<4>("QR chains, rotate = shl+shr+or", w, sink);
        run<5>("QR chains, half alignbit half shl+shr+or", w, sink);
    }
    CHECK(hipDeviceSynchronize());
    return 0;
}
