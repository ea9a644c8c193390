// ubench_int.hip -- issue rates of the integer VALU ops the sharing kernels are built from (gfx950).
// Inline asm keeps exactly one instruction per statement; 8 independent chains per lane, full grid.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_int.hip -o tools/ubench_int && ./tools/ubench_int
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void ubench(uint32_t seed, uint64_t* sink) {
    uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3, w4 = a4, w5 = a5, w6 = a6, w7 = a7;
    uint32_t b = seed * 2654435761u + threadIdx.x;
    for (int it = 0; it < ITERS; ++it) {
#define STEP(i)                                                                                         \
        if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));             \
        if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));          \
        if constexpr (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));          \
        if constexpr (OP == 3) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(w##i) : "v"(b), "v"(b) : "s40", "s41"); \
        if constexpr (OP == 4) asm volatile("v_mad_i64_i32 %0, s[40:41], %1, %2, %0" : "+v"(w##i) : "v"(b), "v"(b) : "s40", "s41"); \
        if constexpr (OP == 5) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a##i));                \
        if constexpr (OP == 6) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));             \
        if constexpr (OP == 7) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(b) : "vcc"); \
        if constexpr (OP == 8) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(w##i));              \
        if constexpr (OP == 9) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##i) : "v"(b));            \
        if constexpr (OP == 10) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(a##i) : "v"(b));      \
        if constexpr (OP == 11) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(a##i));             \
        if constexpr (OP == 12) asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a##i) : "v"(b)); \
        if constexpr (OP == 13) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));            \
        if constexpr (OP == 14) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a##i) : "v"(b));            \
        if constexpr (OP == 15) asm volatile("v_ashrrev_i32 %0, 3, %0" : "+v"(a##i));                   \
        if constexpr (OP == 16) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));            \
        if constexpr (OP == 17) asm volatile("v_min3_u32 %0, %0, %1, %0" : "+v"(a##i) : "v"(b));       \
        if constexpr (OP == 18) asm volatile("v_med3_u32 %0, %0, %1, %0" : "+v"(a##i) : "v"(b));       \
        if constexpr (OP == 19) asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(a##i)); \
        if constexpr (OP == 20) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x6c" : "+v"(a##i) : "v"(b)); \
        if constexpr (OP == 21) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a##i) : "v"(b));       \
        if constexpr (OP == 22) asm volatile("v_sub_i32 %0, %0, %1 clamp" : "+v"(a##i) : "v"(b));      \
        if constexpr (OP == 23) asm volatile("v_bfi_b32 %0, %0, %1, %0" : "+v"(a##i) : "v"(b));        \
        if constexpr (OP == 24) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a##i) : "v"(b) : "s40", "s41"); \
        if constexpr (OP == 25) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a##i) : "v"(b));     \
        if constexpr (OP == 26) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a##i) : "v"(b));        \
        if constexpr (OP == 27) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a##i) : "v"(b) : "vcc"); \
        if constexpr (OP == 28) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a##i) : "v"(b));            \
        if constexpr (OP == 29) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a##i)); \
        if constexpr (OP == 30) { uint32_t t_;                                                          \
            asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n\t" \
                         "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" \
                         : "=&v"(t_) : "v"(a##i), "v"(b)); a##i = t_; }
        REP8(STEP)
    }
    uint64_t s = (uint64_t)a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + w0 + w1 + w2 + w3 + w4 + w5 + w6 + w7;
    if (s == 0x12345) sink[threadIdx.x] = s;
}

// Whole modular steps ("exact reveal: the per-step sequence"): 8 independent chains per lane of
// one Newton divided-difference step (s_i - s_{i-1}) % p * inv % p in the sign-bit form -- the residue through
// the quotient sequence under test, the sign through one v_bitop3.  One asm statement per instruction, so the
// compiler adds nothing; the 64-bit halves are sub-registers (no moves).
//   SEQ 0: Montgomery, as packed_reveal_exact_kernel compiles it: sub, add p, v_mad_u64_u32 (x inv_m),
//          v_mul_lo_u32 (x p'), v_mad_u64_u32 (+ m p), subrev p, min, bitop3           (8 instructions)
//   SEQ 1: Shoup with a precomputed quotient word inv' = floor(inv 2^32 / p): sub, add p, v_mul_hi_u32 (q),
//          v_mul_lo_u32 (x inv), v_mul_lo_u32 (q p), sub, subrev p, min, bitop3        (9 instructions)
//   SEQ 2: Shoup with the low product folded into one v_mad_u64_u32 (q (2^32 - p) + x inv mod 2^32), whose
//          64-bit addend needs the zero high word (v_mov): sub, add p, mul_hi, mul_lo, mov, mad, subrev, min,
//          bitop3                                                                        (9 instructions)
template <int SEQ>
__global__ __launch_bounds__(256) void ubench_seq(uint32_t seed, uint32_t P, uint32_t PINV, uint32_t W, uint32_t WQ,
                                                  uint64_t* sink) {
    uint32_t a0 = (seed + threadIdx.x) % P, a1 = (a0 * 3) % P, a2 = (a0 * 5) % P, a3 = (a0 * 7) % P,
             a4 = (a0 * 11) % P, a5 = (a0 * 13) % P, a6 = (a0 * 17) % P, a7 = (a0 * 19) % P;
    uint32_t n0 = a0, n1 = a1, n2 = a2, n3 = a3, n4 = a4, n5 = a5, n6 = a6, n7 = a7;
    const uint32_t b = (seed * 2654435761u + threadIdx.x) % P, NEGP = 0u - P;
    for (int it = 0; it < ITERS / 8; ++it) {
#define SEQSTEP(i)                                                                                              \
        {                                                                                                       \
            uint32_t d_, x_, m_, r_, rp_, q_, lo_, t_;                                                          \
            uint64_t T_, U_;                                                                                    \
            asm volatile("v_sub_u32 %0, %1, %2" : "=v"(d_) : "v"(a##i), "v"(b));                                \
            asm volatile("v_add_u32 %0, %1, %2" : "=v"(x_) : "s"(P), "v"(d_));                                  \
            if constexpr (SEQ == 0) {                                                                           \
                asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, 0" : "=v"(T_) : "s"(W), "v"(x_) : "s40", "s41"); \
                asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(m_) : "s"(PINV), "v"((uint32_t)T_));             \
                asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %3" : "=v"(U_) : "v"(m_), "s"(P), "v"(T_)     \
                             : "s40", "s41");                                                                   \
                r_ = (uint32_t)(U_ >> 32);                                                                      \
            } else if constexpr (SEQ == 1) {                                                                    \
                asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(q_) : "s"(WQ), "v"(x_));                          \
                asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(lo_) : "s"(W), "v"(x_));                          \
                asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(t_) : "s"(P), "v"(q_));                           \
                asm volatile("v_sub_u32 %0, %1, %2" : "=v"(r_) : "v"(lo_), "v"(t_));                            \
            } else {                                                                                            \
                asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(q_) : "s"(WQ), "v"(x_));                          \
                asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(lo_) : "s"(W), "v"(x_));                          \
                asm volatile("v_mov_b32 %0, 0" : "=v"(t_));                                                     \
                T_ = ((uint64_t)t_ << 32) | lo_;                                                                \
                asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %3" : "=v"(U_) : "v"(q_), "s"(NEGP), "v"(T_)  \
                             : "s40", "s41");                                                                   \
                r_ = (uint32_t)U_;                                                                              \
            }                                                                                                   \
            asm volatile("v_subrev_u32 %0, %1, %2" : "=v"(rp_) : "s"(P), "v"(r_));                              \
            asm volatile("v_min_u32 %0, %1, %2" : "=v"(a##i) : "v"(r_), "v"(rp_));                              \
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xb2" : "+v"(n##i) : "v"(b), "v"(d_));             \
        }
        REP8(SEQSTEP)
    }
    uint64_t s = (uint64_t)a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + n0 + n1 + n2 + n3 + n4 + n5 + n6 + n7;
    if (s == 0x12345) sink[threadIdx.x] = s;
}

template <int SEQ>
void run_seq(const char* name, uint64_t* sink, int insts_per_step) {
    const uint32_t P = 2147482801u, W = 1234567u;                  // configs[2]'s prime, an arbitrary inverse
    uint32_t pinv = 1;                                             // -p^-1 mod 2^32 (Newton)
    for (int i = 0; i < 5; ++i) pinv *= 2 - P * pinv;
    const uint32_t PINV = 0u - pinv;
    const uint32_t WM = (uint32_t)(((uint64_t)W << 32) % P);      // Montgomery form of W
    const uint32_t WQ = (uint32_t)(((uint64_t)W << 32) / P);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int blocks = 256 * 8;
    hipLaunchKernelGGL(ubench_seq<SEQ>, dim3(blocks), dim3(256), 0, 0, 1u, P, PINV, SEQ == 0 ? WM : W, WQ, sink);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(ubench_seq<SEQ>, dim3(blocks), dim3(256), 0, 0, (uint32_t)r + 2, P, PINV, SEQ == 0 ? WM : W,
                           WQ, sink);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double steps = 5.0 * blocks * 256.0 * (ITERS / 8) * 8;
    printf("%-34s %7.2f G steps/s  %7.2f T lane-instr/s  (%.3f ms/launch)\n", name, steps / (ms * 1e-3) / 1e9,
           steps * insts_per_step / (ms * 1e-3) / 1e12, ms / 5);
}

template <int OP>
void run(const char* name, uint64_t* sink, int insts_per_step) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int blocks = 256 * 8;
    hipLaunchKernelGGL(ubench<OP>, dim3(blocks), dim3(256), 0, 0, 1u, sink);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ubench<OP>, dim3(blocks), dim3(256), 0, 0, (uint32_t)r + 2, sink);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double insts = 5.0 * blocks * 256.0 * ITERS * 8 * insts_per_step;
    printf("%-22s %7.2f T lane-instr/s  (%.3f ms/launch)\n", name, insts / (ms * 1e-3) / 1e12, ms / 5);
}

int main() {
    uint64_t* sink;
    (void)hipMalloc(&sink, 4096);
    run<0>("v_add_u32", sink, 1);
    run<9>("v_xor_b32", sink, 1);
    run<6>("v_min_u32", sink, 1);
    run<5>("v_alignbit_b32", sink, 1);
    run<7>("v_cmp + v_cndmask", sink, 2);
    run<1>("v_mul_lo_u32", sink, 1);
    run<2>("v_mul_hi_u32", sink, 1);
    run<3>("v_mad_u64_u32", sink, 1);
    run<4>("v_mad_i64_i32", sink, 1);
    run<8>("v_lshl_add_u64", sink, 1);
    run<10>("v_perm_b32", sink, 1);
    run<11>("v_alignbit_b32 (16)", sink, 1);
    run<12>("v_xad_u32", sink, 1);
    run<13>("v_sub_u32", sink, 1);
    run<14>("v_and_b32", sink, 1);
    run<15>("v_ashrrev_i32", sink, 1);
    run<29>("v_lshrrev_b32", sink, 1);
    run<16>("v_max_u32", sink, 1);
    run<28>("v_min_i32", sink, 1);
    run<17>("v_min3_u32", sink, 1);
    run<18>("v_med3_u32", sink, 1);
    run<19>("v_pk_add_u16 (swap)", sink, 1);
    run<20>("v_bitop3_b32", sink, 1);
    run<21>("v_add3_u32", sink, 1);
    run<22>("v_sub_i32 clamp", sink, 1);
    run<23>("v_bfi_b32", sink, 1);
    run<24>("v_cndmask_b32 (sgpr)", sink, 1);
    run<25>("v_lshl_or_b32", sink, 1);
    run<26>("v_mul_u32_u24", sink, 1);
    run<27>("v_add_co + v_addc_co", sink, 2);
    run<30>("v_xor_b32_sdwa x2 (rot16)", sink, 2);
    run<0>("v_add_u32 (again)", sink, 1);
    run_seq<0>("newton step, Montgomery (shipped)", sink, 8);
    run_seq<1>("newton step, Shoup (mul_lo + sub)", sink, 9);
    run_seq<2>("newton step, Shoup (mad_u64)", sink, 9);
    run_seq<0>("newton step, Montgomery (again)", sink, 8);
    (void)hipFree(sink);
    return 0;
}
