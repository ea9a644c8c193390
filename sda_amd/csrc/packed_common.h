#pragma once
// packed_common.h -- shared by packed_gen.hip / packed_reveal.hip: north-star kernel (2): packed-Shamir share generation and reveal.
//
// Reference call sites: client/src/crypto/sharing/packed_shamir.rs:40-43 (share) and :73-77
// (reconstruct), batched by client/src/crypto/sharing/batched.rs:19-53 / :69-97.  The
// arithmetic lives in threshold-secret-sharing 0.2 (absent from the reference tree):
//   share:       values = [0, secrets(k), randomness(t)]  (length L = k+t+1, a power of 2)
//                coeffs = fft2_inverse(values, omega_secrets)   recursive radix-2, `%` per op
//                points = fft3(coeffs ++ zeros, omega_shares)    recursive radix-3 over n+1
//                shares = points[1..=n]
//   reconstruct: Newton divided differences through (1,0) and (omega_shares^(i+1), share_i),
//                evaluated at omega_secrets^e, e = 1..k.
// Every intermediate is an i64 in (-p, p) whose SIGN depends on the exact operation order
// (Rust's truncated `%`).  The kernels reproduce them bit for bit: for each `(expr) % p` they
// compute (i) the canonical residue with 32-bit Montgomery products (R = 2^32, no 64-bit
// division) and (ii) the sign of the exact i64 expr with one 32x32->64 multiply-add, then
// recombine (trunc_from).  No MFMA: this is not a dense contraction (north star).
//
// One lane = one batch.  The in-place DIT on bit/digit-reversed registers performs exactly the
// butterflies of tss' recursion (same operands, same twiddles, same `%` points).  Batches whose
// inputs fall outside (-p, p) (raw i64 secrets / shares) take a generic exact path that mirrors
// the recursion with wrapping i64 arithmetic.
//
// Reveal comes in two modes: EXACT (Newton, tss' signed representatives; VALU-bound) and
// CANONICAL (Lagrange weights for the clerk-index set, residues in [0, p); HBM-bound), equal
// mod p and equal after RecipientOutput::positive (receive.rs:14-20).
#include <string.h>

#include <vector>

#include "kernels.h"

namespace sda {
namespace packed {

// ------------------------------------------------------------------------------------------
// host-side exact helpers (tss numtheory semantics: truncated `%`)
// ------------------------------------------------------------------------------------------
inline int64_t h_rem(int64_t a, int64_t p) { return a % p; }
inline int64_t h_powmod(int64_t x, uint32_t e, int64_t p) {      // numtheory::mod_pow
    int64_t acc = 1;
    while (e > 0) {
        if (e & 1u) acc = h_rem((int64_t)((uint64_t)acc * (uint64_t)x), p);
        x = h_rem((int64_t)((uint64_t)x * (uint64_t)x), p);
        e >>= 1;
    }
    return acc;
}
inline void h_egcd(int64_t a, int64_t b, int64_t* s, int64_t* t) {     // numtheory::gcd
    if (b == 0) { *s = 1; *t = 0; return; }
    int64_t n = a / b, c = a % b, s1, t1;
    h_egcd(b, c, &s1, &t1);
    *s = t1; *t = s1 - t1 * n;
}
inline int64_t h_modinv(int64_t k, int64_t p) {                 // numtheory::mod_inverse
    int64_t k2 = k % p, s, t, r;
    if (k2 < 0) { h_egcd(p, -k2, &s, &t); r = -t; } else { h_egcd(p, k2, &s, &t); r = t; }
    return (p + r) % p;
}
inline uint32_t to_mont(int64_t x, int64_t p) {            // canonical x -> x R mod p
    int64_t c = x % p; if (c < 0) c += p;
    return (uint32_t)((((unsigned __int128)c) << 32) % (uint64_t)p);
}

// ------------------------------------------------------------------------------------------
// generation tables (kernel argument, uniform => scalar loads)
// ------------------------------------------------------------------------------------------
struct GenTables {
    MontP M;
    uint32_t linv, linv_m;          // L^{-1} mod p (canonical, Montgomery)
    uint32_t tw2[64], tw2_m[64];    // radix-2 level len: entries [len/2 - 1, len - 1)
    uint32_t tw3[120], tw3_m[120];  // radix-3 level len: entries [(len-3)/2, (len-3)/2 + len)
    uint32_t sq3[120], sq3_m[120];  // x^2 % p per radix-3 entry
    // Sign-bit share-gen (packed_gen.hip, SIGNBIT): (u + w c) % p has the sign of c whenever |w c| >= p,
    // i.e. |c| >= ceil(p / w); big2 = the largest such bound over the non-unit radix-2 twiddles, big3 over
    // the radix-3 twiddles of the first radix-3 level (its groups are b + x c: d is zero padding).
    uint32_t big2, big3;
};

inline GenTables make_gen_tables(uint32_t L, uint32_t N3, int64_t p, int64_t ws, int64_t wn) {
    GenTables T;
    memset(&T, 0, sizeof(T));
    T.M = make_mont((uint32_t)p);
    // fft2_inverse: fft2 over omega^-1; recursion squares omega at each level (mod_pow(ω, 2))
    const int64_t winv = h_modinv(ws, p);
    T.linv = (uint32_t)h_modinv((int64_t)L, p);
    T.linv_m = to_mont(T.linv, p);
    {
        int64_t om = winv;                 // omega for the top level (len = L)
        std::vector<int64_t> per_level;    // omega per level, top first
        for (uint32_t len = L; len >= 2; len /= 2) { per_level.push_back(om); om = h_powmod(om, 2, p); }
        int lvl = (int)per_level.size() - 1;
        for (uint32_t len = 2; len <= L; len *= 2, --lvl) {
            for (uint32_t i = 0; i < len / 2; ++i) {
                const int64_t w = h_powmod(per_level[lvl], i, p);
                T.tw2[len / 2 - 1 + i] = (uint32_t)w;
                T.tw2_m[len / 2 - 1 + i] = to_mont(w, p);
            }
        }
    }
    T.big2 = 1;
    for (uint32_t e = 1; e < L - 1; ++e)
        if (T.tw2[e] > 1) { const uint64_t b = ((uint64_t)p + T.tw2[e] - 1) / T.tw2[e]; if (b > T.big2) T.big2 = (uint32_t)b; }
    {
        int64_t om = wn;
        std::vector<int64_t> per_level;
        for (uint32_t len = N3; len >= 3; len /= 3) { per_level.push_back(om); om = h_powmod(om, 3, p); }
        int lvl = (int)per_level.size() - 1;
        for (uint32_t len = 3; len <= N3; len *= 3, --lvl) {
            for (uint32_t j = 0; j < len; ++j) {
                const int64_t x = h_powmod(per_level[lvl], j, p);
                const int64_t x2 = h_rem(x * x, p);
                const uint32_t o = (len - 3) / 2 + j;
                T.tw3[o] = (uint32_t)x; T.tw3_m[o] = to_mont(x, p);
                T.sq3[o] = (uint32_t)x2; T.sq3_m[o] = to_mont(x2, p);
            }
        }
    }
    T.big3 = 1;
    for (uint32_t j = 1; j < 3 && j < N3; ++j) {          // first radix-3 level: entries 1, 2 (len 3)
        const uint64_t b = ((uint64_t)p + T.tw3[j] - 1) / T.tw3[j];
        if (b > T.big3) T.big3 = (uint32_t)b;
    }
    return T;
}


// Rust `v % p` from the canonical residue c and the sign word sw of the exact dividend v.
//   exact (LAZY = false): trunc_rep, 5 VALU ops incl. the c == 0 case (v < 0, v = 0 mod p -> 0);
//   LAZY: c - (p & sign), 3 ops, which gives -p instead of 0 exactly when v < 0 and v = 0 mod p
//   (a nonzero multiple of p: probability ~1/p per value; v == 0 itself is exact).  -p is the only
//   value outside (-p, p), so a running signed min over the outputs finds it (one v_min3 per two
//   values, as opaque asm so the compiler cannot reassociate the chain and stretch live ranges);
//   the batch is then recomputed by the generic exact path (share-gen: logged for the fix-up
//   kernel; reveal: the lane's generic branch).  LAZY is launched only for p >= kLazyTruncMinP.
#ifndef SDA_TRAP_ASM
#define SDA_TRAP_ASM 1
#endif
template <bool LAZY>
struct Trunc {
    int32_t smin = 0x7FFFFFFF;
    int32_t pend = 0;             // note1: values are folded into smin two at a time (one v_min3)
    bool has_pend = false;        // (constant at every point of the unrolled code)
    __device__ __forceinline__ int32_t operator()(uint32_t c, uint32_t sw, uint32_t p) {
        if constexpr (LAZY) {
            return (int32_t)(c - (p & (uint32_t)((int32_t)sw >> 31)));
        }
        else return trunc_rep(c, sw, p);
    }
    __device__ __forceinline__ void note1(int32_t a) {
        if constexpr (LAZY) {
            if (has_pend) {
                note2(pend, a);
                has_pend = false;
            } else {
                pend = a;
                has_pend = true;
            }
        }
    }
    __device__ __forceinline__ void note2(int32_t a, int32_t b) {
        if constexpr (LAZY) {
#if SDA_TRAP_ASM
            asm("v_min3_i32 %0, %0, %1, %2" : "+v"(smin) : "v"(a), "v"(b));
#else
            smin = min(smin, min(a, b));
#endif
        }
    }
    static constexpr bool lazy = LAZY;
    __device__ __forceinline__ bool bad(uint32_t p) {
        if constexpr (LAZY) {
            if (has_pend) note2(pend, pend);
            has_pend = false;
            return smin == -(int32_t)p;
        }
        return false;
    }
};

// Sign-bit logic for the reveal's lazy path: only bit 31 of each operand matters (a sign).
//   maj3(a, b, c)    = MAJ(a, b, c)      one v_bitop3_b32
//   maj3_nb(a, b, c) = MAJ(a, ~b, c)
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
__device__ __forceinline__ uint32_t maj3_nb(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xB2);
}

// Running unsigned min of canonical residues, two per v_min3_u32 (opaque asm, as Trunc): the
// reveal's sign-bit path is exact unless some residue it produced is 0 (probability ~1/p each).
struct ZeroTrap {
    uint32_t zmin = 0xFFFFFFFFu;
    uint32_t pend = 0;
    bool has_pend = false;
    __device__ __forceinline__ void note2(uint32_t a, uint32_t b) {
        asm("v_min3_u32 %0, %0, %1, %2" : "+v"(zmin) : "v"(a), "v"(b));
    }
    __device__ __forceinline__ void note1(uint32_t a) {
        if (has_pend) {
            note2(pend, a);
            has_pend = false;
        } else {
            pend = a;
            has_pend = true;
        }
    }
    __device__ __forceinline__ void flush() {     // call where a runtime branch joins: keeps has_pend constant
        if (has_pend) note2(pend, pend);
        has_pend = false;
    }
    __device__ __forceinline__ bool bad() {
        flush();
        return zmin == 0;
    }
};

// Montgomery product with a uniform (SGPR) multiplier as a fixed instruction sequence:
// v_mad_u64_u32 (T = a' x [+ acc]), v_mul_lo_u32 (u = T pinv), v_mad_u64_u32 (T + u p) -> high word
// in [0, 2p).  (Left to isel, the exact kernel's lazy variant grew a dead mov + mad-by-0 after
// every reduction.)
__device__ __forceinline__ uint64_t mad_su(uint32_t s, uint32_t v, uint64_t acc) {
    uint64_t r, cy;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cy) : "s"(s), "v"(v), "v"(acc));
    return r;
}
__device__ __forceinline__ uint64_t mul_su(uint32_t s, uint32_t v) {
    uint64_t r, cy;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cy) : "s"(s), "v"(v));
    return r;
}
__device__ __forceinline__ uint32_t redc_su(uint64_t T, const MontP& M) {
    const uint32_t u = (uint32_t)T * M.pinv;
    return (uint32_t)(mad_su(M.p, u, T) >> 32);
}
// a' x mod p in [0, p) (a' uniform, Montgomery form); ASM selects the fixed sequence above
// (used by the lazy kernel; the exact-trunc kernel keeps the compiler's, which allocates better).
template <bool ASM>
__device__ __forceinline__ uint32_t montu(uint32_t a_m, uint32_t x, const MontP& M) {
    if constexpr (ASM) return red1(redc_su(mul_su(a_m, x), M), M.p);
    else return red1(redc_lazy((uint64_t)a_m * x, M), M.p);
}
// (a' x + b' y) mod p in [0, p)   (a' x + b' y < 2 p^2 < p R)
template <bool ASM>
__device__ __forceinline__ uint32_t montu2(uint32_t a_m, uint32_t x, uint32_t b_m, uint32_t y, const MontP& M) {
    if constexpr (ASM) return red1(redc_su(mad_su(b_m, y, mul_su(a_m, x)), M), M.p);
    else return red1(redc_lazy((uint64_t)a_m * x + (uint64_t)b_m * y, M), M.p);
}

constexpr int ilog(int x, int b) { return x <= 1 ? 0 : 1 + ilog(x / b, b); }
constexpr int ipow(int b, int e) { return e == 0 ? 1 : b * ipow(b, e - 1); }
constexpr int rev_digits(int i, int base, int ndig) {
    int r = 0;
    for (int d = 0; d < ndig; ++d) { r = r * base + i % base; i /= base; }
    return r;
}

__device__ __forceinline__ int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
__device__ __forceinline__ int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__device__ __forceinline__ int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

}  // namespace packed
}  // namespace sda
