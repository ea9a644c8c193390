// modarith.h -- exact Rust-semantics integer arithmetic for gfx950 kernels.
//
// The reference computes on i64 with Rust's truncated `%` (client/src/crypto/mod.rs:33-36,
// combiner.rs:22-25).  CDNA4 has no integer divider, so every `%` becomes one of:
//   * a compare/adjust when the dividend is known to lie in (-2m, 2m)  (clerk combine);
//   * a Barrett reduction with a precomputed 64-bit reciprocal (generic, any m in [2, 2^63));
//   * Montgomery products (R = 2^32) for the packed-Shamir field (odd p < 2^31), where the
//     canonical residue and the sign of the exact i64 dividend are computed separately and
//     recombined into the truncated representative (see trunc_from()).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace sda {

// Compile-time loop: f(std::integral_constant<int, i>) for i = B, B+S, ... < E.  Keeps every
// register-array index a constant after inlining (no scratch spills from dynamic indexing).
template <int B, int E, int S = 1, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + S, E, S>(f);
    }
}

// ---------------------------------------------------------------------------------------
// Generic truncated remainder by a runtime modulus m >= 1 (Barrett, mu = floor(2^64 / m)).
// ---------------------------------------------------------------------------------------
struct Mod64 {
    uint64_t m;     // modulus, 1 <= m <= 2^63 - 1
    uint64_t mu;    // floor((2^64 - 1) / m); for m == 1 unused
};

__host__ __device__ inline Mod64 make_mod64(int64_t m) {
    Mod64 r;
    r.m = (uint64_t)m;
    r.mu = (m > 1) ? (UINT64_MAX / (uint64_t)m) : 0;
    return r;
}

__device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) {
    return __umul64hi(a, b);
}

// v mod m for any v in [0, 2^64).  q = mulhi(v, mu) is floor(v/m) or one less.
__device__ __forceinline__ uint64_t umod64(uint64_t v, const Mod64& M) {
    if (M.m == 1) return 0;
    uint64_t q = mulhi64(v, M.mu);
    uint64_t r = v - q * M.m;
    if (r >= M.m) r -= M.m;
    if (r >= M.m) r -= M.m;   // mu from UINT64_MAX (not 2^64) can leave one more step
    return r;
}

// Rust i64 `v % m` (truncated: sign of v), any v, m >= 1.
__device__ __forceinline__ int64_t trem64(int64_t v, const Mod64& M) {
    uint64_t a = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;   // |i64::MIN| = 2^63 ok
    uint64_t r = umod64(a, M);
    return v < 0 ? -(int64_t)r : (int64_t)r;
}

// Rust `(r + v) % m` where r in (-m, m) from a previous step, any v (wrapping add).
// Fast path: v in (-m, m) => r + v in (-2m, 2m) => one compare/adjust each side.
__device__ __forceinline__ int64_t add_trem(int64_t r, int64_t v, const Mod64& M, bool small_m) {
    int64_t x = (int64_t)((uint64_t)r + (uint64_t)v);
    const int64_t m = (int64_t)M.m;
    if (small_m && ((uint64_t)v + (uint64_t)(m - 1) < (uint64_t)(2 * m - 1))) {
        x = (x >= m) ? x - m : x;
        x = (x <= -m) ? x + m : x;
        return x;
    }
    return trem64(x, M);
}

// ---------------------------------------------------------------------------------------
// Montgomery field for odd p < 2^31, R = 2^32.
// ---------------------------------------------------------------------------------------
struct MontP {
    uint32_t p;       // odd prime < 2^31
    uint32_t pinv;    // -p^{-1} mod 2^32
    uint32_t r2;      // R^2 mod p
};

__host__ inline MontP make_mont(uint32_t p) {
    MontP M;
    M.p = p;
    uint32_t inv = 1;                       // Newton: inv = p^{-1} mod 2^32
    for (int i = 0; i < 5; ++i) inv *= 2u - p * inv;
    M.pinv = (uint32_t)(0u - inv);
    unsigned __int128 r = ((unsigned __int128)1 << 64) % p;
    M.r2 = (uint32_t)r;
    return M;
}

// REDC(T) = T * R^{-1} mod p, canonical, for T < p * R.
__device__ __forceinline__ uint32_t redc(uint64_t T, const MontP& M) {
    uint32_t u = (uint32_t)T * M.pinv;
    uint64_t s = T + (uint64_t)u * M.p;          // may exceed 2^64 only if T >= 2^64 - pR: not here
    // T < pR, u*p < pR  =>  T + u p < 2pR < 2^64 (p < 2^31)
    uint32_t t = (uint32_t)(s >> 32);
    return t >= M.p ? t - M.p : t;
}

// a * b mod p with a in Montgomery form (a' = a R mod p) and b canonical: returns canonical.
__device__ __forceinline__ uint32_t mont_mul(uint32_t a_mont, uint32_t b, const MontP& M) {
    return redc((uint64_t)a_mont * b, M);
}

// canonical residue of a value in (-p, p)
__device__ __forceinline__ uint32_t canon32(int32_t x, uint32_t p) {
    return x < 0 ? (uint32_t)(x + (int32_t)p) : (uint32_t)x;
}

// truncated-% representative with the sign of the exact dividend:
//   Rust (v % p) == neg ? (c ? c - p : 0) : c   where c = v mod p canonical, neg = v < 0.
__device__ __forceinline__ int32_t trunc_from(uint32_t c, bool neg, uint32_t p) {
    return neg ? (c ? (int32_t)c - (int32_t)p : 0) : (int32_t)c;
}

// ---------------------------------------------------------------------------------------
// Compare-free variants (no VCC write => no VALU->lane-mask hazard s_nops on gfx950).
// ---------------------------------------------------------------------------------------
// [0, 2p) -> [0, p):  t - p wraps above t when t < p, so the unsigned min picks the residue.
__device__ __forceinline__ uint32_t red1(uint32_t t, uint32_t p) { return min(t, t - p); }
__device__ __forceinline__ uint32_t addm(uint32_t a, uint32_t b, uint32_t p) { return red1(a + b, p); }
__device__ __forceinline__ uint32_t subm(uint32_t a, uint32_t b, uint32_t p) {
    const uint32_t d = a - b;            // a < b: wraps to >= 2^32 - p > d + p
    return min(d, d + p);
}
// REDC without the final subtraction: T < p * 2^32  ->  [0, 2p), congruent to T * 2^-32.
__device__ __forceinline__ uint32_t redc_lazy(uint64_t T, const MontP& M) {
    const uint32_t u = (uint32_t)T * M.pinv;
    return (uint32_t)((T + (uint64_t)u * M.p) >> 32);   // T + u p < 2^63 + 2^63
}
// Rust `v % p` from the canonical residue c of v and a word whose bit 31 is the sign of v:
// c - p when v < 0 and c != 0, else c  (sign bit of (sw & -c) is exactly that condition).
__device__ __forceinline__ int32_t trunc_rep(uint32_t c, uint32_t sw, uint32_t p) {
    const int32_t m = (int32_t)(sw & (0u - c)) >> 31;
    return (int32_t)(c - (p & (uint32_t)m));
}
__device__ __forceinline__ uint32_t hi32(int64_t v) { return (uint32_t)((uint64_t)v >> 32); }

// (a + b) mod p for canonical a, b
__device__ __forceinline__ uint32_t addmod(uint32_t a, uint32_t b, uint32_t p) {
    uint32_t s = a + b;          // < 2p < 2^32
    return s >= p ? s - p : s;
}
__device__ __forceinline__ uint32_t submod(uint32_t a, uint32_t b, uint32_t p) {
    return a >= b ? a - b : a + p - b;
}

}  // namespace sda
