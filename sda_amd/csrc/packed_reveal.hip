// packed_reveal.hip -- packed-Shamir reveal, EXACT (Newton) and CANONICAL (Lagrange).
#include <algorithm>

#include "packed_common.h"
#include "xcd.h"

namespace sda {
using namespace packed;

// Device table (u32 words), stride TS = 128 (max points):
//   [0, TS*TS)            inv[j][i]    canonical mod_inverse(points[i] - points[i-j])
//   [TS*TS, 2 TS*TS)      inv_m[j][i]  Montgomery form
//   [2TS^2, +KMAX*TS)     np[e][i]     signed Newton basis at omega_secrets^(e+1)  (EXACT)
//   [.. , +KMAX*TS)       np_m[e][i]   Montgomery form of canon(np)
//   [.. , +KMAX*TS)       lam_m[e][i]  Montgomery Lagrange weight of clerk i      (CANONICAL)
constexpr int TS = 128;
constexpr int KMAX = 64;
[[maybe_unused]] constexpr size_t OFF_INV = 0, OFF_INVM = (size_t)TS * TS, OFF_NP = 2 * (size_t)TS * TS,
                 OFF_NPM = OFF_NP + (size_t)KMAX * TS, OFF_LAM = OFF_NPM + (size_t)KMAX * TS,
                 TAB_WORDS = OFF_LAM + (size_t)KMAX * TS;

// One launcher per MM (the padded point count); each is compiled in its own object
// (Makefile: -DSDA_REVEAL_PART=MM) so the wide instantiations build in parallel.
template <int MM>
hipError_t reveal_launch(int mode, const PackedRevealArgs& a, uint64_t B, uint32_t n_idx, uint32_t k,
                         const uint32_t* tab, const MontP& M, unsigned int* log, hipStream_t s);

#ifdef SDA_REVEAL_PART
namespace {

// A field element: tss' exact representative s in (-p, p) and its canonical residue c.
struct FE {
    int32_t s;
    uint32_t c;
};

// The k secrets of a batch are adjacent in `out` (batched.rs:94 appends batch after batch), so a
// lane's own stores would stride by 8k bytes.  With STAGED the workgroup parks its results in
// LDS ([lane][k]) and writes the nb*k block back with coalesced stores.
// The results leave as nontemporal stores (written once, streamed out), 16 bytes per lane when the block's
// output is 16-byte aligned (lds_o is the dynamic LDS base, so 16-byte aligned too): canonical reveal -1.4 to
// -2.8 %, exact -0.7 to -1.1 % against 8-byte cached stores (in-process A/B on two boxes, profiles/r06ab, r06ac).
template <bool STAGED>
__device__ __forceinline__ void reveal_flush(int64_t* lds_o, int64_t* o, uint64_t b0, uint64_t B, uint64_t D,
                                             uint32_t k) {
    if constexpr (STAGED) {
        __syncthreads();
        const uint64_t first = b0 * k;
        const uint64_t last = (b0 + 256 < B ? b0 + 256 : B) * k;
        const uint32_t cnt = (uint32_t)((last < D ? last : D) - first);
        int64_t* dst = o + first;
        if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            using V2 = int64_t __attribute__((ext_vector_type(2)));
            const V2* src2 = reinterpret_cast<const V2*>(lds_o);
            V2* dst2 = reinterpret_cast<V2*>(dst);
            for (uint32_t j = threadIdx.x; j < cnt / 2; j += 256) __builtin_nontemporal_store(src2[j], dst2 + j);
            if ((cnt & 1) && threadIdx.x == 0) __builtin_nontemporal_store(lds_o[cnt - 1], dst + cnt - 1);
        } else {
            for (uint32_t j = threadIdx.x; j < cnt; j += 256) __builtin_nontemporal_store(lds_o[j], dst + j);
        }
    }
}

// gather [clerk][batch] -> [clerk] (batched.rs:83-85); point 1 carries value 0.  Clamped,
// branch-free indices, so every load can be issued before the first wait; each share is turned into
// its (sign, residue) pair as it lands, so no i64 copy stays live.  Returns whether every share lies
// in (-p, p).
template <int MMAX, bool EAGER>
__device__ __forceinline__ bool load_points(const int64_t* __restrict__ sh, uint64_t B, uint32_t m, uint32_t p,
                                            FE (&s)[MMAX]) {
    const int64_t P = (int64_t)p;
    s[0] = FE{0, 0};
    bool in_range = true;
    auto take = [&](auto i, int64_t v) {
        in_range = in_range && ((uint32_t)i >= m || (uint64_t)(v + (P - 1)) < (uint64_t)(2 * P - 1));
        const int32_t x = (uint32_t)i < m ? (int32_t)v : 0;
        s[i] = FE{x, canon32(x, p)};
    };
    if constexpr (EAGER) {               // every load first (all in flight), then convert
        int64_t v[MMAX];
        static_for<1, MMAX>([&](auto i) { v[i] = sh[(uint64_t)((uint32_t)i < m ? i - 1 : 0) * B]; });
        static_for<1, MMAX>([&](auto i) { take(i, v[i]); });
    } else {                             // convert as they land (no i64 copies live: fewer VGPRs)
        static_for<1, MMAX>([&](auto i) { take(i, sh[(uint64_t)((uint32_t)i < m ? i - 1 : 0) * B]); });
    }
    return in_range;
}

// tss reconstruct of one batch from its m points (shares in (-p, p)): Newton divided differences,
// then newton_evaluate at omega_secrets^(e+1), e < k; secrets e < lim go to dst[e].  With LAZY
// (the sign-bit formulation below) returns whether a zero residue appeared, in which case dst may
// hold garbage and the caller reruns the batch with LAZY = false (tss' `%` verbatim).
// KU > 0: the evaluation loop over the k <= KU secrets is unrolled (table offsets become
// compile-time constants: merged scalar loads, no per-secret loop overhead).
// FULL: m == MMAX, so every `i < m` guard is a compile-time constant: no per-step uniform branches,
// and the table rows load as merged s_load_dwordx16.
//
// LAZY: the sign-bit formulation.  A value is kept as its canonical residue c and a word whose bit 31
// is its sign n (value = c - p n; c = 0 implies n = 0).  Then both of tss' truncations are sign logic:
//   Newton step  sgn(s_i - s_{i-1}) = MAJ(n_i, ~n_{i-1}, [c_i < c_{i-1}])
//   fold step    x = acc + t with acc = (pc, n), t = (tc, sgn s xor sgn np):  y = pc + tc in [0, 2p),
//                sgn(x) = MAJ(n, sgn t, [y < p]) and pc' = y mod p
// (one v_bitop3 each) -- exact whenever no residue on the way is 0 (then tss gives 0 where the logic
// may say "negative"); ZeroTrap flags those batches (probability ~1/p per value) for the exact rerun.
template <int MMAX, int KU, bool FULL>
__device__ __forceinline__ bool newton_reveal_signbit(FE (&s)[MMAX], uint32_t m, uint32_t k,
                                                      const uint32_t* __restrict__ tab, const MontP& M, int64_t* dst,
                                                      uint32_t lim) {
    const uint32_t p = M.p;
    ZeroTrap zt;
    auto newton_step = [&](auto i, uint32_t j) {
        const uint32_t a_m = tab[OFF_INVM + j * TS + i];
        uint32_t fc, n;
        if constexpr (i == 1) {          // (s_1 - s_0) with s_0 = 0, the inserted point (1, 0)
            fc = montu<false>(a_m, s[1].c, M);
            n = (uint32_t)s[1].s;
        } else {
            const uint32_t d = s[i].c - s[i - 1].c;                    // bit 31: c_i < c_{i-1}
            fc = montu<false>(a_m, d + p, M);                          // d + p in (0, 2p): REDC input < pR
            n = maj3_nb((uint32_t)s[i].s, (uint32_t)s[i - 1].s, d);
        }
        s[i] = FE{(int32_t)n, fc};
        zt.note1(fc);
    };
    if constexpr (MMAX <= 16) {
        static_for<1, MMAX>([&](auto j) {
            if (FULL || (uint32_t)j < m) {
                static_for<0, MMAX - j>([&](auto ii) {
                    constexpr int i = MMAX - 1 - ii;
                    if (FULL || (uint32_t)i < m) newton_step(std::integral_constant<int, i>{}, (uint32_t)j);
                });
            }
        });
    } else {
        for (uint32_t j = 1; j < m; ++j) {
            static_for<0, MMAX - 1>([&](auto ii) {
                constexpr int i = MMAX - 1 - ii;
                if ((uint32_t)i < m && (uint32_t)i >= j) newton_step(std::integral_constant<int, i>{}, j);
            });
        }
    }
    // newton_evaluate: coefficient 0 is the inserted point's value 0, so the fold starts at i = 1
    auto eval = [&](uint32_t e) {
        const uint32_t* np = tab + OFF_NP + e * TS;
        const uint32_t* npm = tab + OFF_NPM + e * TS;
        uint32_t pc = 0, n = 0;
        static_for<1, MMAX>([&](auto i) {
            if (FULL || (uint32_t)i < m) {
                const uint32_t tc = montu<false>(npm[i], s[i].c, M);
                const uint32_t st = (uint32_t)s[i].s ^ np[i];               // bit 31: sign of s_i np_i
                if constexpr (i == 1) {
                    pc = tc;
                    n = st;
                } else {                         // (pc at i = 1 is c_1's product: 0 only if c_1 is)
                    const uint32_t y = pc + tc;
                    const uint32_t d = y - p;                               // bit 31: y < p
                    pc = min(y, d);
                    n = maj3(n, st, d);
                    zt.note1(pc);
                }
            }
        });
        zt.flush();
        if (e < lim) dst[e] = (int32_t)(pc - (p & (uint32_t)((int32_t)n >> 31)));     // batched.rs:94
    };
    if constexpr (KU > 0) {
        static_for<0, KU>([&](auto e) { if ((uint32_t)e < k) eval((uint32_t)e); });
    } else {
        for (uint32_t e = 0; e < k; ++e) eval(e);
    }
    return zt.bad();
}

template <int MMAX, int KU, bool LAZY, bool FULL>
__device__ __forceinline__ bool newton_reveal(FE (&s)[MMAX], uint32_t m, uint32_t k, const uint32_t* __restrict__ tab,
                                              const MontP& M, int64_t* dst, uint32_t lim) {
    if constexpr (LAZY) return newton_reveal_signbit<MMAX, KU, FULL>(s, m, k, tab, M, dst, lim);
    const uint32_t p = M.p;
    Trunc<false> tr;
    // numtheory::compute_newton_coefficients: for j in 1..m { for i in (j..m).rev() {
    //   s[i] = (((s[i] - s[i-1]) % p) * inv(points[i] - points[i-j])) % p } }
    // inv >= 0, so the product has the sign of the exact difference (or is 0).
    auto newton_step = [&](auto i, uint32_t j) {
        const uint32_t dc = s[i].c - s[i - 1].c + p;      // lazy: (0, 2p), REDC input < 2p^2 < pR
        const int32_t sg = __builtin_elementwise_sub_sat(s[i].s, s[i - 1].s);
        const uint32_t fc = montu<false>(tab[OFF_INVM + j * TS + i], dc, M);
        s[i] = FE{tr(fc, (uint32_t)sg, p), fc};
        tr.note1(s[i].s);
    };
    if constexpr (MMAX <= 16) {
        // fully unrolled triangle: every table word is a compile-time offset (merged s_loads)
        static_for<1, MMAX>([&](auto j) {
            if (FULL || (uint32_t)j < m) {
                static_for<0, MMAX - j>([&](auto ii) {
                    constexpr int i = MMAX - 1 - ii;
                    if (FULL || (uint32_t)i < m) newton_step(std::integral_constant<int, i>{}, (uint32_t)j);
                });
            }
        });
    } else {
        // wide index sets: runtime j, unrolled i (uniform branches); keeps code size O(MMAX)
        for (uint32_t j = 1; j < m; ++j) {
            static_for<0, MMAX - 1>([&](auto ii) {
                constexpr int i = MMAX - 1 - ii;
                if ((uint32_t)i < m && (uint32_t)i >= j) newton_step(std::integral_constant<int, i>{}, j);
            });
        }
    }
    // numtheory::newton_evaluate at omega_secrets^(e+1): fold((a + (coef * np) % p) % p)
    auto eval = [&](uint32_t e) {
        const uint32_t* np = tab + OFF_NP + e * TS;
        const uint32_t* npm = tab + OFF_NPM + e * TS;
        FE acc{0, 0};
        static_for<0, MMAX>([&](auto i) {
            if (FULL || (uint32_t)i < m) {
                const uint32_t tc = montu<false>(npm[i], s[i].c, M);
                const int32_t ts = tr(tc, (uint32_t)s[i].s ^ np[i], p);     // sign of s * np (np != 0 mod p)
                const uint32_t ac = addm(acc.c, tc, p);
                acc = FE{tr(ac, (uint32_t)__builtin_elementwise_add_sat(acc.s, ts), p), ac};
                tr.note2(ts, acc.s);
            }
        });
        if (e < lim) dst[e] = acc.s;                                                // batched.rs:94
    };
    if constexpr (KU > 0) {
        static_for<0, KU>([&](auto e) { if ((uint32_t)e < k) eval((uint32_t)e); });
    } else {
        for (uint32_t e = 0; e < k; ++e) eval(e);
    }
    return tr.bad(p);
}

// One lane = one batch.  LAZY (p >= kLazyTruncMinP): the sign-bit path with its zero trap.  A lane whose
// batch hit the trap (probability ~1/p per value) or has a share outside (-p, p) (raw i64 input) logs
// the batch and stores garbage; packed_reveal_fixup_kernel, launched right after on the same stream,
// recomputes the logged batches (exact truncation in registers, or the generic i64 path).  Keeping
// the generic path (a 128-entry i64 array per lane) out of this kernel keeps it free of scratch.
template <int MMAX, bool STAGED, int KU, bool LAZY, bool FULL = false>
__global__ __launch_bounds__(256) void packed_reveal_exact_kernel(const int64_t* __restrict__ shares, uint64_t B,
                                                                  uint64_t D, int64_t* __restrict__ out,
                                                                  uint32_t n_idx, uint32_t k,
                                                                  const uint32_t* __restrict__ tab, MontP M,
                                                                  unsigned int* __restrict__ log, int xcd) {
    extern __shared__ int64_t lds_o[];
    const uint32_t tid = threadIdx.x;
    // XCD-chunked tile order (xcd.h), for the point counts up to 16 (the benchmarked sizes; the wide
    // instantiations keep the natural order's code unchanged)
    uint32_t tile = blockIdx.x, vy = blockIdx.y;
    if constexpr (MMAX <= 16) {
        if (xcd) xcd_block_xy(&tile, &vy);
    }
    const uint64_t b0 = (uint64_t)tile * 256, b = b0 + tid;
    const bool live = b < B;
    const uint64_t vec = vy;
    const int64_t* sh = shares + vec * (uint64_t)n_idx * B + (live ? b : B - 1);
    int64_t* o = out + vec * D;
    const uint32_t m = FULL ? (uint32_t)MMAX : n_idx + 1;
    int64_t* dst = STAGED ? lds_o + tid * k : o + b * k;
    const uint32_t lim = STAGED ? k : (b * k < D ? (uint32_t)(D - b * k < k ? D - b * k : k) : 0u);

    FE s[MMAX];
    const bool in_range = load_points<MMAX, (KU > 0)>(sh, B, m, M.p, s);
    const bool redo = !in_range || newton_reveal<MMAX, KU, LAZY, FULL>(s, m, k, tab, M, dst, lim);
    if (redo && live) {                                  // -> packed_reveal_fixup_kernel
        const uint32_t slot = atomicAdd(log, 1u);
        if (slot < kGenLogCap) reinterpret_cast<uint64_t*>(log + 16)[slot] = vec * B + b;
    }
    reveal_flush<STAGED>(lds_o, o, b0, B, D, k);
}

// Generic exact reveal of one batch (shares outside (-p, p)): tss' Newton divided differences and
// evaluation with wrapping i64 arithmetic and truncated `%`, reading the batch's shares from global
// memory.  Writes its first `lim` secrets to dst[0..lim).
__device__ void reveal_exact_generic(const int64_t* __restrict__ sh, uint64_t B, uint32_t m, uint32_t k,
                                     const uint32_t* __restrict__ tab, uint32_t p, int64_t* dst, uint32_t lim) {
    const Mod64 P = make_mod64((int64_t)p);
    int64_t s[TS];
    s[0] = 0;
    for (uint32_t i = 1; i < m; ++i) s[i] = sh[(uint64_t)(i - 1) * B];
    for (uint32_t j = 1; j < m; ++j)
        for (uint32_t i = m - 1; i >= j; --i) {
            const int64_t cd = trem64(wsub(s[i], s[i - 1]), P);
            s[i] = trem64(wmul(cd, (int64_t)tab[OFF_INV + j * TS + i]), P);
        }
    for (uint32_t e = 0; e < k && e < lim; ++e) {
        int64_t acc = 0;
        for (uint32_t i = 0; i < m; ++i) {
            const int64_t np = (int64_t)(int32_t)tab[OFF_NP + e * TS + i];
            acc = trem64(wadd(acc, trem64(wmul(s[i], np), P)), P);
        }
        dst[e] = acc;
    }
}

// The batches packed_reveal_exact_kernel logged: in-range ones (lazy-truncation traps) rerun the
// register path with tss' truncation verbatim; out-of-range ones take the generic i64 path.  If the
// log overflowed, every batch of the launch is recomputed (correct and slow; only reachable with raw
// i64 shares).  One wave per workgroup: a logged batch is rare, so few lanes are busy.
template <int MMAX, int KU>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void packed_reveal_fixup_kernel(const int64_t* __restrict__ shares, uint64_t B,
                                                                 uint64_t D, uint64_t n_vec, int64_t* __restrict__ out,
                                                                 uint32_t n_idx, uint32_t k,
                                                                 const uint32_t* __restrict__ tab, MontP M,
                                                                 const unsigned int* __restrict__ log) {
    const uint32_t n = *log;
    if (n == 0) return;
    const bool all = n > kGenLogCap;
    const uint64_t total = all ? B * n_vec : (uint64_t)n;
    const uint64_t* list = reinterpret_cast<const uint64_t*>(log + 16);
    const uint32_t m = n_idx + 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t gb = all ? i : list[i];
        const uint64_t vec = gb / B, b = gb - vec * B;
        const uint32_t lim = b * k < D ? (uint32_t)(D - b * k < k ? D - b * k : k) : 0u;
        const int64_t* sh = shares + vec * (uint64_t)n_idx * B + b;
        int64_t* dst = out + vec * D + b * k;
        FE s[MMAX];
        if (load_points<MMAX, false>(sh, B, m, M.p, s)) newton_reveal<MMAX, KU, false, false>(s, m, k, tab, M, dst, lim);
        else reveal_exact_generic(sh, B, m, k, tab, M.p, dst, lim);
    }
}

// The same fix-up with one WAVE per logged batch (m <= 64 points): lane i holds Newton point i, so each
// of the m - 1 levels of tss' divided differences is one parallel step (lane i needs only lane i - 1's
// value of the previous level -- the in-place descending loop reads exactly that), and lane e < k folds
// newton_evaluate at omega_secrets^(e+1) with the coefficients broadcast from their lanes.  Exact i64
// arithmetic with truncated `%` throughout (the generic path's), so in-range and raw i64 shares are
// handled alike.  A trapped batch is a serial latency chain for one lane on the register path (~40 us);
// spread over the wave it is m + k short steps.
// Rust `v % p` for |v| < 2^62 (a product of two values in (-p, p), p < 2^31): the quotient from a double
// product (exact operands, relative error 2^-53, so |q - v/p| < 1) and one signed correction step.
__device__ __forceinline__ int64_t trem_prod(int32_t a, int32_t b, uint32_t p, double pinv) {
    const int64_t v = (int64_t)a * b;
    const int64_t q = (int64_t)__builtin_trunc((double)a * (double)b * pinv);
    int64_t r = v - q * (int64_t)p;                     // v - trunc(v/p) p, off by at most one p
    if (v >= 0) { r = r < 0 ? r + p : r; r = r >= (int64_t)p ? r - p : r; }
    else { r = r > 0 ? r - p : r; r = r <= -(int64_t)p ? r + p : r; }
    return r;
}
// Rust `v % p` for |v| < 2p.
__device__ __forceinline__ int32_t trem_small(int64_t v, uint32_t p) {
    const int64_t P = p;
    return (int32_t)(v >= P ? v - P : (v <= -P ? v + P : v));
}

// The same fix-up with one WAVE per logged batch (m <= 64 points): lane i holds Newton point i, so each
// of the m - 1 levels of tss' divided differences is one parallel step (lane i needs only lane i - 1's
// value of the previous level -- the in-place descending loop reads exactly that), and lane e < k folds
// newton_evaluate at omega_secrets^(e+1) with the coefficients broadcast from their lanes.  Each lane
// preloads its column of the inverse table and its row of Newton bases, so no step waits on memory.
// Shares in (-p, p) keep every tss intermediate in (-p, p): 32-bit values, `%` of products through
// trem_prod; otherwise (raw i64 shares) the generic i64 arithmetic.  A trapped batch is a serial
// latency chain for one lane on the register path (~40 us); spread over the wave it is m + k short steps.
template <int MMAX>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void packed_reveal_fixup_wave_kernel(const int64_t* __restrict__ shares, uint64_t B,
                                                                      uint64_t D, uint64_t n_vec,
                                                                      int64_t* __restrict__ out, uint32_t n_idx,
                                                                      uint32_t k, const uint32_t* __restrict__ tab,
                                                                      uint32_t p, const unsigned int* __restrict__ log) {
    static_assert(MMAX <= 64, "one lane per Newton point");
    const uint32_t n = *log;
    if (n == 0) return;
    const bool all = n > kGenLogCap;
    const uint64_t total = all ? B * n_vec : (uint64_t)n;
    if ((uint64_t)blockIdx.x >= total) return;          // waves without a batch skip the table preload
    const uint64_t* list = reinterpret_cast<const uint64_t*>(log + 16);
    const uint32_t m = n_idx + 1, lane = threadIdx.x;
    const Mod64 P = make_mod64((int64_t)p);
    const double pinv = 1.0 / (double)p;
    // this lane's inv[j][lane] and np[lane][i]: in registers up to 16 points; past that in LDS (2 x 16 KiB), so
    // the 32- and 64-point instantiations stay inside 256 VGPRs (round 5 held both tables in registers: 274 and
    // 376 registers, AGPRs standing in for VGPRs -- tests/test_kernel_resources.py)
    constexpr bool REG = MMAX <= 16;
    constexpr int RT = REG ? MMAX : 1;
    int32_t inv_r[RT], np_r[RT];
    __shared__ int32_t tabs[REG ? 1 : 2 * MMAX * 64];
    auto inv = [&](int j) -> int32_t {
        if constexpr (REG) return inv_r[j]; else return tabs[j * 64 + lane];
    };
    auto np = [&](int i) -> int32_t {
        if constexpr (REG) return np_r[i]; else return tabs[(MMAX + i) * 64 + lane];
    };
#pragma unroll
    for (int j = 0; j < MMAX; ++j) {
        const int32_t iv = (j >= 1 && lane < MMAX) ? (int32_t)tab[OFF_INV + j * TS + (lane < MMAX ? lane : 0)] : 0;
        const int32_t nv = lane < k ? (int32_t)tab[OFF_NP + (lane < k ? lane : 0) * TS + j] : 0;
        if constexpr (REG) { inv_r[j] = iv; np_r[j] = nv; }
        else { tabs[j * 64 + lane] = iv; tabs[(MMAX + j) * 64 + lane] = nv; }
    }
    if constexpr (!REG) __syncthreads();
    for (uint64_t w = blockIdx.x; w < total; w += gridDim.x) {
        const uint64_t gb = all ? w : list[w];
        const uint64_t vec = gb / B, b = gb - vec * B;
        // point 0 is the inserted (1, 0); point i >= 1 is clerk share i - 1 (batched.rs:83-85)
        int64_t s = (lane >= 1 && lane < m) ? shares[vec * (uint64_t)n_idx * B + (uint64_t)(lane - 1) * B + b] : 0;
        const bool small = __all((uint64_t)(s + (int64_t)p - 1) < (uint64_t)(2 * (int64_t)p - 1));
        const uint32_t lim = b * k < D ? (uint32_t)(D - b * k < k ? D - b * k : k) : 0u;
        int64_t acc = 0;
        if (small) {
            int32_t x = (int32_t)s;
#pragma unroll
            for (int j = 1; j < MMAX; ++j) {
                const int32_t prev = __shfl_up(x, 1);
                if ((uint32_t)j < m && lane >= (uint32_t)j && lane < m)
                    x = (int32_t)trem_prod(trem_small((int64_t)x - prev, p), inv(j), p, pinv);
            }
            int32_t a = 0;
#pragma unroll
            for (int i = 0; i < MMAX; ++i) {
                const int32_t c = __shfl(x, i);
                if ((uint32_t)i < m) a = trem_small((int64_t)a + trem_prod(c, np(i), p, pinv), p);
            }
            acc = a;
        } else {
#pragma unroll
            for (int j = 1; j < MMAX; ++j) {
                const int64_t prev = __shfl_up(s, 1);
                if ((uint32_t)j < m && lane >= (uint32_t)j && lane < m)
                    s = trem64(wmul(trem64(wsub(s, prev), P), inv(j)), P);
            }
#pragma unroll
            for (int i = 0; i < MMAX; ++i) {
                const int64_t c = __shfl(s, i);
                if ((uint32_t)i < m) acc = trem64(wadd(acc, trem64(wmul(c, np(i)), P)), P);
            }
        }
        if (lane < lim) out[vec * D + b * k + lane] = acc;                     // batched.rs:94
    }
}

template <int NMAX, bool STAGED>
__global__ __launch_bounds__(256) void packed_reveal_canon_kernel(const int64_t* __restrict__ shares, uint64_t B,
                                                                  uint64_t D, int64_t* __restrict__ out,
                                                                  uint32_t n_idx, uint32_t k,
                                                                  const uint32_t* __restrict__ tab, MontP M, int xcd) {
    extern __shared__ int64_t lds_o[];
    const uint32_t tid = threadIdx.x;
    uint32_t tile = blockIdx.x, vy = blockIdx.y;
    if constexpr (NMAX <= 16) {
        if (xcd) xcd_block_xy(&tile, &vy);
    }
    const uint64_t b0 = (uint64_t)tile * 256, b = b0 + tid;
    const bool live = b < B;
    const uint64_t vec = vy;
    const int64_t* sh = shares + vec * (uint64_t)n_idx * B + (live ? b : B - 1);
    int64_t* o = out + vec * D;
    const uint32_t p = M.p;
    const int64_t P = (int64_t)p;
    int64_t* dst = STAGED ? lds_o + tid * k : o + b * k;
    const uint32_t lim = STAGED ? k : (b * k < D ? (uint32_t)(D - b * k < k ? D - b * k : k) : 0u);

    uint32_t S[NMAX];
    bool in_range = true;
    auto take = [&](auto i, int64_t v) {
        in_range = in_range && ((uint32_t)i >= n_idx || (uint64_t)(v + (P - 1)) < (uint64_t)(2 * P - 1));
        S[i] = (uint32_t)i < n_idx ? canon32((int32_t)v, p) : 0u;
    };
    if constexpr (NMAX <= 32) {          // every load first (all in flight), then convert
        int64_t v[NMAX];
        static_for<0, NMAX>([&](auto i) { v[i] = sh[(uint64_t)((uint32_t)i < n_idx ? i : 0) * B]; });
        static_for<0, NMAX>([&](auto i) { take(i, v[i]); });
    } else {                             // wide sets: convert as they land (no i64 copies live)
        static_for<0, NMAX>([&](auto i) { take(i, sh[(uint64_t)((uint32_t)i < n_idx ? i : 0) * B]); });
    }
    if (!in_range) {                    // raw i64 shares: exact canonical residues (rare; reloaded)
        const Mod64 PM = make_mod64(P);
        static_for<0, NMAX>([&](auto i) {
            const int64_t r = trem64(sh[(uint64_t)((uint32_t)i < n_idx ? i : 0) * B], PM);
            S[i] = (uint32_t)i < n_idx ? (uint32_t)(r < 0 ? r + P : r) : 0u;
        });
    }
    // secret_e = sum_i lambda_{e,i} share_i  (mod p); pairs of products share one REDC (2 p^2 < p R)
    for (uint32_t e = 0; e < k; ++e) {
        const uint32_t* lam = tab + OFF_LAM + e * TS;
        uint32_t acc = 0;
        static_for<0, NMAX, 2>([&](auto i) {
            if ((uint32_t)i < n_idx) {
                uint64_t T = (uint64_t)lam[i] * S[i];
                if constexpr (i + 1 < NMAX) T += (uint64_t)lam[i + 1] * S[i + 1];   // lam, S are 0 past n_idx
                acc = addm(acc, red1(redc_lazy(T, M), p), p);
            }
        });
        if (e < lim) dst[e] = (int64_t)acc;
    }
    reveal_flush<STAGED>(lds_o, o, b0, B, D, k);
}

}  // namespace

template <int MM>
hipError_t reveal_launch(int mode, const PackedRevealArgs& a, uint64_t B, uint32_t n_idx, uint32_t k,
                         const uint32_t* tab, const MontP& M, unsigned int* log, hipStream_t s) {
    dim3 grid((unsigned)((B + 255) / 256), (unsigned)a.n_vectors);
    const bool staged = k <= 16;                      // LDS stage: 256 * k * 8 B <= 32 KiB
    const size_t lds = staged ? (size_t)256 * k * sizeof(int64_t) : 0;
    const int xcd = xcd_order_enabled() && (uint64_t)grid.x * grid.y < (1ull << 32) ? 1 : 0;
    if (mode == 0) {
        bool done = false;
        if constexpr (MM <= 16) {
            done = staged && k <= 8;
            if (done && M.p >= kLazyTruncMinP && n_idx + 1 == MM)
                hipLaunchKernelGGL((packed_reveal_exact_kernel<MM, true, 8, true, true>), grid, dim3(256), lds, s,
                                   a.shares, B, a.dimension, a.out, n_idx, k, tab, M, log, xcd);
            else if (done && M.p >= kLazyTruncMinP)
                hipLaunchKernelGGL((packed_reveal_exact_kernel<MM, true, 8, true>), grid, dim3(256), lds, s,
                                   a.shares, B, a.dimension, a.out, n_idx, k, tab, M, log, xcd);
            else if (done)
                hipLaunchKernelGGL((packed_reveal_exact_kernel<MM, true, 8, false>), grid, dim3(256), lds, s,
                                   a.shares, B, a.dimension, a.out, n_idx, k, tab, M, log, xcd);
        }
        if (done) {
        } else if (staged) {
            hipLaunchKernelGGL((packed_reveal_exact_kernel<MM, true, 0, false>), grid, dim3(256), lds, s, a.shares,
                               B, a.dimension, a.out, n_idx, k, tab, M, log, xcd);
        } else {
            hipLaunchKernelGGL((packed_reveal_exact_kernel<MM, false, 0, false>), grid, dim3(256), 0, s, a.shares,
                               B, a.dimension, a.out, n_idx, k, tab, M, log, xcd);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        if constexpr (MM <= 64) {
            if (k <= 64)
                hipLaunchKernelGGL((packed_reveal_fixup_wave_kernel<MM>), dim3(1024), dim3(64), 0, s, a.shares, B,
                                   a.dimension, a.n_vectors, a.out, n_idx, k, tab, M.p, log);
            else
                hipLaunchKernelGGL((packed_reveal_fixup_kernel<MM, 0>), dim3(64), dim3(64), 0, s, a.shares, B,
                                   a.dimension, a.n_vectors, a.out, n_idx, k, tab, M, log);
        } else
            hipLaunchKernelGGL((packed_reveal_fixup_kernel<MM, 0>), dim3(64), dim3(64), 0, s, a.shares, B,
                               a.dimension, a.n_vectors, a.out, n_idx, k, tab, M, log);
    } else if constexpr (MM <= 32) {
        if (staged)
            hipLaunchKernelGGL((packed_reveal_canon_kernel<MM, true>), grid, dim3(256), lds, s, a.shares, B,
                               a.dimension, a.out, n_idx, k, tab, M, xcd);
        else
            hipLaunchKernelGGL((packed_reveal_canon_kernel<MM, false>), grid, dim3(256), 0, s, a.shares, B,
                               a.dimension, a.out, n_idx, k, tab, M, xcd);
    } else {
        return hipErrorInvalidValue;                  // launch_packed_reveal runs these as exact + canonical
    }
    return hipGetLastError();
}
template hipError_t reveal_launch<SDA_REVEAL_PART>(int, const PackedRevealArgs&, uint64_t, uint32_t, uint32_t,
                                                   const uint32_t*, const MontP&, unsigned int*, hipStream_t);

#else  // dispatcher + host tables

// Host precompute of the per-index-set tables (data independent; same ops as tss).
static void build_reveal_tables(std::vector<uint32_t>& tab, const uint64_t* indices, uint32_t n_idx, uint32_t k,
                                int64_t p, int64_t ws, int64_t wn, bool want_lagrange, bool* duplicate) {
    tab.assign(TAB_WORDS, 0);
    const uint32_t m = n_idx + 1;
    std::vector<int64_t> pts(m);
    pts[0] = 1;                                                    // points.insert(0, 1)
    for (uint32_t i = 0; i < n_idx; ++i) pts[i + 1] = h_powmod(wn, (uint32_t)(indices[i] + 1), p);
    for (uint32_t j = 1; j < m; ++j)
        for (uint32_t i = j; i < m; ++i) {
            const int64_t diff = h_rem(pts[i] - pts[i - j], p);    // store[i] covers [i-j, i]
            const int64_t inv = h_modinv(diff, p);
            tab[OFF_INV + j * TS + i] = (uint32_t)inv;
            tab[OFF_INVM + j * TS + i] = to_mont(inv, p);
        }
    *duplicate = false;
    for (uint32_t a = 0; a < m; ++a)
        for (uint32_t c = a + 1; c < m; ++c)
            if (pts[a] == pts[c]) *duplicate = true;
    for (uint32_t e = 0; e < k; ++e) {
        const int64_t point = h_powmod(ws, e + 1, p);
        int64_t np = 1;
        for (uint32_t i = 0; i < m; ++i) {
            tab[OFF_NP + e * TS + i] = (uint32_t)(int32_t)np;
            tab[OFF_NPM + e * TS + i] = to_mont(np, p);
            if (i + 1 < m) np = h_rem(np * h_rem(point - pts[i], p), p);
        }
        if (want_lagrange && !*duplicate) {
            // lambda_i = prod_{j != i+1} (X - x_j) / (x_{i+1} - x_j), over all m points
            for (uint32_t i = 0; i < n_idx; ++i) {
                int64_t num = 1, den = 1;
                for (uint32_t j = 0; j < m; ++j) {
                    if (j == i + 1) continue;
                    int64_t a = (point - pts[j]) % p; if (a < 0) a += p;
                    int64_t d = (pts[i + 1] - pts[j]) % p; if (d < 0) d += p;
                    num = num * a % p; den = den * d % p;
                }
                const int64_t lam = num * h_modinv(den, p) % p;
                tab[OFF_LAM + e * TS + i] = to_mont(lam, p);
            }
        }
    }
}

hipError_t launch_packed_reveal(const PackedRevealArgs& a, const uint64_t* indices, uint32_t n_idx, uint32_t k,
                                uint32_t p, uint32_t omega_secrets, uint32_t omega_shares, int mode,
                                DeviceTable& tab, void* log_buf, hipStream_t s) {
    const uint64_t B = (a.dimension + k - 1) / k;
    if (B == 0 || a.n_vectors == 0) return hipSuccess;
    if ((mode == 0 ? n_idx + 1 : n_idx) > (uint32_t)kRevealMaxPoints || k > (uint32_t)KMAX)   // packed_wide.hip
        return launch_packed_reveal_wide(a, indices, n_idx, k, p, omega_secrets, omega_shares, mode, tab, s);
    if (mode == 1 && n_idx > 32) {
        // CANONICAL from more than 32 shares: the exact Newton kernels, then one canonicalising pass -- the same
        // values by definition (CANONICAL = positive() of the exact reveal, as on the workspace path).  The
        // Lagrange kernel's 64- and 96-point instantiations needed AGPRs standing in for VGPRs, or scratch
        // (tests/test_kernel_resources.py; DESIGN.md §4.2 "Register budget at n + 1 = 81").
        std::vector<int64_t> pts(n_idx);
        for (uint32_t i = 0; i < n_idx; ++i) pts[i] = h_powmod(omega_shares, (uint32_t)(indices[i] + 1), p);
        std::sort(pts.begin(), pts.end());
        if (std::adjacent_find(pts.begin(), pts.end()) != pts.end() || pts[0] == 1)
            return hipErrorInvalidValue;              // repeated points: no Lagrange form (as the canonical tables)
        const uint32_t m = n_idx + 1;
        hipError_t e = m > (uint32_t)kRevealMaxPoints
                           ? launch_packed_reveal_wide(a, indices, n_idx, k, p, omega_secrets, omega_shares, 1, tab, s)
                           : launch_packed_reveal(a, indices, n_idx, k, p, omega_secrets, omega_shares, 0, tab,
                                                  log_buf, s);
        if (e != hipSuccess || m > (uint32_t)kRevealMaxPoints) return e;
        return launch_mod_canonical(a.out, a.dimension * a.n_vectors, a.out, p, s);
    }
    std::vector<uint8_t> key(sizeof(uint32_t) * 6 + sizeof(uint64_t) * n_idx);
    const uint32_t kv[6] = {n_idx, k, p, omega_secrets, omega_shares, (uint32_t)mode};
    memcpy(key.data(), kv, sizeof(kv));
    memcpy(key.data() + sizeof(kv), indices, sizeof(uint64_t) * n_idx);
    if (tab.key != key) {
        std::vector<uint32_t> host;
        bool dup = false;
        build_reveal_tables(host, indices, n_idx, k, p, omega_secrets, omega_shares, mode == 1, &dup);
        if (mode == 1 && dup) return hipErrorInvalidValue;
        hipError_t e = ensure_table(tab, key, host.data(), host.size() * sizeof(uint32_t));
        if (e != hipSuccess) return e;
    }
    const MontP M = make_mont(p);
    const uint32_t* dtab = static_cast<const uint32_t*>(tab.dev);
    const uint32_t m = n_idx + 1;
    const uint32_t need = mode == 0 ? m : n_idx;
    unsigned int* log = static_cast<unsigned int*>(log_buf);
    hipError_t e = hipSuccess;
    if (mode == 0 && (e = hipMemsetAsync(log, 0, sizeof(unsigned int), s)) != hipSuccess) return e;
    if (need <= 8) e = reveal_launch<8>(mode, a, B, n_idx, k, dtab, M, log, s);
    else if (need <= 16) e = reveal_launch<16>(mode, a, B, n_idx, k, dtab, M, log, s);
    else if (need <= 32) e = reveal_launch<32>(mode, a, B, n_idx, k, dtab, M, log, s);
    else if (need <= 64) e = reveal_launch<64>(mode, a, B, n_idx, k, dtab, M, log, s);
    else if (need <= kRevealMaxPoints) e = reveal_launch<kRevealMaxPoints>(mode, a, B, n_idx, k, dtab, M, log, s);
    else return hipErrorInvalidValue;
    return e;
}

#endif  // SDA_REVEAL_PART

}  // namespace sda
