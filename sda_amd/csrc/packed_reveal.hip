// packed_reveal.hip -- packed-Shamir reveal, EXACT (Newton) and CANONICAL (Lagrange).
#include "packed_common.h"

namespace sda {
using namespace packed;

namespace {

// ------------------------------------------------------------------------------------------
// reveal
// ------------------------------------------------------------------------------------------
// Device table (u32 words), stride TS = 128 (max points):
//   [0, TS*TS)            inv[j][i]    canonical mod_inverse(points[i] - points[i-j])
//   [TS*TS, 2 TS*TS)      inv_m[j][i]  Montgomery form
//   [2TS^2, +KMAX*TS)     np[e][i]     signed Newton basis at omega_secrets^(e+1)  (EXACT)
//   [.. , +KMAX*TS)       np_m[e][i]   Montgomery form of canon(np)
//   [.. , +KMAX*TS)       lam_m[e][i]  Montgomery Lagrange weight of clerk i      (CANONICAL)
constexpr int TS = 128;
constexpr int KMAX = 64;
constexpr size_t OFF_INV = 0, OFF_INVM = (size_t)TS * TS, OFF_NP = 2 * (size_t)TS * TS,
                 OFF_NPM = OFF_NP + (size_t)KMAX * TS, OFF_LAM = OFF_NPM + (size_t)KMAX * TS,
                 TAB_WORDS = OFF_LAM + (size_t)KMAX * TS;

__device__ __forceinline__ int64_t trunc_small(int64_t x, int64_t p) {   // x in (-2p, 2p)
    x = x >= p ? x - p : x;
    return x <= -p ? x + p : x;
}

// generic exact reveal for one batch (inputs outside (-p, p) or m > unrolled sizes)
// Reads the batch's shares from global memory and writes its secrets (truncated at D) itself.
__device__ __noinline__ void reveal_exact_generic(const int64_t* __restrict__ sh, uint64_t B, uint32_t m, uint32_t k,
                                                  const uint32_t* __restrict__ tab, const MontP& M,
                                                  int64_t* o, uint64_t b, uint64_t D) {
    const Mod64 P = make_mod64((int64_t)M.p);
    int64_t s[TS];
    s[0] = 0;
    for (uint32_t i = 1; i < m; ++i) s[i] = sh[(uint64_t)(i - 1) * B];
    for (uint32_t j = 1; j < m; ++j)
        for (uint32_t i = m - 1; i >= j; --i) {
            const int64_t cd = trem64(wsub(s[i], s[i - 1]), P);
            s[i] = trem64(wmul(cd, (int64_t)tab[OFF_INV + j * TS + i]), P);
        }
    for (uint32_t e = 0; e < k; ++e) {
        int64_t acc = 0;
        for (uint32_t i = 0; i < m; ++i) {
            const int64_t np = (int64_t)(int32_t)tab[OFF_NP + e * TS + i];
            acc = trem64(wadd(acc, trem64(wmul(s[i], np), P)), P);
        }
        if (b * k + e < D) o[b * k + e] = acc;
    }
}

template <int MMAX>
__global__ __launch_bounds__(256) void packed_reveal_exact_kernel(const int64_t* __restrict__ shares, uint64_t B,
                                                                  uint64_t D, int64_t* __restrict__ out,
                                                                  uint32_t n_idx, uint32_t k,
                                                                  const uint32_t* __restrict__ tab, MontP M) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint64_t vec = blockIdx.y;
    const int64_t* sh = shares + vec * (uint64_t)n_idx * B + b;
    int64_t* o = out + vec * D;
    const uint32_t p = M.p;
    const int64_t P = (int64_t)p;
    const uint32_t m = n_idx + 1;

    // gather [clerk][batch] -> [clerk] (batched.rs:83-85); point 1 carries value 0
    int32_t s[MMAX];
    bool in_range = true;
    s[0] = 0;
    static_for<1, MMAX>([&](auto i) {
        int64_t v = 0;
        if ((uint32_t)i < m) v = sh[(uint64_t)(i - 1) * B];
        in_range = in_range && (v > -P) && (v < P);
        s[i] = (int32_t)v;
    });
    if (!in_range) {
        reveal_exact_generic(sh, B, m, k, tab, M, o, b, D);
        return;
    }
    // numtheory::compute_newton_coefficients: for j in 1..m { for i in (j..m).rev() { ... } }
    static_for<1, MMAX>([&](auto j) {
        if ((uint32_t)j < m) {
            static_for<0, MMAX - j>([&](auto ii) {
                constexpr int i = MMAX - 1 - ii;
                if ((uint32_t)i < m) {
                    const int64_t cd = trunc_small((int64_t)s[i] - (int64_t)s[i - 1], P);   // (upper - lower) % p
                    const uint32_t inv = tab[OFF_INV + j * TS + i], inv_m = tab[OFF_INVM + j * TS + i];
                    const uint32_t c = mont_mul(inv_m, canon32((int32_t)cd, p), M);       // (cd * inv) % p
                    s[i] = trunc_from(c, (cd < 0) && (inv != 0), p);
                }
            });
        }
    });
    // numtheory::newton_evaluate at omega_secrets^e: fold((a + (coef * np) % p) % p)
    for (uint32_t e = 0; e < k; ++e) {
        int64_t acc = 0;
        static_for<0, MMAX>([&](auto i) {
            if ((uint32_t)i < m) {
                const int32_t np = (int32_t)tab[OFF_NP + e * TS + i];
                const uint32_t c = mont_mul(tab[OFF_NPM + e * TS + i], canon32(s[i], p), M);
                const bool neg = (s[i] != 0) && (np != 0) && ((s[i] < 0) != (np < 0));
                acc = trunc_small(acc + trunc_from(c, neg, p), P);
            }
        });
        if (b * k + e < D) o[b * k + e] = acc;                                          // batched.rs:94
    }
}

template <int NMAX>
__global__ __launch_bounds__(256) void packed_reveal_canon_kernel(const int64_t* __restrict__ shares, uint64_t B,
                                                                  uint64_t D, int64_t* __restrict__ out,
                                                                  uint32_t n_idx, uint32_t k,
                                                                  const uint32_t* __restrict__ tab, MontP M) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint64_t vec = blockIdx.y;
    const int64_t* sh = shares + vec * (uint64_t)n_idx * B + b;
    int64_t* o = out + vec * D;
    const uint32_t p = M.p;
    const int64_t P = (int64_t)p;
    const Mod64 PM = make_mod64(P);
    uint32_t S[NMAX];
    static_for<0, NMAX>([&](auto i) {
        uint32_t c = 0;
        if ((uint32_t)i < n_idx) {
            const int64_t v = sh[(uint64_t)i * B];
            if ((v > -P) && (v < P)) c = canon32((int32_t)v, p);
            else { const int64_t r = trem64(v, PM); c = (uint32_t)(r < 0 ? r + P : r); }
        }
        S[i] = c;
    });
    for (uint32_t e = 0; e < k; ++e) {
        uint32_t acc = 0;
        static_for<0, NMAX, 2>([&](auto i) {
            if ((uint32_t)i < n_idx) {
                uint64_t T = (uint64_t)tab[OFF_LAM + e * TS + i] * S[i];
                if constexpr (i + 1 < NMAX) {
                    if ((uint32_t)(i + 1) < n_idx) T += (uint64_t)tab[OFF_LAM + e * TS + i + 1] * S[i + 1];
                }
                acc = addmod(acc, redc(T, M), p);                    // 2 p^2 < p R
            }
        });
        if (b * k + e < D) o[b * k + e] = (int64_t)acc;
    }
}

}  // namespace


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

template <int MM>
static hipError_t reveal_launch(int mode, const PackedRevealArgs& a, uint64_t B, uint32_t n_idx, uint32_t k,
                                const uint32_t* tab, const MontP& M, hipStream_t s) {
    dim3 grid((unsigned)((B + 255) / 256), (unsigned)a.n_vectors);
    if (mode == 0)
        hipLaunchKernelGGL((packed_reveal_exact_kernel<MM>), grid, dim3(256), 0, s, a.shares, B, a.dimension, a.out,
                           n_idx, k, tab, M);
    else
        hipLaunchKernelGGL((packed_reveal_canon_kernel<MM>), grid, dim3(256), 0, s, a.shares, B, a.dimension, a.out,
                           n_idx, k, tab, M);
    return hipGetLastError();
}

hipError_t launch_packed_reveal(const PackedRevealArgs& a, const uint64_t* indices, uint32_t n_idx, uint32_t k,
                                uint32_t p, uint32_t omega_secrets, uint32_t omega_shares, int mode,
                                DeviceTable& tab, hipStream_t s) {
    const uint64_t B = (a.dimension + k - 1) / k;
    if (B == 0 || a.n_vectors == 0) return hipSuccess;
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
    if (need <= 8) return reveal_launch<8>(mode, a, B, n_idx, k, dtab, M, s);
    if (need <= 16) return reveal_launch<16>(mode, a, B, n_idx, k, dtab, M, s);
    if (need <= 32) return reveal_launch<32>(mode, a, B, n_idx, k, dtab, M, s);
    if (need <= 64) return reveal_launch<64>(mode, a, B, n_idx, k, dtab, M, s);
    return hipErrorInvalidValue;
}

}  // namespace sda
