// packed_wide.hip -- packed-Shamir share generation and reveal past the register kernels' sizes:
// k + t + 1 up to kWideMaxL (> 64), n + 1 up to kWideMaxN3 (> 81), and reveals from more than
// kRevealMaxShares clerk shares (tss allows any power of 2 / power of 3, and batched.rs:75 reveals
// from every share it is given).
//
// Same arithmetic as the generic exact path of packed_gen.hip / packed_reveal.hip -- tss' recursive
// fft2_inverse / fft3 (packed::share) and Newton interpolation (packed::reconstruct), i64 wrapping
// products and Rust's truncated `%` after every operation -- so the results are tss' signed
// representatives for ANY i64 input, with no range precondition.  One lane = one batch, as in the
// register kernels, but the transform state ([L] + [n + 1] values, or the m Newton points) lives in a
// device workspace laid out [element][lane], so every access of a wave is one coalesced 512-byte
// row; a fixed grid of lanes walks the batches.  These sizes are outside the benchmark configs; the
// path exists so the engine's domain is tss' domain, not for speed.
#include "packed_common.h"

namespace sda {
using namespace packed;

namespace {

__device__ __forceinline__ uint32_t rev_bits_rt(uint32_t i, uint32_t nbits) {
    return nbits ? __builtin_bitreverse32(i) >> (32 - nbits) : 0u;
}
__device__ __forceinline__ uint32_t rev_trits_rt(uint32_t i, uint32_t ndig) {
    uint32_t r = 0;
    for (uint32_t d = 0; d < ndig; ++d) { r = r * 3 + i % 3; i /= 3; }
    return r;
}

// Device table of the wide share-gen (i64 words): tw2[L-1] (radix-2 level len: entries
// [len/2 - 1, len - 1)), linv, tw3[W3] and sq3[W3] (radix-3 level len: entries [(len-3)/2, (len-3)/2 +
// len)), W3 = (3 (n+1) - 3) / 2 -- the layout of GenTables without its size caps.
__global__ __launch_bounds__(256) void packed_gen_wide_kernel(const int64_t* __restrict__ secrets, uint64_t D,
                                                              const int64_t* __restrict__ draws,
                                                              int64_t* __restrict__ out, uint32_t k, uint32_t t,
                                                              uint64_t B, uint64_t n_vec, uint32_t L, uint32_t N3,
                                                              const int64_t* __restrict__ tab, int64_t p,
                                                              int64_t* __restrict__ ws, uint64_t lanes, int canonical) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= lanes) return;
    const Mod64 P = make_mod64(p);
    const uint32_t LB = (uint32_t)(31 - __builtin_clz(L)), ND = [&] { uint32_t d = 0; for (uint32_t x = N3; x > 1; x /= 3) ++d; return d; }();
    const int64_t* tw2 = tab;
    const int64_t linv = tab[L - 1];
    const uint64_t W3 = (3ull * N3 - 3) / 2;
    const int64_t* tw3 = tab + L;
    const int64_t* sq3 = tw3 + W3;
    int64_t* X = ws + gid;                          // X[e] = X[e * lanes]
    int64_t* Y = ws + (uint64_t)L * lanes + gid;
    auto x = [&](uint32_t e) -> int64_t& { return X[(uint64_t)e * lanes]; };
    auto y = [&](uint32_t e) -> int64_t& { return Y[(uint64_t)e * lanes]; };
    const uint64_t total = B * n_vec;
    for (uint64_t gb = gid; gb < total; gb += lanes) {
        const uint64_t vec = gb / B, b = gb - vec * B;
        const int64_t* sec = secrets + vec * D;
        // packed::share: values = [0, secrets (zero past D: batched.rs:37-43), randomness]
        for (uint32_t i = 0; i < L; ++i) {
            int64_t v = 0;
            if (i >= 1 && i <= k) {
                const uint64_t idx = b * k + (i - 1);
                v = idx < D ? sec[idx] : 0;
            } else if (i > k) {
                v = draws[gb * t + (i - 1 - k)];
            }
            x(rev_bits_rt(i, LB)) = v;
        }
        // fft2_inverse = fft2 over omega_secrets^-1: (u +- w c) % p per butterfly, bottom level first
        for (uint32_t len = 2; len <= L; len *= 2) {
            const uint32_t h = len / 2;
            for (uint32_t g = 0; g < L; g += len)
                for (uint32_t i = 0; i < h; ++i) {
                    const int64_t w = tw2[h - 1 + i];
                    const int64_t u = x(g + i), c = x(g + i + h);
                    x(g + i) = trem64(wadd(u, wmul(w, c)), P);
                    x(g + i + h) = trem64(wsub(u, wmul(w, c)), P);
                }
        }
        // x * len_inv % p, zero-extended to n + 1 coefficients in digit-reversed order
        for (uint32_t i = 0; i < N3; ++i) y(rev_trits_rt(i, ND)) = i < L ? trem64(wmul(x(i), linv), P) : 0;
        // fft3 over omega_shares: (b + x c + x^2 d) % p
        for (uint32_t len = 3; len <= N3; len *= 3) {
            const uint32_t th = len / 3, o = (len - 3) / 2;
            for (uint32_t g = 0; g < N3; g += len)
                for (uint32_t i = 0; i < th; ++i) {
                    const int64_t bb = y(g + i), cc = y(g + i + th), dd = y(g + i + 2 * th);
                    for (uint32_t q = 0; q < 3; ++q) {
                        const uint32_t j = i + q * th;
                        y(g + j) = trem64(wadd(wadd(bb, wmul(tw3[o + j], cc)), wmul(sq3[o + j], dd)), P);
                    }
                }
        }
        // shares = points[1..=n], clerk-major (batched.rs:46-48)
        int64_t* o = out + vec * (uint64_t)(N3 - 1) * B + b;
        for (uint32_t j = 1; j < N3; ++j) {
            const int64_t v = y(j);
            o[(uint64_t)(j - 1) * B] = canonical && v < 0 ? v + p : v;
        }
    }
}

// Wide reveal: tss' Newton divided differences over the m = n_idx + 1 points (the inserted (1, 0)
// first), then newton_evaluate at omega_secrets^(e+1).  inv[j m + i] = mod_inverse(points[i] -
// points[i-j]); np[e m + i] = the signed Newton basis at omega_secrets^(e+1) (as packed_reveal.hip's
// host tables, stride m).  CANONICAL: the exact value's canonical residue (= positive()).
__global__ __launch_bounds__(256) void packed_reveal_wide_kernel(const int64_t* __restrict__ shares, uint64_t B,
                                                                 uint64_t D, uint64_t n_vec, int64_t* __restrict__ out,
                                                                 uint32_t n_idx, uint32_t k,
                                                                 const int64_t* __restrict__ inv,
                                                                 const int64_t* __restrict__ np, int64_t p,
                                                                 int64_t* __restrict__ ws, uint64_t lanes, int canonical) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= lanes) return;
    const Mod64 P = make_mod64(p);
    const uint32_t m = n_idx + 1;
    int64_t* S = ws + gid;
    auto s = [&](uint32_t e) -> int64_t& { return S[(uint64_t)e * lanes]; };
    const uint64_t total = B * n_vec;
    for (uint64_t gb = gid; gb < total; gb += lanes) {
        const uint64_t vec = gb / B, b = gb - vec * B;
        const int64_t* sh = shares + vec * (uint64_t)n_idx * B + b;
        s(0) = 0;
        for (uint32_t i = 1; i < m; ++i) s(i) = sh[(uint64_t)(i - 1) * B];     // batched.rs:83-85
        for (uint32_t j = 1; j < m; ++j) {
            const int64_t* invj = inv + (uint64_t)j * m;
            int64_t hi = s(m - 1);                       // s[i] of this level, walking i downwards
            for (uint32_t i = m - 1; i >= j; --i) {
                const int64_t lo = s(i - 1);
                s(i) = trem64(wmul(trem64(wsub(hi, lo), P), invj[i]), P);
                hi = lo;
            }
        }
        const uint64_t base = b * k;
        for (uint32_t e = 0; e < k && base + e < D; ++e) {
            const int64_t* npe = np + (uint64_t)e * m;
            int64_t acc = 0;
            for (uint32_t i = 0; i < m; ++i) acc = trem64(wadd(acc, trem64(wmul(s(i), npe[i]), P)), P);
            out[vec * D + base + e] = canonical && acc < 0 ? acc + p : acc;     // batched.rs:94
        }
    }
}

// Lanes in flight: enough to fill the chip, few enough that the workspace stays <= ~256 MiB.
uint64_t wide_lanes(uint64_t total, uint64_t words_per_lane) {
    uint64_t cap = (256ull << 20) / (8 * words_per_lane);
    cap = cap < 4096 ? 4096 : (cap > 65536 ? 65536 : cap);
    cap = (cap + 255) / 256 * 256;
    const uint64_t want = (total + 255) / 256 * 256;
    return want < cap ? want : cap;
}

hipError_t ensure_ws(DeviceTable& t, size_t bytes) {
    if (bytes <= t.ws_cap && t.ws) return hipSuccess;
    hipError_t e;
    if ((e = hipDeviceSynchronize()) != hipSuccess) return e;    // earlier launches may still use it
    if (t.ws) (void)hipFree(t.ws);
    t.ws = nullptr;
    t.ws_cap = 0;
    if ((e = hipMalloc(&t.ws, bytes)) != hipSuccess) return e;
    t.ws_cap = bytes;
    return hipSuccess;
}

}  // namespace

hipError_t launch_packed_generate_wide(const PackedGenArgs& a, uint32_t k, uint32_t t, uint32_t n, uint32_t p,
                                       uint32_t omega_secrets, uint32_t omega_shares, DeviceTable& tab,
                                       hipStream_t s) {
    const uint32_t L = k + t + 1, N3 = n + 1;
    const uint64_t B = (a.dimension + k - 1) / k;
    if (B == 0 || a.n_vectors == 0) return hipSuccess;
    const uint64_t W3 = (3ull * N3 - 3) / 2;
    const uint32_t kv[6] = {0x57494445u /* wide */, L, N3, p, omega_secrets, omega_shares};
    std::vector<uint8_t> key((const uint8_t*)kv, (const uint8_t*)kv + sizeof(kv));
    if (tab.key != key) {
        // the twiddles of make_gen_tables, any L / N3
        std::vector<int64_t> h(L + 2 * W3, 0);
        const int64_t P = p;
        const int64_t winv = h_modinv(omega_secrets, P);
        h[L - 1] = h_modinv((int64_t)L, P);
        std::vector<int64_t> lv;
        int64_t om = winv;
        for (uint32_t len = L; len >= 2; len /= 2) { lv.push_back(om); om = h_powmod(om, 2, P); }
        int lvl = (int)lv.size() - 1;
        for (uint32_t len = 2; len <= L; len *= 2, --lvl)
            for (uint32_t i = 0; i < len / 2; ++i) h[len / 2 - 1 + i] = h_powmod(lv[lvl], i, P);
        lv.clear();
        om = omega_shares;
        for (uint32_t len = N3; len >= 3; len /= 3) { lv.push_back(om); om = h_powmod(om, 3, P); }
        lvl = (int)lv.size() - 1;
        for (uint32_t len = 3; len <= N3; len *= 3, --lvl)
            for (uint32_t j = 0; j < len; ++j) {
                const int64_t x = h_powmod(lv[lvl], j, P);
                h[L + (len - 3) / 2 + j] = x;
                h[L + W3 + (len - 3) / 2 + j] = h_rem(x * x, P);
            }
        hipError_t e = ensure_table(tab, key, h.data(), h.size() * sizeof(int64_t));
        if (e != hipSuccess) return e;
    }
    const uint64_t lanes = wide_lanes(B * a.n_vectors, (uint64_t)L + N3);
    hipError_t e = ensure_ws(tab, lanes * ((uint64_t)L + N3) * sizeof(int64_t));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(packed_gen_wide_kernel, dim3((unsigned)(lanes / 256)), dim3(256), 0, s, a.secrets, a.dimension,
                       a.draws, a.out, k, t, B, a.n_vectors, L, N3, static_cast<const int64_t*>(tab.dev), (int64_t)p,
                       static_cast<int64_t*>(tab.ws), lanes, a.canonical ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_packed_reveal_wide(const PackedRevealArgs& a, const uint64_t* indices, uint32_t n_idx, uint32_t k,
                                     uint32_t p, uint32_t omega_secrets, uint32_t omega_shares, int mode,
                                     DeviceTable& tab, hipStream_t s) {
    const uint64_t B = (a.dimension + k - 1) / k;
    if (B == 0 || a.n_vectors == 0) return hipSuccess;
    const uint32_t m = n_idx + 1;
    const int64_t P = p;
    // mode is part of the key: a CANONICAL call must see the duplicate-point refusal below even when an
    // EXACT call already built the table for the same clerk set
    std::vector<uint8_t> key(sizeof(uint32_t) * 7 + sizeof(uint64_t) * n_idx);
    const uint32_t kv[7] = {0x57494445u /* wide */, n_idx, k, p, omega_secrets, omega_shares, (uint32_t)mode};
    memcpy(key.data(), kv, sizeof(kv));
    memcpy(key.data() + sizeof(kv), indices, sizeof(uint64_t) * n_idx);
    if (tab.key != key) {
        // packed_reveal.hip's host tables (same ops as tss), stride m: inv [m][m], np [k][m]
        std::vector<int64_t> h((uint64_t)m * m + (uint64_t)k * m, 0);
        std::vector<int64_t> pts(m);
        pts[0] = 1;                                                    // points.insert(0, 1)
        for (uint32_t i = 0; i < n_idx; ++i) pts[i + 1] = h_powmod(omega_shares, (uint32_t)(indices[i] + 1), P);
        bool dup = false;
        for (uint32_t j = 1; j < m; ++j)
            for (uint32_t i = j; i < m; ++i) h[(uint64_t)j * m + i] = h_modinv(h_rem(pts[i] - pts[i - j], P), P);
        for (uint32_t x = 0; x < m && !dup; ++x)
            for (uint32_t y = x + 1; y < m; ++y)
                if (pts[x] == pts[y]) { dup = true; break; }
        if (mode == 1 && dup) return hipErrorInvalidValue;            // as the Lagrange table refuses them
        int64_t* np = h.data() + (uint64_t)m * m;
        for (uint32_t e = 0; e < k; ++e) {
            const int64_t point = h_powmod(omega_secrets, e + 1, P);
            int64_t v = 1;
            for (uint32_t i = 0; i < m; ++i) {
                np[(uint64_t)e * m + i] = v;
                if (i + 1 < m) v = h_rem(v * h_rem(point - pts[i], P), P);
            }
        }
        hipError_t e = ensure_table(tab, key, h.data(), h.size() * sizeof(int64_t));
        if (e != hipSuccess) return e;
    }
    const uint64_t lanes = wide_lanes(B * a.n_vectors, m);
    hipError_t e = ensure_ws(tab, lanes * (uint64_t)m * sizeof(int64_t));
    if (e != hipSuccess) return e;
    const int64_t* inv = static_cast<const int64_t*>(tab.dev);
    hipLaunchKernelGGL(packed_reveal_wide_kernel, dim3((unsigned)(lanes / 256)), dim3(256), 0, s, a.shares, B,
                       a.dimension, a.n_vectors, a.out, n_idx, k, inv, inv + (uint64_t)m * m, P,
                       static_cast<int64_t*>(tab.ws), lanes, mode == 1 ? 1 : 0);
    return hipGetLastError();
}

}  // namespace sda
