// packed_gen.hip -- packed-Shamir share generation (see packed_common.h for the algorithm).
#include "packed_common.h"

namespace sda {
using namespace packed;

namespace {

// ---------------- generic exact share (inputs outside (-p, p)) ----------------
// Reads its inputs from global memory (nothing escapes from the fast path's registers).
__device__ __noinline__ void packed_share_generic(const int64_t* __restrict__ sec, uint64_t D,
                                                  const int64_t* __restrict__ drw, uint64_t b, uint32_t k,
                                                  int L, int N3, const GenTables& T, int64_t* o, uint64_t B) {
    const Mod64 P = make_mod64((int64_t)T.M.p);
    int64_t x[64];
    const int lb = ilog(L, 2);
    for (int i = 0; i < L; ++i) {
        int r = 0, v = i;
        for (int d = 0; d < lb; ++d) { r = r * 2 + v % 2; v /= 2; }
        int64_t val = 0;
        if (i >= 1 && (uint32_t)i <= k) { const uint64_t idx = b * k + (i - 1); val = idx < D ? sec[idx] : 0; }
        else if (i > 0) val = drw[i - 1 - k];
        x[r] = val;
    }
    for (int len = 2; len <= L; len *= 2) {
        const int h = len / 2;
        for (int g = 0; g < L; g += len)
            for (int i = 0; i < h; ++i) {
                const int64_t w = T.tw2[h - 1 + i];
                const int64_t u = x[g + i], c = x[g + i + h];
                x[g + i] = trem64(wadd(u, wmul(w, c)), P);
                x[g + i + h] = trem64(wsub(u, wmul(w, c)), P);
            }
    }
    for (int i = 0; i < L; ++i) x[i] = trem64(wmul(x[i], T.linv), P);
    int64_t y[81];
    const int nd = ilog(N3, 3);
    for (int i = 0; i < N3; ++i) {
        int r = 0, v = i;
        for (int d = 0; d < nd; ++d) { r = r * 3 + v % 3; v /= 3; }
        y[r] = i < L ? x[i] : 0;
    }
    for (int len = 3; len <= N3; len *= 3) {
        const int th = len / 3, o = (len - 3) / 2;
        for (int g = 0; g < N3; g += len)
            for (int i = 0; i < th; ++i) {
                const int64_t b = y[g + i], c = y[g + i + th], d = y[g + i + 2 * th];
                for (int q = 0; q < 3; ++q) {
                    const int j = i + q * th;
                    y[g + j] = trem64(wadd(wadd(b, wmul(T.tw3[o + j], c)), wmul(T.sq3[o + j], d)), P);
                }
            }
    }
    for (int j = 1; j < N3; ++j) o[(uint64_t)(j - 1) * B] = y[j];
}

// radix-2 butterfly on exact representatives in (-p, p):  (u ± w c) % p
__device__ __forceinline__ void bfly2(int32_t& u, int32_t& c, uint32_t w, uint32_t w_m, const MontP& M) {
    // exact product, |t| < p^2; w < p < 2^31 so a signed 32x32 multiply is exact (one v_mad_i64_i32)
    const int64_t t = (int64_t)(int32_t)w * (int64_t)c;
    const uint32_t tc = mont_mul(w_m, canon32(c, M.p), M);     // t mod p (canonical)
    const uint32_t U = canon32(u, M.p);
    const uint32_t c1 = addmod(U, tc, M.p), c2 = submod(U, tc, M.p);
    const int64_t v1 = (int64_t)u + t, v2 = (int64_t)u - t;    // exact dividends
    u = trunc_from(c1, v1 < 0, M.p);
    c = trunc_from(c2, v2 < 0, M.p);
}

// twiddle index 0 is omega^0 = 1 at every level: (u + c) % p, (u - c) % p, no product
__device__ __forceinline__ void bfly2_unit(int32_t& u, int32_t& c, const MontP& M) {
    const uint32_t U = canon32(u, M.p), C = canon32(c, M.p);
    const uint32_t c1 = addmod(U, C, M.p), c2 = submod(U, C, M.p);
    const int64_t v1 = (int64_t)u + c, v2 = (int64_t)u - c;
    u = trunc_from(c1, v1 < 0, M.p);
    c = trunc_from(c2, v2 < 0, M.p);
}

template <int L, int N3>
__global__ __launch_bounds__(256) void packed_gen_kernel(const int64_t* __restrict__ secrets, uint64_t D,
                                                         const int64_t* __restrict__ draws,
                                                         int64_t* __restrict__ out, uint32_t k, uint32_t t,
                                                         uint64_t B, const GenTables* __restrict__ Tp) {
    const GenTables& T = *Tp;          // global memory: uniform => scalar loads, no per-lane copy
    constexpr int LB = ilog(L, 2);
    constexpr int ND = ilog(N3, 3);
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint64_t vec = blockIdx.y;
    const int64_t* sec = secrets + vec * D;
    const int64_t* drw = draws + (vec * B + b) * t;
    const uint32_t p = T.M.p;
    const int64_t P = (int64_t)p;

    // values = [0, secrets, randomness]; batched.rs:37-43 zero-pads the tail batch
    int64_t raw[L];
    raw[0] = 0;
    bool in_range = true;
    static_for<1, L>([&](auto i) {
        int64_t v;
        if ((uint32_t)i <= k) {
            const uint64_t idx = b * k + (i - 1);
            v = idx < D ? sec[idx] : 0;
        } else {
            v = drw[i - 1 - k];
        }
        raw[i] = v;
        in_range = in_range && (v > -P) && (v < P);
    });

    int64_t* o = out + vec * (uint64_t)(N3 - 1) * B + b;
    if (!in_range) {
        packed_share_generic(sec, D, drw, b, k, L, N3, T, o, B);
        return;
    }

    // ---- fft2_inverse: radix-2 DIT over omega_secrets^-1 on bit-reversed registers ----
    int32_t x[L];
    static_for<0, L>([&](auto i) { x[rev_digits(i, 2, LB)] = (int32_t)raw[i]; });
    static_for<1, LB + 1>([&](auto s) {
        constexpr int H = 1 << (s - 1), LEN = 2 * H;
        static_for<0, L, LEN>([&](auto g) {
            static_for<0, H>([&](auto i) {
                if constexpr (i == 0) bfly2_unit(x[g], x[g + H], T.M);
                else bfly2(x[g + i], x[g + i + H], T.tw2[H - 1 + i], T.tw2_m[H - 1 + i], T.M);
            });
        });
    });
    // x * len_inv % p   (len_inv > 0 => sign of x)
    static_for<0, L>([&](auto i) { x[i] = trunc_from(mont_mul(T.linv_m, canon32(x[i], p), T.M), x[i] < 0, p); });

    // ---- fft3: radix-3 DIT over omega_shares on digit-reversed, zero-extended registers ----
    int32_t y[N3];
    static_for<0, N3>([&](auto i) { y[rev_digits(i, 3, ND)] = i < L ? x[i < L ? (int)i : 0] : 0; });
    static_for<1, ND + 1>([&](auto s) {
        constexpr int th = ipow(3, s - 1);
        constexpr int LEN = 3 * th, OB = (LEN - 3) / 2;
        static_for<0, N3, LEN>([&](auto g) {
            static_for<0, th>([&](auto i) {
                const int32_t bb = y[g + i], cc = y[g + i + th], dd = y[g + i + 2 * th];
                const uint32_t Bc = canon32(bb, p), Cc = canon32(cc, p), Dc = canon32(dd, p);
                int32_t r[3];
                static_for<0, 3>([&](auto q) {
                    constexpr int j = i + q * th;
                    if constexpr (j == 0) {
                        // x = x^2 = 1: (b + c + d) % p
                        const int64_t v = (int64_t)bb + cc + dd;
                        r[q] = trunc_from(addmod(addmod(Bc, Cc, p), Dc, p), v < 0, p);
                    } else {
                        // twiddles < p < 2^31: signed 32x32 products are exact (v_mad_i64_i32)
                        const int32_t xw = (int32_t)T.tw3[OB + j], x2 = (int32_t)T.sq3[OB + j];
                        // exact dividend b + x*c + x^2*d   (|.| < p + 2 p^2 < 2^63)
                        const int64_t v = (int64_t)bb + (int64_t)xw * cc + (int64_t)x2 * dd;
                        // canonical residue: REDC(x' C + x2' D) + B    (x' C + x2' D < 2 p^2 < p R)
                        const uint64_t acc = (uint64_t)T.tw3_m[OB + j] * Cc + (uint64_t)T.sq3_m[OB + j] * Dc;
                        r[q] = trunc_from(addmod(Bc, redc(acc, T.M), p), v < 0, p);
                    }
                });
                y[g + i] = r[0]; y[g + i + th] = r[1]; y[g + i + 2 * th] = r[2];
            });
        });
    });
    // shares = points[1..=n], clerk-major (batched.rs:46-48)
    static_for<1, N3>([&](auto j) { o[(uint64_t)(j - 1) * B] = (int64_t)y[j]; });
}

}  // namespace

template <int L, int N3>
static hipError_t gen_launch(const PackedGenArgs& a, uint32_t k, uint32_t t, uint64_t B, const GenTables* T,
                             hipStream_t s) {
    dim3 grid((unsigned)((B + 255) / 256), (unsigned)a.n_vectors);
    hipLaunchKernelGGL((packed_gen_kernel<L, N3>), grid, dim3(256), 0, s, a.secrets, a.dimension, a.draws, a.out,
                       k, t, B, T);
    return hipGetLastError();
}

template <int N3>
static hipError_t gen_dispatch_L(uint32_t L, const PackedGenArgs& a, uint32_t k, uint32_t t, uint64_t B,
                                 const GenTables* T, hipStream_t s) {
    switch (L) {
        case 2: return gen_launch<2, N3>(a, k, t, B, T, s);
        case 4: if constexpr (N3 >= 4) return gen_launch<4, N3>(a, k, t, B, T, s); break;
        case 8: if constexpr (N3 >= 8) return gen_launch<8, N3>(a, k, t, B, T, s); break;
        case 16: if constexpr (N3 >= 16) return gen_launch<16, N3>(a, k, t, B, T, s); break;
        case 32: if constexpr (N3 >= 32) return gen_launch<32, N3>(a, k, t, B, T, s); break;
        case 64: if constexpr (N3 >= 64) return gen_launch<64, N3>(a, k, t, B, T, s); break;
    }
    return hipErrorInvalidValue;
}

hipError_t launch_packed_generate(const PackedGenArgs& a, uint32_t k, uint32_t t, uint32_t n, uint32_t p,
                                  uint32_t omega_secrets, uint32_t omega_shares, DeviceTable& tab, hipStream_t s) {
    const uint32_t L = k + t + 1, N3 = n + 1;
    const uint64_t B = (a.dimension + k - 1) / k;
    if (B == 0 || a.n_vectors == 0) return hipSuccess;
    const uint32_t kv[5] = {L, N3, p, omega_secrets, omega_shares};
    std::vector<uint8_t> key((const uint8_t*)kv, (const uint8_t*)kv + sizeof(kv));
    if (tab.key != key) {
        const GenTables T = make_gen_tables(L, N3, p, omega_secrets, omega_shares);
        hipError_t e = ensure_table(tab, key, &T, sizeof(T));
        if (e != hipSuccess) return e;
    }
    const GenTables* T = static_cast<const GenTables*>(tab.dev);
    switch (N3) {
        case 3: return gen_dispatch_L<3>(L, a, k, t, B, T, s);
        case 9: return gen_dispatch_L<9>(L, a, k, t, B, T, s);
        case 27: return gen_dispatch_L<27>(L, a, k, t, B, T, s);
        case 81: return gen_dispatch_L<81>(L, a, k, t, B, T, s);
    }
    return hipErrorInvalidValue;
}

hipError_t ensure_table(DeviceTable& t, const std::vector<uint8_t>& key, const void* host, size_t bytes) {
    if (t.key == key && t.dev) return hipSuccess;
    hipError_t e;
    // earlier launches may still read the old contents
    if ((e = hipDeviceSynchronize()) != hipSuccess) return e;
    if (bytes > t.cap) {
        if (t.dev) (void)hipFree(t.dev);
        t.dev = nullptr;
        t.cap = 0;
        if ((e = hipMalloc(&t.dev, bytes)) != hipSuccess) return e;
        t.cap = bytes;
    }
    if ((e = hipMemcpy(t.dev, host, bytes, hipMemcpyHostToDevice)) != hipSuccess) return e;
    t.key = key;
    return hipSuccess;
}

void free_table(DeviceTable& t) {
    if (t.dev) (void)hipFree(t.dev);
    t.dev = nullptr;
    t.cap = 0;
    t.key.clear();
}

}  // namespace sda
