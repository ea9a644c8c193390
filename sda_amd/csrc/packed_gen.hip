// packed_gen.hip -- packed-Shamir share generation (see packed_common.h for the algorithm).
#include <stdlib.h>

#include "packed_common.h"
#include "xcd.h"

namespace sda {
using namespace packed;

// One launcher per (L = k+t+1, N3 = n+1); each is compiled in its own object (Makefile:
// -DSDA_GEN_PART=N3 -DSDA_GEN_L=L) so the instantiations build in parallel.
template <int L, int N3>
hipError_t gen_launch(const PackedGenArgs& a, uint32_t k, uint32_t t, uint64_t B, const GenTables* T,
                      const GenFixupLog& log, hipStream_t s);

// Which schemes the register kernels serve (the rest run packed_wide.hip's workspace kernels).  At n + 1 = 81
// the exact kernel without lazy truncation (p < 2^24, or odd B) needs its 64-bit sign products on top of 81
// (sign, residue) pairs: at L >= 16 that is more than the 256 VGPRs of a wave (round 5: 335-512 registers at
// L >= 32, 79-256 of them AGPRs used as VGPR overflow, scratch at L = 64 -- the class of kernel that faulted in
// rounds 4 and 5; 46-74 VGPRs spilled at L = 16 even with 256).  DESIGN.md §4.2, "Register budget at
// n + 1 = 81"; tests/test_kernel_resources.py checks every shipped code object.
constexpr bool gen_register_path(uint32_t L, uint32_t N3, bool exact_nonlazy) {
    return L <= 64 && N3 <= 81 && !(N3 == 81 && L >= 16 && exact_nonlazy);
}

#ifdef SDA_GEN_PART
namespace {

// A field element on the fast path: tss' exact representative s in (-p, p) and its canonical
// residue c in [0, p).  Carrying both saves re-canonicalising every operand at every stage.
struct FE {
    int32_t s;
    uint32_t c;
};

// radix-2 butterfly (u ± w c) % p.  The signs come from the exact i64 dividends (one
// v_mad_i64_i32 each), the residues from one lazy Montgomery product shared by both outputs.

template <class TR>
__device__ __forceinline__ void bfly2(FE& u, FE& c, int32_t w, int32_t nw, uint32_t w_m, const MontP& M, TR& tr) {
    const int64_t v1 = (int64_t)u.s + (int64_t)w * c.s;
    const int64_t v2 = (int64_t)u.s + (int64_t)nw * c.s;
    const uint32_t tc = montu<TR::lazy>(w_m, c.c, M);
    const uint32_t c1 = addm(u.c, tc, M.p), c2 = subm(u.c, tc, M.p);
    u = FE{tr(c1, hi32(v1), M.p), c1};
    c = FE{tr(c2, hi32(v2), M.p), c2};
    tr.note2(u.s, c.s);
}

// twiddle omega^0 = 1: (u + c) % p, (u - c) % p.  A saturating add keeps the exact sum's sign.
template <class TR>
__device__ __forceinline__ void bfly2_unit(FE& u, FE& c, uint32_t p, TR& tr) {
    const uint32_t c1 = addm(u.c, c.c, p), c2 = subm(u.c, c.c, p);
    const int32_t s1 = __builtin_elementwise_add_sat(u.s, c.s), s2 = __builtin_elementwise_sub_sat(u.s, c.s);
    u = FE{tr(c1, (uint32_t)s1, p), c1};
    c = FE{tr(c2, (uint32_t)s2, p), c2};
    tr.note2(u.s, c.s);
}

// SIGNBIT (lazy exact kernel): the radix-2 half of the transform on (residue c, sign word n) pairs,
// value = c - p [n < 0] -- the reveal's sign-bit formulation carried to share-gen:
//   unit butterfly   (u + c) % p: sign MAJ(n_u, n_c, [c_u + c_c < p]);  (u - c) % p: MAJ(n_u, ~n_c, [c_u < c_c])
//   twiddle w != 1   (u +- w c) % p: the exact product dominates |u| < p whenever |w c| >= p, so the
//                    signs are n_c and ~n_c -- no 64-bit sign products, no truncation ops;
//   x * len_inv % p  keeps the sign of x (len_inv > 0).
// Exact unless a butterfly output's residue is 0 (it might then carry the sign of a nonzero multiple of
// p, which tss truncates to 0) or a multiplied operand is small, |c| < ceil(p / w).  RangeTrap keeps a
// running min of the output residues and a running max of the shifted multiplied ones (two values per
// v_min3 / v_max3); such batches (probability ~ 1/p per output, ~ 2 big2 / p per product: ~1e-8 at
// configs[2]) go to the generic fix-up kernel like the lazy truncation's -p trap.
struct RangeTrap {
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    uint32_t lpend = 0, hpend = 0;
    bool lhas = false, hhas = false;      // constant at every point of the unrolled code
    __device__ __forceinline__ void lo2(uint32_t a, uint32_t b) { asm("v_min3_u32 %0, %0, %1, %2" : "+v"(lo) : "v"(a), "v"(b)); }
    __device__ __forceinline__ void hi2(uint32_t a, uint32_t b) { asm("v_max3_u32 %0, %0, %1, %2" : "+v"(hi) : "v"(a), "v"(b)); }
    // a butterfly output's residue: 0 is the trap (0 with the sign set would be a nonzero multiple of p)
    __device__ __forceinline__ void out1(uint32_t c) {
        if (lhas) { lo2(lpend, c); lhas = false; } else { lpend = c; lhas = true; }
    }
    // a multiplied operand's residue c must lie in [big, p - big]: c - big (wrapping below big) <= p - 2 big
    __device__ __forceinline__ void mul1(uint32_t c, uint32_t big) {
        const uint32_t x = c - big;
        if (hhas) { hi2(hpend, x); hhas = false; } else { hpend = x; hhas = true; }
    }
    __device__ __forceinline__ bool bad(uint32_t big, uint32_t p) {
        if (lhas) lo2(lpend, lpend);
        if (hhas) hi2(hpend, hpend);
        lhas = hhas = false;
        return lo == 0 || hi > p - 2 * big;
    }
};

// Compile-time map of the radix-3 registers that hold a known zero (the zero padding of
// coefficients L..N3-1) after `stage` levels: a group whose c and d are zero just copies b.
template <int L, int N3>
struct Zero3 {
    static constexpr int ND = ilog(N3, 3);
    static constexpr bool is_zero(int stage, int pos) {
        if (stage == 0) return rev_digits(pos, 3, ND) >= L;
        const int th = ipow(3, stage - 1), len = 3 * th;
        const int g = pos - pos % len, i = (pos % len) % th;
        return is_zero(stage - 1, g + i) && is_zero(stage - 1, g + i + th) && is_zero(stage - 1, g + i + 2 * th);
    }
};

// Streaming policy of the tile loads / share stores (A/B knobs; default: non-temporal both ways).
#ifndef SDA_GEN_NT_LOAD
#define SDA_GEN_NT_LOAD 1
#endif
#ifndef SDA_GEN_NT_STORE
#define SDA_GEN_NT_STORE 1
#endif
__device__ __forceinline__ int64_t gen_load(const int64_t* a) {
    if constexpr (SDA_GEN_NT_LOAD) return __builtin_nontemporal_load(a);
    else return *a;
}
template <class V>
__device__ __forceinline__ void gen_store(const V& v, V* a) {
    if constexpr (SDA_GEN_NT_STORE) __builtin_nontemporal_store(v, a);
    else *a = v;
}

// Workgroup size: 256 batches, fewer for the wide transforms so the LDS stage stays <= 32 KiB.
template <int L>
constexpr int gen_block() { return L <= 16 ? 256 : (L == 32 ? 128 : 64); }

#ifndef SDA_GEN_FULLTILE
#define SDA_GEN_FULLTILE 1
#endif
#ifndef SDA_GEN_WAVES
#define SDA_GEN_WAVES 4
#endif
// Wave priorities by phase (s_setprio) in the exact kernel: SDA_GEN_PRIO_LOAD while a wave issues its tile
// loads, 0 during the transform, SDA_GEN_PRIO_STORE for its share stores -- so the memory phases of a CU's
// waves are not starved by the other waves' VALU streams.  Exact share-gen 7.18-7.20 -> 7.01-7.02 ms and
// 7.36 -> 7.19-7.21 ms and 7.14-7.16 -> 6.97-7.08 ms on three boxes (3 interleaved rounds each, profiles/r05o,
// r05p, r05q; dropping to 0 after the LDS reads, or levels 2/1, measured the same); the canonical kernel,
// memory-bound, got 1.5 % slower with it and runs without; so did the exact reveal.  SDA_GEN_PRIO = 0 turns it
// off (A/B knob).
#ifndef SDA_GEN_PRIO
#define SDA_GEN_PRIO 1
#endif
#ifndef SDA_GEN_PRIO_LOAD
#define SDA_GEN_PRIO_LOAD 3
#endif
#ifndef SDA_GEN_PRIO_STORE
#define SDA_GEN_PRIO_STORE 2
#endif
// Tile inputs staged by LDS DMA (global_load_lds_dwordx4) instead of loads into registers + ds_write:
// share-gen 7.01-7.02 -> 6.96-6.99 ms exact, 6.52-6.56 -> 6.44-6.48 ms canonical (profiles/r05u).  On in every
// object since round 6 ("LDS-DMA staging"); SDA_GEN_DMA = 0 is the A/B knob.
#ifndef SDA_GEN_DMA_AUX
#define SDA_GEN_DMA_AUX 2    // the DMA loads are nontemporal (exact share-gen -1.0 %, profiles/r06aj); 0 = cached (A/B)
#endif
#ifndef SDA_GEN_DMA
#define SDA_GEN_DMA 1
#endif
template <int LEVEL>
__device__ __forceinline__ void set_prio() {
    if constexpr (SDA_GEN_PRIO) __builtin_amdgcn_s_setprio(LEVEL);
}

// Waves per EU: 5 where the transform fits 102 VGPRs without spilling (canonical and lazy-exact at
// L <= 16), else SDA_GEN_WAVES (4: 128 VGPRs).  n + 1 = 81 keeps 81 shares in registers (162 VGPRs for the
// exact kernels' (sign, residue) pairs): 2 waves, 256 VGPRs, so no instantiation spills (round 5 ran them at
// 4-5 waves with up to 1.1 KiB of scratch per lane).
template <int L, int N3, bool CANON, bool LAZY>
constexpr int gen_waves() {
    return N3 >= 81 ? 2 : (L <= 16 && (CANON || LAZY)) ? 5 : SDA_GEN_WAVES;
}


// CANONICAL share generation: the same transform in canonical residues [0, p) only -- no sign
// tracking.  Each share equals tss' (signed) share mod p, so everything downstream (combine,
// reveal, unmask, RecipientOutput::positive) ends in the same canonical output when the masking
// modulus is the sharing prime.  Radix-3 groups use omega_3 = omega_len^(len/3):
// with C = x c, D = x^2 d:  y0 = b + C + D,  y1 = b - D + w3 (C - D),  y2 = b - C - w3 (C - D)
// -- 3 Montgomery products per 3 outputs instead of 6.
template <int L, int N3>
__device__ __forceinline__ void transform_canon(const int64_t (&raw)[L], const GenTables& T, const MontP& M,
                                                int32_t (&ys)[N3]) {
    constexpr int LB = ilog(L, 2);
    constexpr int ND = ilog(N3, 3);
    using Z = Zero3<L, N3>;
    const uint32_t p = M.p;
    auto mont = [&](uint32_t a_m, uint32_t x) { return red1(redc_lazy((uint64_t)a_m * x, M), p); };
    uint32_t x[L];
    static_for<0, L>([&](auto i) { x[rev_digits(i, 2, LB)] = canon32((int32_t)raw[i], p); });
    static_for<1, LB + 1>([&](auto s) {
        constexpr int H = 1 << (s - 1), LEN = 2 * H;
        static_for<0, L, LEN>([&](auto g) {
            static_for<0, H>([&](auto i) {
                const uint32_t u = x[g + i];
                const uint32_t c = (i == 0) ? x[g + i + H] : mont(T.tw2_m[H - 1 + i], x[g + i + H]);
                x[g + i] = addm(u, c, p);
                x[g + i + H] = subm(u, c, p);
            });
        });
    });
    static_for<0, L>([&](auto i) { x[i] = mont(T.linv_m, x[i]); });
    uint32_t y[N3];
    static_for<0, N3>([&](auto i) {
        if constexpr (i < L) y[rev_digits(i, 3, ND)] = x[i < L ? (int)i : 0];
        else y[rev_digits(i, 3, ND)] = 0u;
    });
    const uint32_t w3 = T.tw3_m[1];                      // omega_3 (stage len 3, j = 1), Montgomery form
    static_for<1, ND + 1>([&](auto s) {
        constexpr int th = ipow(3, s - 1);
        constexpr int LEN = 3 * th, OB = (LEN - 3) / 2;
        static_for<0, N3, LEN>([&](auto g) {
            static_for<0, th>([&](auto i) {
                constexpr bool zc = Z::is_zero(s - 1, g + i + th), zd = Z::is_zero(s - 1, g + i + 2 * th);
                if constexpr (zc && zd) {
                    y[g + i + th] = y[g + i];
                    y[g + i + 2 * th] = y[g + i];
                } else {
                    const uint32_t bb = y[g + i];
                    const uint32_t C = (i == 0) ? y[g + i + th] : mont(T.tw3_m[OB + i], y[g + i + th]);
                    if constexpr (zd) {
                        const uint32_t E = mont(w3, C);
                        y[g + i] = addm(bb, C, p);
                        y[g + i + th] = addm(bb, E, p);
                        y[g + i + 2 * th] = subm(subm(bb, C, p), E, p);
                    } else {
                        const uint32_t Dd = (i == 0) ? y[g + i + 2 * th] : mont(T.tw3_m[OB + (2 * i) % LEN], y[g + i + 2 * th]);
                        const uint32_t E = mont(w3, subm(C, Dd, p));
                        y[g + i] = addm(addm(bb, C, p), Dd, p);
                        y[g + i + th] = addm(subm(bb, Dd, p), E, p);
                        y[g + i + 2 * th] = subm(subm(bb, C, p), E, p);
                    }
                }
            });
        });
    });
    static_for<0, N3>([&](auto j) { ys[j] = (int32_t)y[j]; });
}

// One workgroup = one tile: vector lin / gridDim.x, BS batches from (lin % gridDim.x) * BS, where lin is
// the XCD-chunked linear workgroup id (xcd.h).
//
// Lane -> batch map: lane i < 32 takes batch 2i of its wave's 64, lane 32 + i batch 2i + 1.  After
// the transform one v_permlane32_swap per pair of clerk rows leaves lane i holding batches
// (2i, 2i+1) of row j and lane 32 + i the same batches of row j + 1: one 16-byte store per lane
// per row pair (13 dwordx4 instead of 26 dwordx2 at n = 26) when WIDE (B even, 16-B aligned out).
// (A persistent grid-stride variant was measured slower: the loop made hipcc keep the twiddle
// words in SGPRs across tiles and spill.)
template <int L, int N3, bool WIDE, bool CANON, bool LAZY, bool SIGNBIT = false>
__global__ __launch_bounds__(gen_block<L>())
__attribute__((amdgpu_waves_per_eu(gen_waves<L, N3, CANON, LAZY>(), gen_waves<L, N3, CANON, LAZY>())))
void packed_gen_kernel(const int64_t* __restrict__ secrets, uint64_t D, const int64_t* __restrict__ draws,
                       int64_t* __restrict__ out, uint32_t k, uint32_t t, uint64_t B,
                       const GenTables* __restrict__ Tp, unsigned int* __restrict__ log, int xcd) {
    constexpr int LB = ilog(L, 2);
    constexpr int ND = ilog(N3, 3);
    constexpr int BS = gen_block<L>();
    constexpr int NR = N3 - 1;         // share rows (clerks); N3 = 3^ND so NR is even
    using Z = Zero3<L, N3>;
    const uint32_t tid = threadIdx.x;
    if constexpr (!CANON) set_prio<SDA_GEN_PRIO_LOAD>();
    const uint32_t lane = tid & 63, half = lane >> 5;
    const uint32_t lb = (tid & ~63u) + 2 * (lane & 31) + half;       // this lane's batch in the tile
    const uint32_t pb_off = (tid & ~63u) + 2 * (lane & 31);          // first batch of its store pair
    const MontP M = Tp->M;
    const uint32_t p = M.p;
    const int64_t P = (int64_t)p;
    // LDS word e (batch-major [batch][k] secrets, then [batch][t] draws) lives at lpos(e): one pad
    // word per 16 keeps the even/odd lane->batch reads below 2-way bank conflicted (b64 optimum).
    // (Unpadded at 5 waves/EU: 5 tiles of <= 31.75 KiB fit the 160 KiB LDS; the pad measured neutral.  Unpadded
    // at n + 1 = 81 too: 2 waves per EU, VALU-bound, and the layout the LDS-DMA stage needs.)
    constexpr bool PAD = gen_waves<L, N3, CANON, LAZY>() < 5 && N3 < 81;
    __shared__ int64_t lds[BS * (L - 1) + (PAD ? BS * (L - 1) / 16 + 1 : 0)];
    auto lpos = [](uint32_t e) { return PAD ? e + (e >> 4) : e; };

    {
        const GenTables& T = *Tp;
        // XCD-chunked tile order (xcd.h): each XCD streams one contiguous eighth of the [vector][tile] grid.
        // Only for the transforms up to L = 16 (the benchmarked sizes): the wide register kernels run at
        // 1-2 waves with their registers full, and keep the natural order's code unchanged.
        uint32_t tile = blockIdx.x, vec = blockIdx.y;
        if constexpr (L <= 16) {
            if (xcd) xcd_block_xy(&tile, &vec);
        }
        const uint64_t b0 = (uint64_t)tile * BS;
        const int64_t* sec = secrets + (uint64_t)vec * D;

        // ---- stage the tile's inputs through LDS with coalesced loads ----
        // lds[0, BS k): the secrets of batches b0.. (zero past D: batched.rs:37-43 pads the tail
        // batch); lds[BS k, BS (k + t)): their randomness.  U loads in flight before the first wait.
        // uniform: no tail batch, no padding (SDA_GEN_FULLTILE = 0, a build-time A/B knob, stages every tile
        // through the bounds-checked loops)
        const bool full = SDA_GEN_FULLTILE && b0 + BS <= B && (b0 + BS) * k <= D;
        bool staged = false;
        if constexpr (SDA_GEN_DMA && !PAD && BS == 256) {
            // a full tile's inputs are two contiguous blocks, BS k secrets and BS t draws, laid out in LDS
            // exactly as in HBM: global_load_lds_dwordx4 copies them straight in, 1 KiB per wave
            // instruction, no VGPRs, no ds_write (when both blocks are 16-byte aligned).  One loop over the
            // 2 (k + t) chunks with a computed source and a wave-uniform chunk index: every DMA of the tile is
            // issued before any wait (round 5's two loops put an s_waitcnt vmcnt(0) between them).
            const int64_t* sblk = sec + b0 * k;
            const int64_t* dblk = draws + ((uint64_t)vec * B + b0) * t;
            if (full && (((uintptr_t)sblk | (uintptr_t)dblk) & 15) == 0) {
                typedef __attribute__((address_space(3))) char lds_char;
                lds_char* lbase = (lds_char*)lds;
                const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
                const uint32_t nsc = 2 * k, nc = 2 * (k + t);    // 1 KiB chunks: BS k * 8 / 1024 = 2 k
                for (uint32_t c = w; c < nc; c += BS / 64) {
                    const int64_t* src = c < nsc ? sblk + (uint64_t)c * 128 : dblk + (uint64_t)(c - nsc) * 128;
                    __builtin_amdgcn_global_load_lds((const void*)(src + 2 * l), lbase + c * 1024, 16, 0,
                                                     SDA_GEN_DMA_AUX);
                }
                // the LDS writes of a DMA count in vmcnt, and s_barrier does not wait for them: every wave drains
                // its own DMAs before the barrier, so the other waves' reads see every chunk
                __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0) (gfx9 encoding; lgkm/exp counters untouched)
                staged = true;
            }
        }
        if (staged) {
        } else if (full) {
            // the tile's BS (k + t) = BS (L - 1) input words as L - 1 rows of BS: row u < k is secrets
            // [b0 k + u BS, +BS), row u >= k draws [(vec B + b0) t + (u - k) BS, +BS) -- each row one
            // coalesced load from a uniform base, landing at lds[u BS + tid] (the layout below)
            const int64_t* ssrc = sec + b0 * k + tid;
            const int64_t* dsrc = draws + ((uint64_t)vec * B + b0) * t + tid;
            int64_t v[L - 1];
            static_for<0, L - 1>([&](auto u) {
                v[u] = gen_load((uint32_t)u < k ? ssrc + (uint64_t)u * BS : dsrc + (uint64_t)(u - k) * BS);
            });
            static_for<0, L - 1>([&](auto u) { lds[lpos((uint32_t)u * BS + tid)] = v[u]; });
        } else {
            constexpr int U = 8;
            const uint64_t nb = B - b0 < (uint64_t)BS ? B - b0 : (uint64_t)BS;
            const uint64_t s0 = b0 * k;
            const uint32_t ns = (uint32_t)nb * k;
            const uint32_t valid = D > s0 ? (uint32_t)(D - s0 < ns ? D - s0 : ns) : 0u;
            const int64_t* ssrc = sec + s0;
            for (uint32_t base = 0; base < ns; base += U * BS) {
                int64_t v[U];
                static_for<0, U>([&](auto u) {
                    const uint32_t e = base + u * BS + tid;
                    v[u] = gen_load(ssrc + (e < valid ? e : 0));   // read once
                });
                static_for<0, U>([&](auto u) {
                    const uint32_t e = base + u * BS + tid;
                    if (e < ns) lds[lpos(e)] = e < valid ? v[u] : 0;
                });
            }
            const uint32_t nd = (uint32_t)nb * t;
            const int64_t* dsrc = draws + ((uint64_t)vec * B + b0) * t;
            const uint32_t dbase = (uint32_t)BS * k;
            for (uint32_t base = 0; base < nd; base += U * BS) {
                int64_t v[U];
                static_for<0, U>([&](auto u) {
                    const uint32_t e = base + u * BS + tid;
                    v[u] = gen_load(dsrc + (e < nd ? e : 0));
                });
                static_for<0, U>([&](auto u) {
                    const uint32_t e = base + u * BS + tid;
                    if (e < nd) lds[lpos(dbase + e)] = v[u];
                });
            }
        }
        __syncthreads();
        if constexpr (!CANON) set_prio<0>();

        // values = [0, secrets, randomness]; lanes past B run on zeros and store nothing
        const uint64_t b = b0 + lb;
        const bool live = b < B;
        int64_t raw[L];
        raw[0] = 0;
        {
            const uint32_t es = lb * k - 1;                                    // + i,      i <= k
            const uint32_t ed = (uint32_t)BS * k + lb * t - 1 - k;             // + i,      i >  k
            // (lanes past B read whatever the LDS holds: they log nothing, store nothing and count as in range)
            static_for<1, L>([&](auto i) { raw[i] = lds[lpos(((uint32_t)i <= k ? es : ed) + i)]; });
        }
        bool in_range = true;
        static_for<1, L>([&](auto i) { in_range = in_range && ((uint64_t)(raw[i] + (P - 1)) < (uint64_t)(2 * P - 1)); });
        // a dead lane's stale LDS words must not send its live partner to the fix-up kernel: it counts as in
        // range, so how much fix-up work runs depends only on the inputs
        in_range = in_range || !live;
        // A store pair (see the lane map above) takes the fast path only when both of its batches
        // are in range; otherwise both lanes log their batch for the generic exact fix-up kernel
        // (rare: raw i64 secrets) and the fast path below stores nothing for the pair.  (A call
        // to the generic path from inside this loop would force the live FFT state to spill.)
        const uint32_t ok = in_range ? 1u : 0u;
        const auto okx = __builtin_amdgcn_permlane32_swap(ok, ok, false, false);
        bool pair_ok = in_range && (half ? okx[0] : okx[1]);
        if (live && !pair_ok) {                  // -> packed_gen_fixup_kernel
            const uint32_t slot = atomicAdd(log, 1u);
            if (slot < kGenLogCap) reinterpret_cast<uint64_t*>(log + 16)[slot] = (uint64_t)vec * B + b;
        }

        Trunc<LAZY> tr;
        [[maybe_unused]] RangeTrap rt, rt3;      // SIGNBIT: radix-2 half, first radix-3 level
        int32_t ys[N3];                  // shares (tss' signed values, or canonical residues)
        if constexpr (CANON) {
            transform_canon<L, N3>(raw, T, M, ys);
        } else {
        // ---- fft2_inverse: radix-2 DIT over omega_secrets^-1 on bit-reversed registers ----
        FE x[L];
        if constexpr (SIGNBIT) {
            uint32_t xc[L], xn[L];               // residue, sign word (bit 31)
            static_for<0, L>([&](auto i) {
                const int32_t s = (int32_t)raw[i];
                xc[rev_digits(i, 2, LB)] = canon32(s, p);
                xn[rev_digits(i, 2, LB)] = (uint32_t)s;
            });
            static_for<1, LB + 1>([&](auto s) {
                constexpr int H = 1 << (s - 1), LEN = 2 * H;
                static_for<0, L, LEN>([&](auto g) {
                    static_for<0, H>([&](auto i) {
                        constexpr int a = g + i, b = g + i + H;
                        const uint32_t cu = xc[a], nu = xn[a], cc = xc[b], nc = xn[b];
                        if constexpr (i == 0) {
                            const uint32_t t = cu + cc, d1 = t - p;           // bit 31: cu + cc < p
                            const uint32_t d2 = cu - cc;                      // bit 31: cu < cc
                            xc[a] = min(t, d1);
                            xn[a] = maj3(nu, nc, d1);
                            xc[b] = min(d2, d2 + p);
                            xn[b] = maj3_nb(nu, nc, d2);
                        } else {
                            rt.mul1(cc, T.big2);
                            const uint32_t tc = montu<true>(T.tw2_m[H - 1 + i], cc, M);
                            xc[a] = addm(cu, tc, p);
                            xc[b] = subm(cu, tc, p);
                            xn[a] = nc;
                            xn[b] = ~nc;
                        }
                        // a zero residue is wrong only as 0 with the sign set (a nonzero multiple of p);
                        // the first butterfly's u is the structural value 0 (values[0]): (0 +- c) % p is
                        // exact for c = 0 too, so sparse secrets do not trip the trap there
                        if constexpr (!(s == 1 && g == 0)) {
                            rt.out1(xc[a]);
                            rt.out1(xc[b]);
                        }
                    });
                });
            });
            // x * len_inv % p keeps x's sign; the radix-3 half takes tss' signed values again
            static_for<0, L>([&](auto i) {
                const uint32_t c = montu<true>(T.linv_m, xc[i], M);      // 0 only for x = 0: exact
                x[i] = FE{(int32_t)(c - (p & (uint32_t)((int32_t)xn[i] >> 31))), c};
            });
        } else {
        static_for<0, L>([&](auto i) {
            const int32_t s = (int32_t)raw[i];
            x[rev_digits(i, 2, LB)] = FE{s, canon32(s, p)};
        });
        static_for<1, LB + 1>([&](auto s) {
            constexpr int H = 1 << (s - 1), LEN = 2 * H;
            static_for<0, L, LEN>([&](auto g) {
                static_for<0, H>([&](auto i) {
                    if constexpr (i == 0) {
                        bfly2_unit(x[g], x[g + H], p, tr);
                    } else {
                        const int32_t w = (int32_t)T.tw2[H - 1 + i];
                        bfly2(x[g + i], x[g + i + H], w, -w, T.tw2_m[H - 1 + i], M, tr);
                    }
                });
            });
        });
        // x * len_inv % p   (len_inv > 0 => the exact product has the sign of x)
        static_for<0, L>([&](auto i) {
            const uint32_t c = montu<LAZY>(T.linv_m, x[i].c, M);
            x[i] = FE{tr(c, (uint32_t)x[i].s, p), c};
        });
        }

        // ---- fft3: radix-3 DIT over omega_shares on digit-reversed, zero-extended registers ----
        FE y[N3];
        static_for<0, N3>([&](auto i) {
            if constexpr (i < L) y[rev_digits(i, 3, ND)] = x[i < L ? (int)i : 0];
            else y[rev_digits(i, 3, ND)] = FE{0, 0};
        });
        static_for<1, ND + 1>([&](auto s) {
            constexpr int th = ipow(3, s - 1);
            constexpr int LEN = 3 * th, OB = (LEN - 3) / 2;
            constexpr bool last = (s == ND);
            static_for<0, N3, LEN>([&](auto g) {
                static_for<0, th>([&](auto i) {
                    constexpr bool zc = Z::is_zero(s - 1, g + i + th), zd = Z::is_zero(s - 1, g + i + 2 * th);
                    if constexpr (zc && zd) {
                        // (b + x 0 + x^2 0) % p == b for b in (-p, p): all three outputs are b
                        y[g + i + th] = y[g + i];
                        y[g + i + 2 * th] = y[g + i];
                    } else {
                        const FE bb = y[g + i], cc = y[g + i + th], dd = y[g + i + 2 * th];
                        if constexpr (zd && SIGNBIT && s == 1) rt3.mul1(cc.c, T.big3);
                        FE r[3];
                        static_for<0, 3>([&](auto q) {
                            constexpr int j = i + q * th;
                            if constexpr (last && g + j == 0) {
                                r[q] = FE{0, 0};            // points[0] is dropped (shares = points[1..])
                            } else if constexpr (j == 0) {
                                // x = x^2 = 1: (b + c + d) % p
                                if constexpr (zd) {
                                    const uint32_t c = addm(bb.c, cc.c, p);
                                    r[q] = FE{tr(c, (uint32_t)__builtin_elementwise_add_sat(bb.s, cc.s), p), c};
                                } else {
                                    const int64_t v = (int64_t)bb.s + cc.s + dd.s;
                                    const uint32_t c = addm(addm(bb.c, cc.c, p), dd.c, p);
                                    r[q] = FE{tr(c, hi32(v), p), c};
                                }
                            } else if constexpr (zd && SIGNBIT && s == 1) {
                                // first level, b + x c: the sign of c when |c| >= big3 (RangeTrap: c is
                                // checked against big3 below, the residue for 0)
                                const uint32_t c = addm(bb.c, montu<LAZY>(T.tw3_m[OB + j], cc.c, M), p);
                                r[q] = FE{tr(c, (uint32_t)cc.s, p), c};
                            } else if constexpr (zd) {
                                const int32_t xw = (int32_t)T.tw3[OB + j];
                                const int64_t v = (int64_t)bb.s + (int64_t)xw * cc.s;
                                const uint32_t c = addm(bb.c, montu<LAZY>(T.tw3_m[OB + j], cc.c, M), p);
                                r[q] = FE{tr(c, hi32(v), p), c};
                            } else {
                                // twiddles < p < 2^31: signed 32x32 products are exact (v_mad_i64_i32)
                                // x^2 % p = omega_len^(2j mod len): the same level's entry (2j) % len, so
                                // the stage needs half the uniform words (fewer SGPR spills)
                                constexpr int j2 = (2 * j) % LEN;
                                const int32_t xw = (int32_t)T.tw3[OB + j], x2 = (int32_t)T.tw3[OB + j2];
                                const int64_t v = (int64_t)bb.s + (int64_t)xw * cc.s + (int64_t)x2 * dd.s;
                                // residue: REDC(x' C + x2' D) + B
                                const uint32_t c = addm(bb.c, montu2<LAZY>(T.tw3_m[OB + j], cc.c, T.tw3_m[OB + j2], dd.c, M), p);
                                r[q] = FE{tr(c, hi32(v), p), c};
                            }
                        });
                        y[g + i] = r[0]; y[g + i + th] = r[1]; y[g + i + 2 * th] = r[2];
                        tr.note2(r[0].s, r[1].s);
                        tr.note1(r[2].s);
                    }
                });
            });
        });

        static_for<0, N3>([&](auto j) { ys[j] = y[j].s; });
        }

        if constexpr (LAZY) {                    // a -p under lazy truncation (see Trunc): same rule
            bool trapped = tr.bad(p);
            if constexpr (SIGNBIT) trapped = trapped || rt.bad(T.big2, p) || rt3.bad(T.big3, p);
            const uint32_t z = trapped ? 1u : 0u;
            const auto zx = __builtin_amdgcn_permlane32_swap(z, z, false, false);
            const bool pair_zero = z || (half ? zx[0] : zx[1]);
            if (pair_ok && pair_zero) {
                pair_ok = false;
                if (live) {
                    const uint32_t slot = atomicAdd(log, 1u);
                    if (slot < kGenLogCap)
                        reinterpret_cast<uint64_t*>(log + 16)[slot] = (uint64_t)vec * B + b0 + lb;
                }
            }
        }

        // ---- shares = points[1..=n], clerk-major (batched.rs:46-48) ----
        if constexpr (!CANON) set_prio<SDA_GEN_PRIO_STORE>();
        const uint64_t pb = b0 + pb_off;
        const bool st1 = pair_ok && pb + 1 < B;
        int64_t* orow = out + ((uint64_t)vec * NR + half) * B + pb;
        if constexpr (WIDE) {              // B even => pb + 1 < B whenever pb < B
            static_for<0, NR / 2>([&](auto q) {
                const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)ys[1 + 2 * q], (uint32_t)ys[2 + 2 * q],
                                                                false, false);
                const int32_t lo = (int32_t)r[0], hi = (int32_t)r[1];  // batches pb, pb + 1 of row 1+2q+half
                if (st1) {
                    typedef int32_t v4i __attribute__((ext_vector_type(4)));
                    v4i* d4 = reinterpret_cast<v4i*>(orow + (uint64_t)(2 * q) * B);
                    const v4i val = {lo, lo >> 31, hi, hi >> 31};
                    gen_store(val, d4);       // streamed once: keep it out of L2/MALL
                }
            });
        } else {                           // odd B: each lane stores its own batch
            int64_t* own = out + (uint64_t)vec * NR * B + b;
            static_for<1, N3>([&](auto j) { if (live && pair_ok) own[(uint64_t)(j - 1) * B] = (int64_t)ys[j]; });
        }
    }
}

}  // namespace

// The non-lazy exact kernels (p < 2^24, or odd B / unaligned out) exist only where gen_register_path admits them.
template <int L, int N3, bool CANON>
static hipError_t gen_launch_mode(const PackedGenArgs& a, uint32_t k, uint32_t t, uint64_t B, const GenTables* T,
                                  uint32_t p, const GenFixupLog& log, hipStream_t s) {
    constexpr int BS = gen_block<L>();
    const dim3 grid((unsigned)((B + BS - 1) / BS), (unsigned)a.n_vectors);
    const bool wide = B % 2 == 0 && ((uintptr_t)a.out % 16) == 0;
    const int xcd = a.xcd_order && (uint64_t)grid.x * grid.y < (1ull << 32) ? 1 : 0;
    constexpr bool NONLAZY = CANON || gen_register_path(L, N3, true);
    if (wide && !CANON && p >= kLazyTruncMinP && a.signbit)   // exact shares, sign-bit radix-2 half
        hipLaunchKernelGGL((packed_gen_kernel<L, N3, true, false, true, true>), grid, dim3(BS), 0, s, a.secrets,
                           a.dimension, a.draws, a.out, k, t, B, T, log.count, xcd);
    else if (wide && !CANON && p >= kLazyTruncMinP)          // exact shares, lazy zero handling
        hipLaunchKernelGGL((packed_gen_kernel<L, N3, true, false, true>), grid, dim3(BS), 0, s, a.secrets,
                           a.dimension, a.draws, a.out, k, t, B, T, log.count, xcd);
    else if constexpr (!NONLAZY)
        return hipErrorInvalidValue;                          // the dispatcher sends these to packed_wide.hip
    else if (wide)
        hipLaunchKernelGGL((packed_gen_kernel<L, N3, true, CANON, false>), grid, dim3(BS), 0, s, a.secrets,
                           a.dimension, a.draws, a.out, k, t, B, T, log.count, xcd);
    else
        hipLaunchKernelGGL((packed_gen_kernel<L, N3, false, CANON, false>), grid, dim3(BS), 0, s, a.secrets,
                           a.dimension, a.draws, a.out, k, t, B, T, log.count, xcd);
    return hipSuccess;
}

template <int L, int N3>
hipError_t gen_launch(const PackedGenArgs& a, uint32_t k, uint32_t t, uint64_t B, const GenTables* T,
                      const GenFixupLog& log, hipStream_t s) {
    constexpr int BS = gen_block<L>();
    if ((B + BS - 1) / BS > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const uint32_t p = a.prime;
    const hipError_t e = a.canonical ? gen_launch_mode<L, N3, true>(a, k, t, B, T, p, log, s)
                                     : gen_launch_mode<L, N3, false>(a, k, t, B, T, p, log, s);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}
template hipError_t gen_launch<SDA_GEN_L, SDA_GEN_PART>(const PackedGenArgs&, uint32_t, uint32_t, uint64_t,
                                                        const GenTables*, const GenFixupLog&, hipStream_t);

#else  // dispatcher, tables, generic fix-up

namespace {

// ---------------- generic exact share-gen fix-up ----------------
// Batches the fast kernel logged -- inputs outside (-p, p) (raw i64 secrets), or a lazy-truncation /
// sign-bit trap -- recomputed with tss' operations verbatim: wrapping i64 products and sums, Rust's
// truncated % after every butterfly, the fast kernels' tables.  One wave per batch (the transform is the
// same one lane's generic path used to run serially, ~55 us per launch): lane j takes butterfly j of a
// radix-2 level and outputs j, j + 64 of a radix-3 level, the state in LDS (radix-3 levels double
// buffered, as their outputs overwrite other lanes' inputs).  If the log overflowed, every batch of the
// launch is recomputed (correct, slow, and only reachable with raw i64 secrets far outside the field).
__global__ __launch_bounds__(64) void packed_gen_fixup_kernel(const int64_t* __restrict__ secrets, uint64_t D,
                                                              const int64_t* __restrict__ draws,
                                                              int64_t* __restrict__ out, uint32_t k, uint32_t t,
                                                              uint64_t B, uint64_t n_vec, int L, int N3,
                                                              const GenTables* __restrict__ T, GenFixupLog log,
                                                              int canonical) {
    const uint32_t n = *log.count;
    if (n == 0) return;
    const bool all = n > log.cap;
    const uint64_t total = all ? B * n_vec : (uint64_t)n;
    __shared__ int64_t xa[64];
    __shared__ int64_t ya[2][81];
    const Mod64 P = make_mod64((int64_t)T->M.p);
    const int lane = threadIdx.x;
    const int lb = ilog(L, 2), nd = ilog(N3, 3);
    for (uint64_t i = blockIdx.x; i < total; i += gridDim.x) {
        const uint64_t gb = all ? i : log.list[i];
        const uint64_t vec = gb / B, b = gb - vec * B;
        __syncthreads();                                 // the previous batch's stores have read ya
        // values = [0, secrets (zero past D: batched.rs:37-43), randomness], bit-reversed
        if (lane < L) {
            int64_t val = 0;
            if (lane >= 1 && (uint32_t)lane <= k) {
                const uint64_t idx = b * k + (lane - 1);
                val = idx < D ? secrets[vec * D + idx] : 0;
            } else if (lane > 0) {
                val = draws[gb * t + (lane - 1 - k)];
            }
            xa[rev_digits(lane, 2, lb)] = val;
        }
        // fft2_inverse: butterfly `lane` of each level, (u +- w c) % p
        for (int len = 2; len <= L; len *= 2) {
            const int h = len / 2, g = (lane / h) * len, ii = lane % h;
            __syncthreads();
            int64_t u = 0, c = 0, w = 0;
            if (lane < L / 2) {
                u = xa[g + ii];
                c = xa[g + ii + h];
                w = T->tw2[h - 1 + ii];
            }
            __syncthreads();
            if (lane < L / 2) {
                xa[g + ii] = trem64(wadd(u, wmul(w, c)), P);
                xa[g + ii + h] = trem64(wsub(u, wmul(w, c)), P);
            }
        }
        __syncthreads();
        // x * len_inv % p, zero-extended to N3 and digit-reversed
        for (int j = lane; j < N3; j += 64)
            ya[0][rev_digits(j, 3, nd)] = j < L ? trem64(wmul(xa[j], (int64_t)T->linv), P) : 0;
        // fft3: output j of each level, (b + x c + x^2 d) % p
        int cur = 0;
        for (int len = 3; len <= N3; len *= 3) {
            const int th = len / 3, o = (len - 3) / 2;
            __syncthreads();
            for (int j = lane; j < N3; j += 64) {
                const int g = j - j % len, jj = j % len, i0 = jj % th;
                const int64_t bb = ya[cur][g + i0], cc = ya[cur][g + i0 + th], dd = ya[cur][g + i0 + 2 * th];
                ya[cur ^ 1][j] = trem64(wadd(wadd(bb, wmul((int64_t)T->tw3[o + jj], cc)), wmul((int64_t)T->sq3[o + jj], dd)), P);
            }
            cur ^= 1;
        }
        __syncthreads();
        // shares = points[1..=n], clerk-major; CANONICAL: the exact share's canonical residue
        int64_t* ob = out + vec * (uint64_t)(N3 - 1) * B + b;
        for (int j = lane + 1; j < N3; j += 64) {
            const int64_t v = ya[cur][j];
            ob[(uint64_t)(j - 1) * B] = (canonical && v < 0) ? v + (int64_t)T->M.p : v;
        }
    }
}

}  // namespace

bool xcd_order_enabled() {
    static const bool on = [] {
        const char* e = getenv("SDA_XCD_ORDER");
        return !(e && e[0] == '0');
    }();
    return on;
}

size_t packed_gen_log_bytes() { return 64 + (size_t)kGenLogCap * sizeof(uint64_t); }

hipError_t launch_packed_generate(const PackedGenArgs& args, uint32_t k, uint32_t t, uint32_t n, uint32_t p,
                                  uint32_t omega_secrets, uint32_t omega_shares, DeviceTable& tab, void* log_buf,
                                  hipStream_t s) {
    PackedGenArgs a = args;
    a.prime = p;
    const uint32_t L = k + t + 1, N3 = n + 1;
    const uint64_t B = (a.dimension + k - 1) / k;
    // the register kernels' variant: WIDE stores need even B and 16-byte aligned out; lazy truncation p >= 2^24
    const bool exact_nonlazy = !a.canonical && !(B % 2 == 0 && ((uintptr_t)a.out % 16) == 0 && p >= kLazyTruncMinP);
    if (!gen_register_path(L, N3, exact_nonlazy))            // past the register kernels: packed_wide.hip
        return launch_packed_generate_wide(a, k, t, n, p, omega_secrets, omega_shares, tab, s);
    if (B == 0 || a.n_vectors == 0) return hipSuccess;
    const uint32_t kv[5] = {L, N3, p, omega_secrets, omega_shares};
    std::vector<uint8_t> key((const uint8_t*)kv, (const uint8_t*)kv + sizeof(kv));
    if (tab.key != key) {
        const GenTables T = make_gen_tables(L, N3, p, omega_secrets, omega_shares);
        hipError_t e = ensure_table(tab, key, &T, sizeof(T));
        if (e != hipSuccess) return e;
        // the sign-bit kernel when its range traps stay rare (every multiplied operand must reach
        // ceil(p / w); bounds above 2^12 would send a measurable share of batches to the fix-up)
        tab.flags = (T.big2 <= 4096 && T.big3 <= 4096) ? 1u : 0u;
    }
    const char* sb = getenv("SDA_GEN_SIGNBIT");                 // A/B knob: 0 = the mad_i64 sign kernel
    a.signbit = (tab.flags & 1u) && !(sb && sb[0] == '0');
    a.xcd_order = xcd_order_enabled();
    const GenTables* T = static_cast<const GenTables*>(tab.dev);
    GenFixupLog log{static_cast<unsigned int*>(log_buf),
                    reinterpret_cast<uint64_t*>(static_cast<unsigned int*>(log_buf) + 16), kGenLogCap};
    hipError_t e = hipMemsetAsync(log.count, 0, sizeof(unsigned int), s);
    if (e != hipSuccess) return e;
    switch (N3 * 128 + L) {             // one object per (N3, L): Makefile GEN_PARTS
#define SDA_GEN_CASE(N, LL) case N * 128 + LL: e = gen_launch<LL, N>(a, k, t, B, T, log, s); break;
        SDA_GEN_CASE(3, 2)
        SDA_GEN_CASE(9, 2) SDA_GEN_CASE(9, 4) SDA_GEN_CASE(9, 8)
        SDA_GEN_CASE(27, 2) SDA_GEN_CASE(27, 4) SDA_GEN_CASE(27, 8) SDA_GEN_CASE(27, 16)
        SDA_GEN_CASE(81, 2) SDA_GEN_CASE(81, 4) SDA_GEN_CASE(81, 8) SDA_GEN_CASE(81, 16) SDA_GEN_CASE(81, 32)
        SDA_GEN_CASE(81, 64)
#undef SDA_GEN_CASE
        default: e = hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(packed_gen_fixup_kernel, dim3(512), dim3(64), 0, s, a.secrets, a.dimension, a.draws, a.out,
                       k, t, B, a.n_vectors, (int)L, (int)N3, T, log, a.canonical ? 1 : 0);
    return hipGetLastError();
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
    if (t.ws) (void)hipFree(t.ws);
    t.dev = t.ws = nullptr;
    t.cap = t.ws_cap = 0;
    t.key.clear();
}

#endif  // SDA_GEN_PART

}  // namespace sda
