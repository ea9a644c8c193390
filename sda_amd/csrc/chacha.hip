// chacha.hip -- north-star kernel (3): ChaCha PRG mask expansion in counter mode.
//
// Reference: client/src/crypto/masking/chacha.rs
//   mask     :25-53  ChaChaRng::from_seed(seed); D x gen_range(0, m); masked = (s + mask) % m
//   combine  :57-76  for each participant seed: re-seed, D x gen_range, result = (r + m) % m
// rand 0.3 (absent from the reference tree) defines the stream: ChaCha20 (10 double rounds),
// state = "expand 32-byte k" | key = seed words (zero-padded, first 8) | 128-bit block counter
// from 0; next_u64 = (next_u32 << 32) | next_u32; gen_range(0, m) draws v = next_u64 and
// rejects v >= zone = u64::MAX - u64::MAX % m, else returns v % m.
//
// Counter mode makes the stream randomly accessible: absent rejections, element i of a stream
// is words (2i, 2i+1) = block i/8.  One lane expands one 64-byte block (8 mask elements) per
// seed and loops over seeds, accumulating canonical sums (every draw is >= 0, so the reference
// result is the canonical sum and order-independent).  A rejection shifts every later element
// of that stream by one word pair: the main kernel adds the un-shifted draw and records the
// (seed, pair) event; a host-driven fix-up then recomputes only the affected stream suffixes
// (probability < 2^-33 per draw for 31-bit m).  Roofline: VALU (~1000 int32 ops per block).
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include <atomic>

#include "kernels.h"

namespace sda {

namespace {

constexpr uint32_t C0 = 0x61707865u, C1 = 0x3320646Eu, C2 = 0x79622D32u, C3 = 0x6B206574u;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, 32 - r); }

#define SDA_QR(a, b, c, d)                    \
    a += b; d ^= a; d = rotl(d, 16);          \
    c += d; b ^= c; b = rotl(b, 12);          \
    a += b; d ^= a; d = rotl(d, 8);           \
    c += d; b ^= c; b = rotl(b, 7);

struct Key8 { uint32_t k[8]; };

// Round 1's column quarter-rounds on columns 1-3 read only the key, the constants and the counter's high
// word -- per stream (and per workgroup) uniform -- so a kernel that walks many blocks of one stream per
// iteration computes them once, as scalar code, and hands them to chacha_block_pre.
struct ChachaPre {
    uint32_t x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15;
};

__device__ __forceinline__ ChachaPre chacha_pre(const uint32_t* key, uint32_t ctr_hi) {
    ChachaPre P{C1, key[1], key[5], ctr_hi, C2, key[2], key[6], 0u, C3, key[3], key[7], 0u};
    SDA_QR(P.x1, P.x5, P.x9, P.x13);
    SDA_QR(P.x2, P.x6, P.x10, P.x14);
    SDA_QR(P.x3, P.x7, P.x11, P.x15);
    return P;
}

// chacha_block with round 1's columns 1-3 taken from P (= chacha_pre(key, counter >> 32))
__device__ __forceinline__ void chacha_block_pre(const ChachaPre& P, const uint32_t* key, uint64_t counter,
                                                 uint32_t (&o)[16]) {
    uint32_t x0 = C0, x4 = key[0], x8 = key[4], x12 = (uint32_t)counter;
    uint32_t x1 = P.x1, x5 = P.x5, x9 = P.x9, x13 = P.x13, x2 = P.x2, x6 = P.x6, x10 = P.x10, x14 = P.x14;
    uint32_t x3 = P.x3, x7 = P.x7, x11 = P.x11, x15 = P.x15;
    SDA_QR(x0, x4, x8, x12);
    SDA_QR(x0, x5, x10, x15); SDA_QR(x1, x6, x11, x12); SDA_QR(x2, x7, x8, x13); SDA_QR(x3, x4, x9, x14);
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        SDA_QR(x0, x4, x8, x12); SDA_QR(x1, x5, x9, x13); SDA_QR(x2, x6, x10, x14); SDA_QR(x3, x7, x11, x15);
        SDA_QR(x0, x5, x10, x15); SDA_QR(x1, x6, x11, x12); SDA_QR(x2, x7, x8, x13); SDA_QR(x3, x4, x9, x14);
    }
    o[0] = x0 + C0; o[1] = x1 + C1; o[2] = x2 + C2; o[3] = x3 + C3;
    o[4] = x4 + key[0]; o[5] = x5 + key[1]; o[6] = x6 + key[2]; o[7] = x7 + key[3];
    o[8] = x8 + key[4]; o[9] = x9 + key[5]; o[10] = x10 + key[6]; o[11] = x11 + key[7];
    o[12] = x12 + (uint32_t)counter; o[13] = x13 + (uint32_t)(counter >> 32); o[14] = x14; o[15] = x15;
}

// Two independent blocks (two seeds, same counter) with their quarter-rounds interleaved statement by
// statement, so each dependent add -> xor -> rotate chain has a partner to issue beside it.
#define SDA_QR2(a, b, c, d, A, B, C, D)                                        \
    a += b; A += B; d ^= a; D ^= A; d = rotl(d, 16); D = rotl(D, 16);        \
    c += d; C += D; b ^= c; B ^= C; b = rotl(b, 12); B = rotl(B, 12);        \
    a += b; A += B; d ^= a; D ^= A; d = rotl(d, 8); D = rotl(D, 8);          \
    c += d; C += D; b ^= c; B ^= C; b = rotl(b, 7); B = rotl(B, 7);

__device__ __forceinline__ void chacha_block_pre_x2(const ChachaPre& P, const uint32_t* key, const ChachaPre& Q,
                                                    const uint32_t* kq, uint64_t counter, uint32_t (&o)[16],
                                                    uint32_t (&u)[16]) {
    uint32_t x0 = C0, x4 = key[0], x8 = key[4], x12 = (uint32_t)counter;
    uint32_t x1 = P.x1, x5 = P.x5, x9 = P.x9, x13 = P.x13, x2 = P.x2, x6 = P.x6, x10 = P.x10, x14 = P.x14;
    uint32_t x3 = P.x3, x7 = P.x7, x11 = P.x11, x15 = P.x15;
    uint32_t y0 = C0, y4 = kq[0], y8 = kq[4], y12 = (uint32_t)counter;
    uint32_t y1 = Q.x1, y5 = Q.x5, y9 = Q.x9, y13 = Q.x13, y2 = Q.x2, y6 = Q.x6, y10 = Q.x10, y14 = Q.x14;
    uint32_t y3 = Q.x3, y7 = Q.x7, y11 = Q.x11, y15 = Q.x15;
    SDA_QR2(x0, x4, x8, x12, y0, y4, y8, y12);
    SDA_QR2(x0, x5, x10, x15, y0, y5, y10, y15); SDA_QR2(x1, x6, x11, x12, y1, y6, y11, y12);
    SDA_QR2(x2, x7, x8, x13, y2, y7, y8, y13); SDA_QR2(x3, x4, x9, x14, y3, y4, y9, y14);
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        SDA_QR2(x0, x4, x8, x12, y0, y4, y8, y12); SDA_QR2(x1, x5, x9, x13, y1, y5, y9, y13);
        SDA_QR2(x2, x6, x10, x14, y2, y6, y10, y14); SDA_QR2(x3, x7, x11, x15, y3, y7, y11, y15);
        SDA_QR2(x0, x5, x10, x15, y0, y5, y10, y15); SDA_QR2(x1, x6, x11, x12, y1, y6, y11, y12);
        SDA_QR2(x2, x7, x8, x13, y2, y7, y8, y13); SDA_QR2(x3, x4, x9, x14, y3, y4, y9, y14);
    }
    o[0] = x0 + C0; o[1] = x1 + C1; o[2] = x2 + C2; o[3] = x3 + C3;
    o[4] = x4 + key[0]; o[5] = x5 + key[1]; o[6] = x6 + key[2]; o[7] = x7 + key[3];
    o[8] = x8 + key[4]; o[9] = x9 + key[5]; o[10] = x10 + key[6]; o[11] = x11 + key[7];
    o[12] = x12 + (uint32_t)counter; o[13] = x13 + (uint32_t)(counter >> 32); o[14] = x14; o[15] = x15;
    u[0] = y0 + C0; u[1] = y1 + C1; u[2] = y2 + C2; u[3] = y3 + C3;
    u[4] = y4 + kq[0]; u[5] = y5 + kq[1]; u[6] = y6 + kq[2]; u[7] = y7 + kq[3];
    u[8] = y8 + kq[4]; u[9] = y9 + kq[5]; u[10] = y10 + kq[6]; u[11] = y11 + kq[7];
    u[12] = y12 + (uint32_t)counter; u[13] = y13 + (uint32_t)(counter >> 32); u[14] = y14; u[15] = y15;
}

// one ChaCha20 block: core(state) = rounds(state) + state
__device__ __forceinline__ void chacha_block(const uint32_t* key, uint64_t counter, uint32_t (&o)[16]) {
    uint32_t x0 = C0, x1 = C1, x2 = C2, x3 = C3;
    uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
    uint32_t x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
    uint32_t x12 = (uint32_t)counter, x13 = (uint32_t)(counter >> 32), x14 = 0, x15 = 0;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        SDA_QR(x0, x4, x8, x12); SDA_QR(x1, x5, x9, x13); SDA_QR(x2, x6, x10, x14); SDA_QR(x3, x7, x11, x15);
        SDA_QR(x0, x5, x10, x15); SDA_QR(x1, x6, x11, x12); SDA_QR(x2, x7, x8, x13); SDA_QR(x3, x4, x9, x14);
    }
    o[0] = x0 + C0; o[1] = x1 + C1; o[2] = x2 + C2; o[3] = x3 + C3;
    o[4] = x4 + key[0]; o[5] = x5 + key[1]; o[6] = x6 + key[2]; o[7] = x7 + key[3];
    o[8] = x8 + key[4]; o[9] = x9 + key[5]; o[10] = x10 + key[6]; o[11] = x11 + key[7];
    o[12] = x12 + (uint32_t)counter; o[13] = x13 + (uint32_t)(counter >> 32); o[14] = x14; o[15] = x15;
}

struct RejectLog {
    unsigned long long* count;   // number of rejected pairs seen
    uint32_t* seed_of;           // [cap]
    uint64_t* pair_of;           // [cap]
    uint64_t cap;
};

// A lane owns elements 8 blk .. 8 blk + 7; the workgroup's 2048 results go through LDS so that the
// write-back is coalesced (lane t writes element t + 256 j).
constexpr int kChachaPad = 9;                  // LDS row stride (u64) of a lane's 8 results
#ifndef SDA_CHACHA_PAIR
#define SDA_CHACHA_PAIR 0                      // build-time A/B knob: two interleaved seeds per step
#endif
// One tile (256 lanes x 8 draws = 2048 elements from tile x * 2048) over seeds [s0, s1): the lane's
// canonical partial sums, written back through LDS (`st`) so that the stores are coalesced -- plain
// stores when DIRECT (one chunk: acc is the output), atomics into acc otherwise.
template <bool LAZY, bool DIRECT, bool PRE>
__device__ __forceinline__ void chacha_tile(const uint32_t* __restrict__ seeds, uint32_t w, uint64_t s0, uint64_t s1,
                                            uint64_t x, uint64_t D, unsigned long long* __restrict__ acc,
                                            const Mod64& M, uint64_t zone, uint64_t r64, const RejectLog& log,
                                            const ChachaPre* __restrict__ pre, unsigned long long* st,
                                            bool opaque_tid = false) {
    uint32_t tid = threadIdx.x;
    // inside the stream-K run loop: an opaque lane id, so that no per-lane value is hoisted out of the loop
    // and held across runs (the hoisted form held 94 VGPRs instead of 80)
    if (opaque_tid) asm volatile("" : "+v"(tid));
    const uint64_t blk = x * 256 + tid;
    const uint64_t n_blk = (D + 7) / 8;
    const bool live = blk < n_blk;
    // the seed loop is uniform (lanes past D run it on draws they never keep), so each seed's key and
    // round-1 columns 1-3 are scalar work; a 256-block group never straddles 2^32, so the counter's high
    // word is uniform too
    const uint32_t ctr_hi = (uint32_t)((x * 256) >> 32);
    const uint32_t nw = w < 8 ? w : 8;
    const uint64_t m = M.m;
    const uint32_t nvalid = !live ? 0u : (D - blk * 8 < 8 ? (uint32_t)(D - blk * 8) : 8u);   // pairs inside D
    const uint32_t zone_hi = (uint32_t)(zone >> 32);     // v >= zone needs hi(v) >= zone_hi
    uint64_t a[8];
    uint32_t hi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) { a[q] = 0; hi[q] = 0; }
    // one block's draws (seed S, words O): the rejection screen, then the running sums
#define SDA_CHACHA_TAKE(S, O)                                                                                  \
    do {                                                                                                       \
        /* rejections (< 2^-28 per draw): one max over the 8 high words screens the block */                   \
        const uint32_t hmax = max(max(max(O[0], O[2]), max(O[4], O[6])), max(max(O[8], O[10]), max(O[12], O[14]))); \
        if (hmax >= zone_hi) {                                                                                 \
            _Pragma("unroll") for (int q = 0; q < 8; ++q) {                                                    \
                const uint64_t v = ((uint64_t)O[2 * q] << 32) | O[2 * q + 1];                                  \
                if ((uint32_t)q < nvalid && v >= zone) { /* rejected: log it */                               \
                    const unsigned long long slot = atomicAdd(log.count, 1ull);                                \
                    if (slot < log.cap) { log.seed_of[slot] = (uint32_t)(S); log.pair_of[slot] = blk * 8 + q; } \
                }                                                                                              \
            }                                                                                                  \
        }                                                                                                      \
        /* pairs past D are summed too and never stored (only the last block of the grid has any) */           \
        _Pragma("unroll") for (int q = 0; q < 8; ++q) {                                                        \
            const uint64_t v = ((uint64_t)O[2 * q] << 32) | O[2 * q + 1]; /* high word first */                \
            if constexpr (LAZY) {                                                                              \
                const uint64_t y = a[q] + v;                                                                   \
                hi[q] += y < v ? 1u : 0u;                                                                      \
                a[q] = y;                                                                                      \
            } else {                                                                                           \
                const uint64_t y = a[q] + umod64(v, M);                                                        \
                a[q] = y >= m ? y - m : y;                                                                     \
            }                                                                                                  \
        }                                                                                                      \
    } while (0)
    uint64_t s = s0;
    if constexpr (SDA_CHACHA_PAIR) {             // two seeds per step, their rounds interleaved
        for (; s + 1 < s1; s += 2) {
            uint32_t ka[8], kb[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                ka[q] = (uint32_t)q < nw ? seeds[s * w + q] : 0u;          // uniform: scalar loads
                kb[q] = (uint32_t)q < nw ? seeds[(s + 1) * w + q] : 0u;
            }
            uint32_t o[16], u[16];
            chacha_block_pre_x2(PRE ? pre[s] : chacha_pre(ka, ctr_hi), ka, PRE ? pre[s + 1] : chacha_pre(kb, ctr_hi),
                                kb, blk, o, u);
            SDA_CHACHA_TAKE(s, o);
            SDA_CHACHA_TAKE(s + 1, u);
        }
    }
    for (; s < s1; ++s) {
        uint32_t key[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) key[q] = (uint32_t)q < nw ? seeds[s * w + q] : 0u;   // uniform: scalar loads
        uint32_t o[16];
        chacha_block_pre(PRE ? pre[s] : chacha_pre(key, ctr_hi), key, blk, o);
        SDA_CHACHA_TAKE(s, o);
    }
#undef SDA_CHACHA_TAKE
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        uint64_t r = a[q];
        if constexpr (LAZY) {       // (hi 2^64 + lo) mod m, m <= 2^32: hi mod m < m, r64 = 2^64 mod m
            const uint64_t t = umod64((uint64_t)hi[q], M) * r64;          // < m^2 <= 2^64
            const uint64_t y = umod64(t, M) + umod64(r, M);               // < 2m
            r = y >= m ? y - m : y;
        }
        st[tid * kChachaPad + q] = r;
    }
    __syncthreads();
    const uint64_t e0 = x * 2048;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t idx = j * 256 + tid;
        const uint64_t e = e0 + idx;
        if (e < D) {
            const unsigned long long r = st[(idx >> 3) * kChachaPad + (idx & 7)];
            if constexpr (DIRECT) acc[e] = r;
            else atomicAdd(&acc[e], r);
        }
    }
}

// acc[i] += sum over seeds in this y-chunk of draw_i  (un-shifted), canonical per chunk.
// Every draw is >= 0, so the reference's running `(r + draw) % m` equals (sum of draws) mod m.
// LAZY (m <= 2^32): the raw 64-bit words v are summed into 96-bit accumulators (3 adds per draw)
// and reduced once per chunk -- (sum of v) mod m == sum of (v mod m) mod m; otherwise each draw
// is reduced with the 64-bit Barrett `%`.
// PRE: round 1's uniform columns of every seed come precomputed from `pre` (chacha_pre_kernel, counter
// high word 0: the grid then holds < 2^32 blocks); otherwise the kernel computes them per seed.
template <bool LAZY, bool DIRECT, bool PRE = false>
__global__ __launch_bounds__(256) void chacha_combine_kernel(const uint32_t* __restrict__ seeds, uint32_t w, uint64_t n_seeds,
                           uint64_t seeds_per_chunk, uint64_t D, unsigned long long* __restrict__ acc, Mod64 M,
                           uint64_t zone, uint64_t r64, RejectLog log, const ChachaPre* __restrict__ pre = nullptr) {
    __shared__ unsigned long long st[256 * kChachaPad];
    const uint64_t s0 = (uint64_t)blockIdx.y * seeds_per_chunk;
    const uint64_t s1 = s0 + seeds_per_chunk < n_seeds ? s0 + seeds_per_chunk : n_seeds;
    chacha_tile<LAZY, DIRECT, PRE>(seeds, w, s0, s1, blockIdx.x, D, acc, M, zone, r64, log, pre, st);
}

// Stream-K form of the same combine: the (tile, seed) units, tile-major, split evenly over exactly one
// round of resident workgroups (workgroup g takes units [g q + min(g, r), ..) -- q or q + 1 of them),
// each walking its range as runs of consecutive seeds of one tile and adding every run's partials into
// acc with atomics.  The chunked grid above rounds the work to whole (tile, chunk) workgroups: at the
// bench shape (489 tiles x 256 seeds, 1,792 resident workgroups) it launched 1,956 of them, a second
// round 9 % full behind the first.  Here every workgroup ends within one unit of the others.
template <bool LAZY, bool PRE>
#ifndef SDA_CHACHA_SK_WAVES
#define SDA_CHACHA_SK_WAVES 6                  // waves per SIMD the stream-K kernel is built for (80 VGPRs)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SDA_CHACHA_SK_WAVES, 8))) void chacha_combine_sk_kernel(const uint32_t* __restrict__ seeds, uint32_t w,
                                                                uint64_t n_seeds, uint64_t q, uint64_t r, uint64_t D,
                                                                unsigned long long* __restrict__ acc, Mod64 M,
                                                                uint64_t zone, uint64_t r64, RejectLog log,
                                                                const ChachaPre* __restrict__ pre) {
    __shared__ unsigned long long st[256 * kChachaPad];
    const uint64_t g = blockIdx.x;
    const uint64_t u = g * q + (g < r ? g : r);
    uint64_t left = q + (g < r ? 1 : 0);              // units still to do
    uint64_t x = u / n_seeds, s0 = u - x * n_seeds;   // the first run's tile and seed (one division)
    while (left) {
        const uint64_t s1 = n_seeds - s0 < left ? n_seeds : s0 + left;
        chacha_tile<LAZY, false, PRE>(seeds, w, s0, s1, x, D, acc, M, zone, r64, log, pre, st, true);
        left -= s1 - s0;
        ++x;
        s0 = 0;
        if (left) __syncthreads();                // st is rewritten by the next run
    }
}

// chacha_pre of every seed (counter high word 0), one lane per seed, for chacha_combine_kernel<PRE>
__global__ __launch_bounds__(256) void chacha_pre_kernel(const uint32_t* __restrict__ seeds, uint32_t w, uint64_t n_seeds,
                                                         ChachaPre* __restrict__ pre) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_seeds) return;
    const uint32_t nw = w < 8 ? w : 8;
    uint32_t key[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) key[q] = (uint32_t)q < nw ? seeds[s * w + q] : 0u;
    pre[s] = chacha_pre(key, 0u);
}

// One stream, the participant's mask (chacha.rs:36-45): out[e] = (secrets[e] + draw_e) % m; the mask itself
// is never stored.  A lane owns the 8 draws of ChaCha block `blk` (as in chacha_combine_kernel, whose
// reduction of a single draw is umod64(v) on both of its paths).  The lane's 8 secrets -- elements
// e0 + 256 j + tid, the coalesced write-back order -- are loaded before the block is computed, so their
// latency hides under the ChaCha rounds instead of following them.
__global__ __launch_bounds__(256) void chacha_mask_add_kernel(const uint32_t* __restrict__ seeds, uint32_t w, uint64_t D,
                                                              unsigned long long* __restrict__ out, Mod64 M,
                                                              uint64_t zone, RejectLog log,
                                                              const int64_t* __restrict__ secrets, bool small_m) {
    __shared__ unsigned long long st[256 * kChachaPad];
    const uint32_t tid = threadIdx.x;
    const uint64_t blk = (uint64_t)blockIdx.x * blockDim.x + tid;
    const uint64_t e0 = (uint64_t)blockIdx.x * 2048;
    int64_t sec[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint64_t e = e0 + j * 256 + tid;
        sec[j] = e < D ? __builtin_nontemporal_load(secrets + e) : 0;
    }
    const uint32_t nw = w < 8 ? w : 8;
    uint32_t key[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) key[q] = (uint32_t)q < nw ? seeds[q] : 0u;
    uint32_t o[16];
    chacha_block(key, blk, o);
    const uint32_t nvalid = blk * 8 >= D ? 0u : (D - blk * 8 < 8 ? (uint32_t)(D - blk * 8) : 8u);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const uint64_t v = ((uint64_t)o[2 * q] << 32) | o[2 * q + 1];      // high word first
        if ((uint32_t)q < nvalid && v >= zone) {                         // rejected: log it
            const unsigned long long slot = atomicAdd(log.count, 1ull);
            if (slot < log.cap) { log.seed_of[slot] = 0u; log.pair_of[slot] = blk * 8 + q; }
        }
        st[tid * kChachaPad + q] = umod64(v, M);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t idx = j * 256 + tid;
        const uint64_t e = e0 + idx;
        if (e < D) out[e] = (unsigned long long)add_trem((int64_t)st[(idx >> 3) * kChachaPad + (idx & 7)], sec[j], M, small_m);
    }
}

// Fix one stream: for elements i >= i0, replace draw(pair i) by draw(pair a_i), where a_i is the
// i-th non-rejected pair: a_i = i + #{r in rej : r <= a_i}.  acc[i] <- (acc[i] + new - old) mod m.
__global__ __launch_bounds__(256) void chacha_fix_kernel(Key8 key, uint64_t i0, uint64_t D,
                                                         const uint64_t* __restrict__ rej, uint32_t n_rej,
                                                         unsigned long long* __restrict__ acc, Mod64 M) {
    const uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= D) return;
    auto count_le = [&](uint64_t x) -> uint64_t {   // #{r <= x}
        uint32_t lo = 0, hi = n_rej;
        while (lo < hi) { uint32_t mid = (lo + hi) / 2; if (rej[mid] <= x) lo = mid + 1; else hi = mid; }
        return lo;
    };
    uint64_t k = count_le(i);
    for (;;) { const uint64_t k2 = count_le(i + k); if (k2 == k) break; k = k2; }
    const uint64_t ai = i + k;
    uint32_t o[16];
    chacha_block(key.k, i / 8, o);
    const uint64_t vo = ((uint64_t)o[2 * (i % 8)] << 32) | o[2 * (i % 8) + 1];
    chacha_block(key.k, ai / 8, o);
    const uint64_t vn = ((uint64_t)o[2 * (ai % 8)] << 32) | o[2 * (ai % 8) + 1];
    // acc[i] is canonical here (acc_mod_kernel ran in place first): stay in [0, m)
    uint64_t a = acc[i] + umod64(vn, M);          // < 2m <= 2^64 - 2
    a = a >= M.m ? a - M.m : a;
    const uint64_t od = umod64(vo, M);
    acc[i] = a >= od ? a - od : a + (M.m - od);
}

__global__ __launch_bounds__(256) void acc_mod_kernel(const unsigned long long* acc, uint64_t D,
                                                      int64_t* out, Mod64 M) {   // may run in place
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < D) out[i] = (int64_t)umod64(acc[i], M);
}

// ---- host ChaCha (product code: extends a stream's rejection list past D) ----
inline uint32_t h_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
void h_block(const uint32_t* key, uint64_t counter, uint32_t o[16]) {
    uint32_t in[16] = {C0, C1, C2, C3, key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                       (uint32_t)counter, (uint32_t)(counter >> 32), 0, 0};
    uint32_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = in[i];
#define H_QR(a, b, c, d) \
    x[a] += x[b]; x[d] ^= x[a]; x[d] = h_rotl(x[d], 16); x[c] += x[d]; x[b] ^= x[c]; x[b] = h_rotl(x[b], 12); \
    x[a] += x[b]; x[d] ^= x[a]; x[d] = h_rotl(x[d], 8);  x[c] += x[d]; x[b] ^= x[c]; x[b] = h_rotl(x[b], 7);
    for (int r = 0; r < 10; ++r) {
        H_QR(0, 4, 8, 12) H_QR(1, 5, 9, 13) H_QR(2, 6, 10, 14) H_QR(3, 7, 11, 15)
        H_QR(0, 5, 10, 15) H_QR(1, 6, 11, 12) H_QR(2, 7, 8, 13) H_QR(3, 4, 9, 14)
    }
#undef H_QR
    for (int i = 0; i < 16; ++i) o[i] = x[i] + in[i];
}
uint64_t h_pair(const uint32_t* key, uint64_t pair) {
    uint32_t o[16];
    h_block(key, pair / 8, o);
    return ((uint64_t)o[2 * (pair % 8)] << 32) | o[2 * (pair % 8) + 1];
}


// ---- exact stream expansion (any rejection rate): the draws of T streams as rows [T][D] ----
// Pass 1 counts the accepted pairs among the first n_pairs pairs per workgroup, pass 2 scans the
// counts of each stream, pass 3 recomputes the blocks and writes the i-th accepted draw (mod m) to
// element i -- exactly gen_range's rejection loop, with no per-stream limit on rejections.
__device__ __forceinline__ void stream_key(const uint32_t* seeds, uint32_t w, uint64_t s, uint32_t (&key)[8]) {
    const uint32_t nw = w < 8 ? w : 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) key[q] = (uint32_t)q < nw ? seeds[s * w + q] : 0u;
}

__device__ __forceinline__ uint32_t block_sum256(uint32_t v, uint32_t* lds) {
    lds[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) lds[threadIdx.x] += lds[threadIdx.x + h];
        __syncthreads();
    }
    const uint32_t r = lds[0];
    __syncthreads();
    return r;
}

// exclusive prefix of v over the 256 lanes of the workgroup (Hillis-Steele in LDS)
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* lds) {
    lds[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {
        const uint32_t add = threadIdx.x >= d ? lds[threadIdx.x - d] : 0u;
        __syncthreads();
        lds[threadIdx.x] += add;
        __syncthreads();
    }
    const uint32_t incl = lds[threadIdx.x];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(256) void chacha_stream_count_kernel(const uint32_t* __restrict__ seeds, uint32_t w,
                                                                  uint64_t seed0, uint64_t n_pairs, uint64_t zone,
                                                                  uint64_t* __restrict__ cnt, uint32_t nwg) {
    __shared__ uint32_t lds[256];
    const uint64_t blk = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t key[8];
    stream_key(seeds, w, seed0 + blockIdx.y, key);
    uint32_t c = 0;
    if (blk * 8 < n_pairs) {
        uint32_t o[16];
        chacha_block(key, blk, o);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t v = ((uint64_t)o[2 * q] << 32) | o[2 * q + 1];
            c += (blk * 8 + q < n_pairs && v < zone) ? 1u : 0u;
        }
    }
    c = block_sum256(c, lds);
    if (threadIdx.x == 0) cnt[(uint64_t)blockIdx.y * nwg + blockIdx.x] = c;
}

// one workgroup per stream: exclusive scan of its nwg counts in place; tot[t] = accepted pairs
__global__ __launch_bounds__(256) void chacha_stream_scan_kernel(uint64_t* __restrict__ cnt, uint32_t nwg,
                                                                 uint64_t* __restrict__ tot) {
    __shared__ uint32_t lds[256];
    uint64_t* row = cnt + (uint64_t)blockIdx.x * nwg;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < nwg; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < nwg ? (uint32_t)row[i] : 0u;   // <= 2048 per workgroup
        const uint32_t ex = block_excl_scan256(v, lds);
        const uint32_t sum = block_sum256(v, lds);
        if (i < nwg) row[i] = carry + ex;
        carry += sum;
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

__global__ __launch_bounds__(256) void chacha_stream_scatter_kernel(const uint32_t* __restrict__ seeds, uint32_t w,
                                                                    uint64_t seed0, uint64_t n_pairs, uint64_t zone,
                                                                    Mod64 M, const uint64_t* __restrict__ off,
                                                                    uint32_t nwg, uint64_t D,
                                                                    int64_t* __restrict__ rows) {
    __shared__ uint32_t lds[256];
    const uint64_t blk = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t base = off[(uint64_t)blockIdx.y * nwg + blockIdx.x];
    if (base >= D) return;                                   // uniform: the whole workgroup is past D
    uint32_t key[8];
    stream_key(seeds, w, seed0 + blockIdx.y, key);
    uint32_t o[16];
    uint32_t flags = 0;
    if (blk * 8 < n_pairs) {
        chacha_block(key, blk, o);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t v = ((uint64_t)o[2 * q] << 32) | o[2 * q + 1];
            flags |= (blk * 8 + q < n_pairs && v < zone) ? (1u << q) : 0u;
        }
    }
    uint64_t pos = base + block_excl_scan256((uint32_t)__builtin_popcount(flags), lds);
    int64_t* row = rows + (uint64_t)blockIdx.y * D;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (flags & (1u << q)) {
            const uint64_t v = ((uint64_t)o[2 * q] << 32) | o[2 * q + 1];
            if (pos < D) row[pos] = (int64_t)umod64(v, M);
            ++pos;
        }
    }
}

}  // namespace

// ---- fast path: work layout [acc: D u64][count u64][seed_of: cap u32][pair_of: cap u64][rej upload: cap u64]
//      [pre: n_seeds ChachaPre, 64-byte aligned]
static constexpr uint64_t kRejectCap = 1 << 16;

static uint64_t chacha_pre_off(uint64_t D) { return (D * 8 + 16 + kRejectCap * (4 + 8 + 8) + 63) & ~(uint64_t)63; }

size_t chacha_work_bytes(uint64_t dimension, uint64_t n_seeds) {
    return chacha_pre_off(dimension) + n_seeds * sizeof(ChachaPre) + 64;
}

bool chacha_needs_stream_path(int64_t modulus) {
    const uint64_t m = (uint64_t)modulus;
    const uint64_t rejected = UINT64_MAX % m + 1;           // #{v : v >= zone}, zone = u64::MAX - u64::MAX % m
    return m > (1ull << 62) || rejected > (1ull << 36);    // signed (wrapping) sums, or > 2^-28 rejections
}

// ---- stream path: [rows: T x D i64][off: T x nwg u64][tot: T u64] ----
static uint64_t stream_pairs(uint64_t D, int64_t modulus, uint32_t slack_shift) {
    const double q = (double)(UINT64_MAX % (uint64_t)modulus + 1) / 18446744073709551616.0;
    const double extra = (double)D * q / (1.0 - q);
    uint64_t P = D + (uint64_t)(extra * 1.25 + 64.0 * __builtin_sqrt(extra + 1.0)) + 8192;
    P <<= slack_shift;                                      // retry: more pairs
    return (P + 7) & ~(uint64_t)7;
}
static uint64_t stream_tile(uint64_t D, uint64_t n_seeds) {
    uint64_t T = (512ull << 20) / (D * 8 + 1);              // ~512 MiB of draws per tile
    if (T < 1) T = 1;
    if (T > 1024) T = 1024;
    if (n_seeds && T > n_seeds) T = n_seeds;
    return T;
}
static uint32_t stream_nwg(uint64_t P) { return (uint32_t)((P / 8 + 255) / 256); }

// rows[t][0..D) = the draws of stream seed0 + t, t < T; `scratch` holds the scan (stream_scan_bytes).
// Host-synchronous: checks that every stream had D accepted pairs among the pairs it scanned, and
// rescans with more pairs if not.
static size_t stream_scan_bytes(uint64_t D, uint64_t T, int64_t modulus) {
    return T * (uint64_t)stream_nwg(stream_pairs(D, modulus, 2)) * 8 + T * 8 + 64;
}
static hipError_t expand_streams(int64_t modulus, uint64_t D, const uint32_t* seeds, uint32_t w, uint64_t seed0,
                                 uint64_t T, int64_t* rows, char* scratch, hipStream_t s) {
    const Mod64 M = make_mod64(modulus);
    const uint64_t zone = UINT64_MAX - UINT64_MAX % (uint64_t)modulus;
    for (uint32_t slack = 0; slack <= 2; ++slack) {
        const uint64_t P = stream_pairs(D, modulus, slack);
        const uint32_t nwg = stream_nwg(P);
        uint64_t* off = reinterpret_cast<uint64_t*>(scratch);
        uint64_t* tot = off + T * nwg;
        const dim3 grid(nwg, (unsigned)T);
        hipLaunchKernelGGL(chacha_stream_count_kernel, grid, dim3(256), 0, s, seeds, w, seed0, P, zone, off, nwg);
        hipLaunchKernelGGL(chacha_stream_scan_kernel, dim3((unsigned)T), dim3(256), 0, s, off, nwg, tot);
        hipLaunchKernelGGL(chacha_stream_scatter_kernel, grid, dim3(256), 0, s, seeds, w, seed0, P, zone, M, off, nwg,
                           D, rows);
        hipError_t e;
        if ((e = hipGetLastError()) != hipSuccess) return e;
        std::vector<uint64_t> got(T);
        if ((e = hipMemcpyAsync(got.data(), tot, T * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (*std::min_element(got.begin(), got.end()) >= D) return hipSuccess;
    }
    return hipErrorUnknown;    // 4x the expected pairs did not hold D accepted draws: practically impossible
}

size_t chacha_stream_work_bytes(uint64_t D, uint64_t n_seeds, int64_t modulus) {
    const uint64_t T = stream_tile(D, n_seeds);
    return T * D * 8 + stream_scan_bytes(D, T, modulus) + 256;
}

hipError_t launch_chacha_streams_combine(int64_t modulus, uint64_t D, const uint32_t* seeds, uint32_t w,
                                         uint64_t n_seeds, int64_t* out, void* work, hipStream_t s) {
    if (D == 0) return hipSuccess;
    if (n_seeds == 0) return hipMemsetAsync(out, 0, D * 8, s);            // chacha.rs:58 vec![0; dimension]
    const uint64_t T = stream_tile(D, n_seeds);
    int64_t* rows = static_cast<int64_t*>(work);
    char* scratch = static_cast<char*>(work) + ((T * D * 8 + 255) & ~(uint64_t)255);
    for (uint64_t s0 = 0; s0 < n_seeds; s0 += T) {
        const uint64_t t = n_seeds - s0 < T ? n_seeds - s0 : T;
        hipError_t e = expand_streams(modulus, D, seeds, w, s0, t, rows, scratch, s);
        if (e != hipSuccess) return e;
        // chacha.rs:68-72: r = (r + draw) % m over the seeds in order -- the exact combine recurrence,
        // wrapping i64 add included (m > 2^62 gives order-dependent signed sums, as in the reference)
        if ((e = launch_combine_exact(rows, t, D, D, out, modulus, s, s0 > 0)) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_chacha_stream(int64_t modulus, uint64_t D, const uint32_t* seed, uint32_t w, int64_t* mask,
                                void* work, hipStream_t s) {
    if (D == 0) return hipSuccess;
    return expand_streams(modulus, D, seed, w, 0, 1, mask, static_cast<char*>(work), s);
}

// Workgroups of 256 lanes of `kernel` resident at once on the current device: one full round of the
// grid.  Cached per (device, which) -- a process may drive devices of different sizes; a racing first
// call computes the same value twice, and the relaxed atomics make that benign.
static int resident_wgs(int which, const void* kernel) {
    static std::atomic<int> cache[64][4];
    int dev = 0;
    (void)hipGetDevice(&dev);
    int cap = (dev >= 0 && dev < 64) ? cache[dev][which].load(std::memory_order_relaxed) : 0;
    if (cap) return cap;
    int cus = 0, per_cu = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0);
    // the API can be one block per CU high at 81-96 SGPRs (MI355X_MICROARCH.md): also bound it by the
    // VGPR allocation (8-register granule, 512 per SIMD lane, 4 waves per block of 256)
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, kernel) == hipSuccess && fa.numRegs > 0) {
        const int by_vgpr = 512 / (((fa.numRegs + 7) / 8) * 8);
        if (by_vgpr < per_cu) per_cu = by_vgpr;
    }
    cap = (cus > 0 && per_cu > 0) ? cus * per_cu : 2048;
    if (dev >= 0 && dev < 64) cache[dev][which].store(cap, std::memory_order_relaxed);
    return cap;
}

// ---- fast path (counter mode + rejection log) ----
// Split in two so a pipeline can keep queueing work behind the combine: chacha_fast_enqueue launches it
// (canonical results land in `out`) and copies the rejection count to `count_host` (pinned); once the
// stream has drained, chacha_fast_resolve applies the fix-ups for that count (rare: each draw is
// rejected with probability < 2^-28 on this path) or reports a log overflow (the caller then runs the
// stream path).
// secrets != nullptr (one seed): out = (secrets + draw) % m, the masked secrets (chacha_mask_add_kernel).
static hipError_t chacha_fast_enqueue(int64_t modulus, uint64_t D, const uint32_t* seeds_dev, uint32_t w,
                                      uint64_t n_seeds, int64_t* out, void* work, hipStream_t s,
                                      unsigned long long* count_host, const int64_t* secrets = nullptr) {
    const Mod64 M = make_mod64(modulus);
    const uint64_t zone = UINT64_MAX - UINT64_MAX % (uint64_t)modulus;
    char* base = static_cast<char*>(work);
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(base);
    unsigned long long* count = reinterpret_cast<unsigned long long*>(base + D * 8);
    uint32_t* seed_of = reinterpret_cast<uint32_t*>(base + D * 8 + 16);
    uint64_t* pair_of = reinterpret_cast<uint64_t*>(base + D * 8 + 16 + kRejectCap * 4);
    hipError_t e;
    const uint64_t n_blk = (D + 7) / 8;
    const uint64_t gx = (n_blk + 255) / 256;
    const uint64_t mm = (uint64_t)modulus;
    const bool lazy = mm <= (1ull << 32);
    // Seeds split over grid.y chunks until the grid holds one full round of resident workgroups (the
    // kernel is VALU-bound: more chunks only add atomic merges -- A/B in profiles/r02/ab_chacha.txt).
    // The u64 accumulators receive one canonical partial (< m) per chunk (headroom).
    const int cap_wgs = lazy ? resident_wgs(0, reinterpret_cast<const void*>(chacha_combine_kernel<true, false, true>))
                             : resident_wgs(1, reinterpret_cast<const void*>(chacha_combine_kernel<false, false, true>));
    const int cap_sk = lazy ? resident_wgs(2, reinterpret_cast<const void*>(chacha_combine_sk_kernel<true, true>))
                            : resident_wgs(3, reinterpret_cast<const void*>(chacha_combine_sk_kernel<false, true>));
    uint64_t max_c = n_seeds ? n_seeds : 1;
    if (max_c > 65535) max_c = 65535;
    if (M.m > 1 && max_c > UINT64_MAX / (M.m - 1)) max_c = UINT64_MAX / (M.m - 1);
    uint64_t chunks = ((uint64_t)cap_wgs + gx - 1) / gx;
    if (chunks > max_c) chunks = max_c;
    const char* ce = getenv("SDA_CHACHA_CHUNKS");                 // A/B knob: the chunked grid, c chunks
    if (ce) {
        const uint64_t c = strtoull(ce, nullptr, 10);
        if (c >= 1 && c <= max_c) chunks = c;
    }
    if (secrets) chunks = 1;                     // one stream: its own grid, no accumulator
    // Stream-K (chacha_combine_sk_kernel) when the chunked grid leaves a partial last round of workgroups
    // (< 95 % of its rounds' slots busy) and every tile's runs fit the u64 accumulator's headroom.
    const uint64_t units = gx * n_seeds, G = units < (uint64_t)cap_sk ? units : (uint64_t)cap_sk;
    const uint64_t chunk_wgs = gx * chunks, rounds = (chunk_wgs + cap_wgs - 1) / cap_wgs;
    const uint64_t per_wg = G ? units / G : 0;
    const uint64_t runs_per_tile = per_wg ? (n_seeds + per_wg - 1) / per_wg + 1 : UINT64_MAX;
    const char* ske = getenv("SDA_CHACHA_SK");                    // A/B knob: "0" = the chunked grid
    const bool sk = !secrets && !ce && !(ske && ske[0] == '0') && n_seeds && G && runs_per_tile <= max_c &&
                    (double)chunk_wgs < 0.95 * (double)(rounds * (uint64_t)cap_wgs);
    if (sk) chunks = 2;                          // not direct: acc is zeroed, merged and reduced below
    const uint64_t per = n_seeds ? (n_seeds + chunks - 1) / chunks : 0;
    const bool direct = chunks == 1;             // results stored straight into `out`
    unsigned long long* dst = direct ? reinterpret_cast<unsigned long long*>(out) : acc;
    if ((e = hipMemsetAsync(count, 0, 16, s)) != hipSuccess) return e;
    if (!direct && (e = hipMemsetAsync(acc, 0, D * 8, s)) != hipSuccess) return e;
    RejectLog log{count, seed_of, pair_of, kRejectCap};
    const dim3 grid((unsigned)gx, (unsigned)chunks);
    const uint64_t r64 = lazy ? (UINT64_MAX % mm + 1) % mm : 0;          // 2^64 mod m
    // round 1's uniform columns per seed, once (every block counter's high word is 0 below 2^32 blocks)
    ChachaPre* pre = reinterpret_cast<ChachaPre*>(base + chacha_pre_off(D));
    const bool use_pre = !secrets && n_seeds && n_blk <= (1ull << 32);
    if (use_pre) {
        hipLaunchKernelGGL(chacha_pre_kernel, dim3((unsigned)((n_seeds + 255) / 256)), dim3(256), 0, s, seeds_dev, w,
                           n_seeds, pre);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
#define SDA_CHACHA_LAUNCH(L, DI)                                                                              \
    do {                                                                                                      \
        if (use_pre)                                                                                          \
            hipLaunchKernelGGL((chacha_combine_kernel<L, DI, true>), grid, dim3(256), 0, s, seeds_dev, w,     \
                               n_seeds, per, D, dst, M, zone, r64, log, (const ChachaPre*)pre);               \
        else                                                                                                  \
            hipLaunchKernelGGL((chacha_combine_kernel<L, DI>), grid, dim3(256), 0, s, seeds_dev, w, n_seeds,  \
                               per, D, dst, M, zone, r64, log, (const ChachaPre*)nullptr);                    \
    } while (0)
    const bool small_m = mm <= (1ull << 62);
    if (sk) {
        const uint64_t q = units / G, r = units % G;
        if (lazy && use_pre)
            hipLaunchKernelGGL((chacha_combine_sk_kernel<true, true>), dim3((unsigned)G), dim3(256), 0, s, seeds_dev, w,
                               n_seeds, q, r, D, acc, M, zone, r64, log, (const ChachaPre*)pre);
        else if (lazy)
            hipLaunchKernelGGL((chacha_combine_sk_kernel<true, false>), dim3((unsigned)G), dim3(256), 0, s, seeds_dev, w,
                               n_seeds, q, r, D, acc, M, zone, r64, log, (const ChachaPre*)nullptr);
        else if (use_pre)
            hipLaunchKernelGGL((chacha_combine_sk_kernel<false, true>), dim3((unsigned)G), dim3(256), 0, s, seeds_dev, w,
                               n_seeds, q, r, D, acc, M, zone, r64, log, (const ChachaPre*)pre);
        else
            hipLaunchKernelGGL((chacha_combine_sk_kernel<false, false>), dim3((unsigned)G), dim3(256), 0, s, seeds_dev, w,
                               n_seeds, q, r, D, acc, M, zone, r64, log, (const ChachaPre*)nullptr);
    } else if (secrets)
        hipLaunchKernelGGL(chacha_mask_add_kernel, dim3((unsigned)gx), dim3(256), 0, s, seeds_dev, w, D, dst, M, zone,
                           log, secrets, small_m);
    else if (lazy && direct) SDA_CHACHA_LAUNCH(true, true);
    else if (lazy) SDA_CHACHA_LAUNCH(true, false);
    else if (direct) SDA_CHACHA_LAUNCH(false, true);
    else SDA_CHACHA_LAUNCH(false, false);
#undef SDA_CHACHA_LAUNCH
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (!direct) {     // canonical residues into out (the fix-ups, if any, then work on out modulo m)
        hipLaunchKernelGGL(acc_mod_kernel, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, s, acc, D, out, M);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipMemcpyAsync(count_host, count, 8, hipMemcpyDeviceToHost, s);
}

static hipError_t chacha_fast_resolve(int64_t modulus, uint64_t D, const uint32_t* seeds_dev, uint32_t w,
                                      uint64_t n_seeds, int64_t* out, void* work, hipStream_t s,
                                      unsigned long long n_rej, bool* overflow, int* fixups_out) {
    if (n_rej == 0) return hipSuccess;
    if (n_rej > kRejectCap) {          // the caller reruns the job on the stream path
        *overflow = true;
        return hipSuccess;
    }
    const Mod64 M = make_mod64(modulus);
    const uint64_t zone = UINT64_MAX - UINT64_MAX % (uint64_t)modulus;
    char* base = static_cast<char*>(work);
    uint32_t* seed_of = reinterpret_cast<uint32_t*>(base + D * 8 + 16);
    uint64_t* pair_of = reinterpret_cast<uint64_t*>(base + D * 8 + 16 + kRejectCap * 4);
    uint64_t* rej_up = pair_of + kRejectCap;
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(out);   // canonical sums of the draws
    hipError_t e;
    std::vector<uint32_t> so(n_rej);
    std::vector<uint64_t> po(n_rej);
    std::vector<uint32_t> seeds_host((size_t)n_seeds * w);     // only now: keys of the affected streams
    if ((e = hipMemcpy(so.data(), seed_of, n_rej * 4, hipMemcpyDeviceToHost)) != hipSuccess) return e;
    if ((e = hipMemcpy(po.data(), pair_of, n_rej * 8, hipMemcpyDeviceToHost)) != hipSuccess) return e;
    if ((e = hipMemcpy(seeds_host.data(), seeds_dev, seeds_host.size() * 4, hipMemcpyDeviceToHost)) != hipSuccess)
        return e;
    std::vector<std::pair<uint32_t, uint64_t>> ev(n_rej);
    for (size_t i = 0; i < n_rej; ++i) ev[i] = {so[i], po[i]};
    std::sort(ev.begin(), ev.end());
    const uint32_t nw = w < 8 ? w : 8;
    size_t i = 0;
    while (i < ev.size()) {
        const uint32_t sd = ev[i].first;
        std::vector<uint64_t> rej;
        while (i < ev.size() && ev[i].first == sd) rej.push_back(ev[i++].second);
        Key8 key{};
        for (uint32_t q = 0; q < nw; ++q) key.k[q] = seeds_host[(size_t)sd * w + q];
        // extend past D: pairs D .. D + |rej| - 1 (+ any further rejections there)
        uint64_t scanned = D;
        while (scanned < D + rej.size()) {
            const uint64_t v = h_pair(key.k, scanned);
            if (v >= zone) rej.push_back(scanned);
            ++scanned;
        }
        if (rej.size() > kRejectCap) {
            *overflow = true;
            return hipSuccess;
        }
        if ((e = hipMemcpy(rej_up, rej.data(), rej.size() * 8, hipMemcpyHostToDevice)) != hipSuccess) return e;
        const uint64_t i0 = rej.front();
        const uint64_t nfix = D - i0;
        hipLaunchKernelGGL(chacha_fix_kernel, dim3((unsigned)((nfix + 255) / 256)), dim3(256), 0, s, key, i0, D,
                           rej_up, (uint32_t)rej.size(), acc, M);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;   // rej_up is reused
        if (fixups_out) ++*fixups_out;
    }
    return hipSuccess;
}

hipError_t launch_chacha_mask_combine(int64_t modulus, uint64_t dimension, const uint32_t* seeds, uint32_t w,
                                      uint64_t n_seeds, int64_t* out, void* work, hipStream_t s, bool* overflow,
                                      int* fixups_out) {
    *overflow = false;
    if (fixups_out) *fixups_out = 0;
    if (dimension == 0) return hipSuccess;
    unsigned long long n_rej = 0;      // pageable: the copy completes before the sync returns
    hipError_t e = chacha_fast_enqueue(modulus, dimension, seeds, w, n_seeds, out, work, s, &n_rej);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    return chacha_fast_resolve(modulus, dimension, seeds, w, n_seeds, out, work, s, n_rej, overflow, fixups_out);
}

hipError_t launch_chacha_mask_combine_async(int64_t modulus, uint64_t dimension, const uint32_t* seeds, uint32_t w,
                                            uint64_t n_seeds, int64_t* out, void* work, hipStream_t s,
                                            unsigned long long* count_host) {
    *count_host = 0;
    if (dimension == 0) return hipSuccess;
    return chacha_fast_enqueue(modulus, dimension, seeds, w, n_seeds, out, work, s, count_host);
}

hipError_t launch_chacha_mask_add_async(int64_t modulus, uint64_t dimension, const uint32_t* seed, uint32_t w,
                                        const int64_t* secrets, int64_t* masked, void* work, hipStream_t s,
                                        unsigned long long* count_host) {
    *count_host = 0;
    if (dimension == 0) return hipSuccess;
    return chacha_fast_enqueue(modulus, dimension, seed, w, 1, masked, work, s, count_host, secrets);
}

hipError_t resolve_chacha_mask_combine(int64_t modulus, uint64_t dimension, const uint32_t* seeds, uint32_t w,
                                       uint64_t n_seeds, int64_t* out, void* work, hipStream_t s,
                                       unsigned long long n_rej, bool* overflow, int* fixups_out) {
    *overflow = false;
    if (fixups_out) *fixups_out = 0;
    if (dimension == 0) return hipSuccess;
    return chacha_fast_resolve(modulus, dimension, seeds, w, n_seeds, out, work, s, n_rej, overflow, fixups_out);
}

}  // namespace sda
