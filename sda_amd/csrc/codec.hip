// codec.hip -- share payload codec on gfx950.
//
// Reference: client/src/crypto/encryption/sodium.rs
//   encrypt (:36-41):  for share in shares { size = share.encode_var(&mut buf); bytes.extend(&buf[..size]) }
//   decrypt (:82-88):  while reader.len() > 0 { (i, size) = Share::decode_var(reader); push(i); reader = &reader[size..] }
// with integer-encoding 1.0 VarInt for i64 (third-party, absent from the tree): zigzag
// z = (v << 1) ^ (v >> 63), then LEB128 (7 bits per byte, low group first, 0x80 = "more").
// u64::decode_var stops at the first byte without 0x80 or once shift > 70, so a run of >= 11
// continuation bytes forms an 11-byte element whose 11th group lands at shift 70 & 63 (Rust
// release semantics), and a truncated final varint yields its partial value.
//
// The clerk decrypts N participations (sodium stays on the host) and combines them
// (clerk.rs:79-86).  On the device the blobs are one concatenated byte stream; decoding is a
// stream compaction over terminator bytes (b & 0x80 == 0), in ONE pass over the payload: a
// workgroup takes the next 16 KiB aligned region of a blob (regions handed out in blob order by an
// atomic ticket), stages it (plus a 16-byte halo) in LDS, counts its terminators and flags runs of
// >= 11 continuation bytes, publishes the count, takes its element base from a decoupled look-back
// over the blob's earlier regions, and decodes: each terminator byte decodes the <= 10-byte varint
// that ends at it (its start is the previous terminator, within the halo) into out[blob][index].
// Blobs flagged irregular (malformed streams) are redone afterwards by a sequential exact kernel.
// Encoding is the mirror image: a workgroup takes the next 2048-value chunk (rows back to back),
// sizes its varints, looks back for its byte offset, and writes the bytes assembled in LDS.
// Roofline: HBM.  Algorithmic bytes = payload bytes read + 8 B per decoded element written.
#include "kernels.h"

namespace sda {

namespace {

constexpr int kThreads = 256;
constexpr int kWPT = 4;                       // 16-byte words per thread: word t + 256 k, k < kWPT
constexpr uint64_t kSubBytes = kThreads * 16; // one sub-region = one word per thread
constexpr uint64_t kRegionBytes = kSubBytes * kWPT;



// 16 bytes as a 16-bit mask of "continuation" bytes (bit j = byte j has 0x80).
__device__ __forceinline__ uint32_t cont_mask(uint4 w) {
    uint32_t m = 0;
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t hb = d[q] & 0x80808080u;
        // gather bits 7, 15, 23, 31 into bits 0..3
        const uint32_t g = (hb >> 7) | (hb >> 14) | (hb >> 21) | (hb >> 28);
        m |= (g & 0xFu) << (4 * q);
    }
    return m;
}

__device__ __forceinline__ uint8_t byte_of(const uint4& w, int j) {
    const uint32_t d = j < 4 ? w.x : (j < 8 ? w.y : (j < 12 ? w.z : w.w));
    return (uint8_t)(d >> (8 * (j & 3)));
}

// The region word this thread owns and its 32-byte window (previous word + own word):
//   valid  bit j (16..31): window byte j is inside the blob
//   term   bit j: a terminator (no 0x80) inside the blob, or the blob's last byte (truncated tail)
//   cont   bit j: a continuation byte inside the blob (bytes outside the blob count as neither)
struct Window {
    uint4 prev, own;
    uint32_t valid, term, cont;
};

__device__ __forceinline__ Window make_window(uint4 prev, uint4 own, uint64_t word, uint64_t begin, uint64_t end) {
    Window W;
    const uint64_t a0 = word * 16;                      // byte offset of own word (aligned)
    W.own = own;
    W.prev = prev;
    const uint32_t cm = cont_mask(W.prev) | (cont_mask(W.own) << 16);
    // window byte j sits at a0 - 16 + j
    uint32_t in = 0;
    {
        const int64_t lo = (int64_t)begin - (int64_t)(a0 - 16);   // first valid window index
        const int64_t hi = (int64_t)end - (int64_t)(a0 - 16);     // one past last
        const int l = lo < 0 ? 0 : (lo > 32 ? 32 : (int)lo);
        const int h = hi < 0 ? 0 : (hi > 32 ? 32 : (int)hi);
        if (h > l) in = (h - l == 32 ? 0xFFFFFFFFu : ((1u << (h - l)) - 1u)) << l;
        W.valid = in & 0xFFFF0000u;
        uint32_t lastbit = 0;
        if (hi >= 1 && hi <= 32) lastbit = 1u << (hi - 1);      // the blob's last byte is in the window
        W.cont = cm & in;
        W.term = (~cm & in) | (lastbit & in);
    }
    return W;
}

// ---- decoupled look-back: one status word per item, flag in the top 2 bits, value below ----
constexpr unsigned long long kAggReady = 1ull << 62, kIncReady = 2ull << 62, kValMask = (1ull << 62) - 1;

// The status words carry only counts (nothing else is published through them), so relaxed
// agent-scope atomics suffice: a release here would write back the whole L2 of the XCD before
// every publication, an acquire would invalidate it after every poll.
__device__ __forceinline__ void lb_publish(unsigned long long* st, unsigned long long v) {
    __hip_atomic_store(st, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of item i over items [first, i), computed by one whole wave (wave 0 of the
// workgroup, every lane calls it; the result is uniform): each step reads the status words of the
// 64 preceding items at once (relaxed agent-scope atomic loads, one per lane), waits until each has
// at least its aggregate, and sums back to the nearest inclusive prefix -- or over all 64 and steps
// another 64 back.  Item `first` publishes its inclusive value at once, so the walk ends there at the
// latest.  Every predecessor holds an earlier ticket, so it is running or done; the spin is bounded
// all the same (err flag).
__device__ uint64_t lb_exclusive(unsigned long long* status, uint64_t i, uint64_t first, unsigned int* err) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t excl = 0;
    uint64_t end = i;                                         // this window: items [end - 64, end)
    while (end > first) {
        const bool valid = end - first > lane;                // item end - 1 - lane >= first
        const uint64_t j = end - 1 - lane;
        unsigned long long v = 0;
        if (valid) {
            uint32_t spins = 0;
            while (((v = __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 62) == 0) {
                if (++spins > (1u << 22)) {
                    atomicOr(err, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        const uint64_t inc = __ballot(valid && (v >> 62) == 2);
        const uint32_t stop = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;    // nearest inclusive predecessor
        uint64_t c = (valid && lane <= stop) ? (v & kValMask) : 0;
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        excl += c;
        if (inc) break;
        end = end - first > 64 ? end - 64 : first;
    }
    return excl;
}

__device__ __forceinline__ uint32_t block_sum(uint32_t n, uint32_t* red) {
    for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
    __syncthreads();
    uint32_t s = 0;
    for (int i = 0; i < kThreads / 64; ++i) s += red[i];
    __syncthreads();
    return s;
}

// 7-bit groups of the (zero-padded past the element) little-endian bytes of `x`, packed:
// group i -> bits 7i..7i+6  (LEB128 payload of up to 8 bytes).
__device__ __forceinline__ uint64_t leb_pack8(uint64_t x) {
    x &= 0x7F7F7F7F7F7F7F7Full;
    x = (x & 0x007F007F007F007Full) | ((x & 0x7F007F007F007F00ull) >> 1);
    x = (x & 0x00003FFF00003FFFull) | ((x & 0x3FFF00003FFF0000ull) >> 2);
    x = (x & 0x000000000FFFFFFFull) | ((x & 0x0FFFFFFF00000000ull) >> 4);
    return x;
}

constexpr uint32_t kTileRegions = 8;          // regions per decode workgroup (128 KiB of payload)

// One pass over the payload: a workgroup takes the next tile of up to kTileRegions consecutive
// regions of one blob (atomic ticket; tiles numbered blob by blob, [blob_tile[b], blob_tile[b+1])
// for blob b), counts the tile's terminators (and flags runs of >= 11 continuation bytes: irregular
// blob), publishes the count, gets its element base from the look-back over the blob's earlier
// tiles, and decodes region by region: stage the region and the 16-byte halo before it in LDS (the
// second read of those bytes, from the caches); per sub-region (one word per thread) a block-wide
// scan of the terminator counts compacts the elements' (start, length) into LDS; then lane i
// decodes element i (balanced work, coalesced stores) from three funnel-shifted dwords.  Big tiles
// keep the look-back chain short (one status word per 128 KiB).  Values at index >= out_stride are
// counted, not stored.
__global__ __launch_bounds__(kThreads) void varint_decode_kernel(const uint8_t* __restrict__ bytes,
                                                                 const uint64_t* __restrict__ blob_tile,
                                                                 const uint64_t* __restrict__ blob_off, uint64_t n_blobs,
                                                                 unsigned long long* __restrict__ status,
                                                                 unsigned int* __restrict__ ticket,
                                                                 uint32_t* __restrict__ blob_irregular,
                                                                 uint64_t* __restrict__ blob_count,
                                                                 unsigned int* __restrict__ err,
                                                                 int64_t* __restrict__ out, uint64_t out_stride) {
    __shared__ uint32_t lb[(kRegionBytes + 32) / 4];          // [halo 16 B | region 16 KiB | tail 16 B]
    __shared__ uint32_t wsum[kThreads / 64];
    __shared__ uint32_t el[kSubBytes];                        // one sub-region's elements: start | len << 16
    __shared__ uint32_t rcount[kTileRegions];
    __shared__ uint64_t sh[3];
    if (threadIdx.x == 0) {
        const uint64_t t = atomicAdd(ticket, 1u);
        uint64_t lo = 0, hi = n_blobs;                        // the last blob whose first tile is <= t
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) / 2;
            if (blob_tile[mid] <= t) lo = mid; else hi = mid;
        }
        sh[0] = t;
        sh[1] = lo;
    }
    __syncthreads();
    const uint64_t t = sh[0], b = sh[1];
    const uint64_t first = blob_tile[b], last = blob_tile[b + 1] - 1;
    const uint64_t begin = blob_off[b], end = blob_off[b + 1];
    const uint64_t r0 = begin / kRegionBytes + (t - first) * kTileRegions;   // first region (buffer-aligned)
    const uint64_t r_end = (end - 1) / kRegionBytes + 1;
    const uint32_t nreg = (uint32_t)(r_end - r0 < kTileRegions ? r_end - r0 : kTileRegions);
    const uint4* p = reinterpret_cast<const uint4*>(bytes);

    // ---- phase 1: terminator count per region, irregular runs ----
    uint32_t bad = 0;
    for (uint32_t k = 0; k < nreg; ++k) {
        const uint64_t word = (r0 + k) * (kRegionBytes / 16);
        uint4 v[kWPT];
#pragma unroll
        for (int q = 0; q < kWPT; ++q) {
            const uint64_t wk = word + threadIdx.x + q * kThreads;
            v[q] = wk * 16 < end ? p[wk] : make_uint4(0, 0, 0, 0);
        }
        // continuation masks of the words (LDS: lb as u32 scratch), slot 0 = the word before the region
        if (threadIdx.x == 0) {
            const uint4 halo = word * 16 > begin ? p[word - 1] : make_uint4(0, 0, 0, 0);
            lb[0] = make_window(make_uint4(0, 0, 0, 0), halo, word - 1, begin, end).cont >> 16;
        }
        Window W[kWPT];
        uint32_t n = 0;
#pragma unroll
        for (int q = 0; q < kWPT; ++q) {
            const uint32_t wl = threadIdx.x + q * kThreads;
            W[q] = make_window(make_uint4(0, 0, 0, 0), v[q], word + wl, begin, end);   // own-word masks only
            lb[wl + 1] = W[q].cont >> 16;
            n += __builtin_popcount(W[q].term & W[q].valid);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kWPT; ++q) {
            const uint32_t wl = threadIdx.x + q * kThreads;
            const uint32_t cont = W[q].cont | lb[wl];        // 11 continuation bytes ending in this word?
            uint32_t run = cont;
#pragma unroll
            for (int z = 1; z <= 10; ++z) run &= cont << z;
            bad |= run & W[q].valid;
        }
        const uint32_t c = block_sum(n, wsum);               // (its barriers also free lb)
        if (threadIdx.x == 0) rcount[k] = c;
    }
    if (bad) atomicOr(&blob_irregular[b], 1u);
    __syncthreads();
    uint32_t agg = 0;
    for (uint32_t k = 0; k < nreg; ++k) agg += rcount[k];
    if (threadIdx.x < 64) {                                   // wave 0: publish, look back, publish
        uint64_t excl = 0;
        if (t == first) {
            if (threadIdx.x == 0) lb_publish(status + t, kIncReady | agg);
        } else {
            if (threadIdx.x == 0) lb_publish(status + t, kAggReady | agg);
            excl = lb_exclusive(status, t, first, err);
            if (threadIdx.x == 0) lb_publish(status + t, kIncReady | (excl + agg));
        }
        if (threadIdx.x == 0) {
            if (t == last) blob_count[b] = excl + agg;
            sh[2] = excl;
        }
    }
    __syncthreads();

    // ---- phase 2: decode region by region ----
    int64_t* dst = out + b * out_stride;
    uint64_t base = sh[2];                                    // elements before this region / sub-region
    for (uint32_t kr = 0; kr < nreg; ++kr) {
        const uint64_t word = (r0 + kr) * (kRegionBytes / 16);
        {
            uint4 v[kWPT];
#pragma unroll
            for (int k = 0; k < kWPT; ++k) {
                const uint64_t wk = word + threadIdx.x + k * kThreads;
                v[k] = wk * 16 < end ? p[wk] : make_uint4(0, 0, 0, 0);
            }
            if (threadIdx.x == 0)
                reinterpret_cast<uint4*>(lb)[0] = (word * 16 > begin) ? p[word - 1] : make_uint4(0, 0, 0, 0);
            if (threadIdx.x == kThreads - 1) reinterpret_cast<uint4*>(lb)[kWPT * kThreads + 1] = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k < kWPT; ++k) reinterpret_cast<uint4*>(lb)[threadIdx.x + k * kThreads + 1] = v[k];
        }
        __syncthreads();
        Window W[kWPT];
#pragma unroll
        for (int k = 0; k < kWPT; ++k) {
            const uint32_t wl = threadIdx.x + k * kThreads;
            W[k] = make_window(reinterpret_cast<const uint4*>(lb)[wl], reinterpret_cast<const uint4*>(lb)[wl + 1],
                               word + wl, begin, end);
        }
#pragma unroll
        for (int k = 0; k < kWPT; ++k) {
            // 1. compaction: each thread lists the (start, length) of the elements ending in its word
            const uint32_t tm = W[k].term & W[k].valid;
            const uint32_t nk = __builtin_popcount(tm);
            uint32_t incl = nk;                               // exclusive scan of nk over the block
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t tt = __shfl_up(incl, o);
                if ((threadIdx.x & 63) >= (uint32_t)o) incl += tt;
            }
            __syncthreads();                                  // el / wsum free for reuse
            if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
            __syncthreads();
            uint32_t e = incl - nk, total = 0;
            for (uint32_t w = 0; w < kThreads / 64; ++w) {
                if (w < (threadIdx.x >> 6)) e += wsum[w];
                total += wsum[w];
            }
            // an element starts after the previous boundary (a terminator or a byte outside the blob)
            const uint32_t boundary = W[k].term | ~(W[k].term | W[k].cont);
            uint32_t rem = tm;
            while (rem) {
                const int j = __builtin_ctz(rem);
                rem &= rem - 1;
                const uint32_t below = boundary & ((1u << j) - 1u);
                const int st = below ? 32 - __builtin_clz(below) : 0;      // window index of the first byte
                el[e++] = ((threadIdx.x + k * kThreads) * 16 + st) | ((uint32_t)(j - st + 1) << 16);
            }
            __syncthreads();
            // 2. decode: lane i takes element i -> balanced work, coalesced stores
            for (uint32_t i = threadIdx.x; i < total; i += kThreads) {
                if (base + i >= out_stride) break;
                const uint32_t P = el[i] & 0xFFFFu;              // byte position in lb
                const int len = (int)(el[i] >> 16);               // 1..11 on regular blobs
                const uint32_t q = P >> 2, sh8 = (P & 3) * 8;
                const uint32_t d0 = lb[q], d1 = lb[q + 1], d2 = lb[q + 2], d3 = lb[q + 3];
                const uint32_t b0 = __builtin_amdgcn_alignbit(d1, d0, sh8), b1 = __builtin_amdgcn_alignbit(d2, d1, sh8),
                               b2 = __builtin_amdgcn_alignbit(d3, d2, sh8);
                uint64_t lo = ((uint64_t)b1 << 32) | b0;
                if (len < 8) lo &= (1ull << (8 * len)) - 1;
                uint64_t z = leb_pack8(lo);
                if (len > 8) {          // groups 8, 9, 10 at shifts 56, 63, 70 & 63 = 6 (Rust release)
                    const uint32_t hb = b2 & ((len >= 11) ? 0xFFFFFFu : (len == 10 ? 0xFFFFu : 0xFFu));
                    z |= ((uint64_t)(hb & 0x7F) << 56) | ((uint64_t)((hb >> 8) & 0x7F) << 63) |
                         ((uint64_t)((hb >> 16) & 0x7F) << 6);
                }
                dst[base + i] = (int64_t)((z >> 1) ^ (0 - (z & 1)));
            }
            base += total;
        }
        __syncthreads();                                      // lb is restaged for the next region
    }
}

// Irregular blobs: the reference loop, one lane per blob (only malformed streams get here); it
// rewrites the blob's row (values past `cap` are counted, not stored) and its count.
__global__ void varint_sequential_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ blob_off,
                                         uint32_t n_blobs, const uint32_t* __restrict__ blob_irregular,
                                         uint64_t* __restrict__ blob_count, int64_t* __restrict__ out,
                                         uint64_t out_stride, uint64_t cap) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_blobs || !blob_irregular[b]) return;
    uint64_t r = blob_off[b];
    const uint64_t e = blob_off[b + 1];
    uint64_t c = 0;
    while (r < e) {
        uint64_t z = 0;
        unsigned shift = 0;
        while (r < e) {
            const uint8_t by = bytes[r++];
            z |= (uint64_t)(by & 0x7f) << (shift & 63);
            shift += 7;
            if (!(by & 0x80) || shift > 70) break;
        }
        if (c < cap) out[(uint64_t)b * out_stride + c] = (int64_t)((z >> 1) ^ (0 - (z & 1)));
        ++c;
    }
    blob_count[b] = c;
}

// ---------------- encode ----------------
__device__ __forceinline__ uint32_t varint_size(int64_t v) {
    const uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
    const int bits = 64 - __builtin_clzll(z | 1);
    return (uint32_t)((bits + 6) / 7);
}

constexpr uint32_t kEncChunk = 2048;          // elements per encode block
constexpr uint32_t kEncPer = kEncChunk / kThreads;

// inverse of leb_pack8: 7-bit groups of z -> bytes (group i in byte i), continuation bits not set
__device__ __forceinline__ uint64_t leb_spread8(uint64_t z) {
    uint64_t x = z & 0x00FFFFFFFFFFFFFFull;
    x = (x & 0x000000000FFFFFFFull) | ((x & 0x00FFFFFFF0000000ull) << 4);
    x = (x & 0x00003FFF00003FFFull) | ((x & 0x0FFFC0000FFFC000ull) << 2);
    x = (x & 0x007F007F007F007Full) | ((x & 0x3F803F803F803F80ull) << 1);
    return x;
}

constexpr uint32_t kEncTileChunks = 8;        // chunks per encode workgroup (16384 values)

// One pass: a workgroup takes the next tile of up to 8 chunks of 2048 values (atomic ticket; tiles
// numbered row by row, and the rows' payloads lie back to back), sizes the tile's varints (first
// read of the values), gets the tile's byte offset from the look-back over all earlier tiles, then
// per chunk reloads the values (from the caches), assembles the bytes in LDS at the chunk's offset
// mod 4 (so LDS dwords line up with global dwords) and writes dwords for the interior, bytes for
// the two partial ends (shared with the neighbouring chunks).  Bytes at or past dst_cap are not
// written; row_end[row] = end offset of the row (its last tile writes it).
__global__ __launch_bounds__(kThreads) void varint_encode_kernel(const int64_t* __restrict__ vals, uint64_t len,
                                                                 uint64_t stride, uint64_t tiles_per_row,
                                                                 unsigned long long* __restrict__ status,
                                                                 unsigned int* __restrict__ ticket,
                                                                 uint64_t* __restrict__ row_end,
                                                                 unsigned int* __restrict__ err,
                                                                 uint8_t* __restrict__ dst, uint64_t dst_cap) {
    __shared__ uint32_t buf[(kEncChunk * 10 + 8) / 4];
    __shared__ uint32_t wsum[kThreads / 64];
    __shared__ uint32_t cbytes[kEncTileChunks];
    __shared__ uint64_t sh[2];
    if (threadIdx.x == 0) sh[0] = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint64_t t = sh[0];
    const uint64_t row = t / tiles_per_row, x = t - row * tiles_per_row;
    const int64_t* rv = vals + row * stride;
    const uint64_t c0 = x * kEncTileChunks, n_chunks = (len + kEncChunk - 1) / kEncChunk;
    const uint32_t nc = (uint32_t)(n_chunks - c0 < kEncTileChunks ? n_chunks - c0 : kEncTileChunks);
    // ---- phase 1: bytes per chunk ----
    for (uint32_t k = 0; k < nc; ++k) {
        const uint64_t e0 = (c0 + k) * kEncChunk;
        uint32_t mine = 0;
#pragma unroll
        for (uint32_t q = 0; q < kEncPer; ++q) {
            const uint64_t e = e0 + q * kThreads + threadIdx.x;
            mine += e < len ? varint_size(rv[e]) : 0u;
        }
        const uint32_t cb = block_sum(mine, wsum);
        if (threadIdx.x == 0) cbytes[k] = cb;
    }
    __syncthreads();
    uint32_t agg = 0;
    for (uint32_t k = 0; k < nc; ++k) agg += cbytes[k];
    if (threadIdx.x < 64) {                                   // wave 0: publish, look back, publish
        uint64_t excl = 0;
        if (t == 0) {
            if (threadIdx.x == 0) lb_publish(status, kIncReady | agg);
        } else {
            if (threadIdx.x == 0) lb_publish(status + t, kAggReady | agg);
            excl = lb_exclusive(status, t, 0, err);
            if (threadIdx.x == 0) lb_publish(status + t, kIncReady | (excl + agg));
        }
        if (threadIdx.x == 0) {
            if (x + 1 == tiles_per_row) row_end[row] = excl + agg;
            sh[1] = excl;
        }
    }
    __syncthreads();
    // ---- phase 2: write chunk by chunk ----
    uint64_t go = sh[1];
    uint8_t* b8 = reinterpret_cast<uint8_t*>(buf);
    for (uint32_t k = 0; k < nc; ++k) {
        const uint64_t e0 = (c0 + k) * kEncChunk;
        int64_t v[kEncPer];
        uint32_t n[kEncPer];
#pragma unroll
        for (uint32_t q = 0; q < kEncPer; ++q) {
            const uint64_t e = e0 + q * kThreads + threadIdx.x;
            v[q] = e < len ? rv[e] : 0;
            n[q] = e < len ? varint_size(v[q]) : 0u;
        }
        const uint32_t lead = (uint32_t)(go & 3);
        uint32_t base = lead;
#pragma unroll
        for (uint32_t q = 0; q < kEncPer; ++q) {
            const uint64_t z = ((uint64_t)v[q] << 1) ^ (uint64_t)(v[q] >> 63);
            uint32_t incl = n[q];
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t tt = __shfl_up(incl, o);
                if ((threadIdx.x & 63) >= (uint32_t)o) incl += tt;
            }
            __syncthreads();                                 // wsum of the previous q consumed
            if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
            __syncthreads();
            uint32_t off = base + incl - n[q], total = 0;
            for (uint32_t w = 0; w < kThreads / 64; ++w) {
                if (w < (threadIdx.x >> 6)) off += wsum[w];
                total += wsum[w];
            }
            base += total;
            // bytes: groups 0..7 from the spread, continuation bit on every byte but the last
            const uint64_t lo = leb_spread8(z);
            const uint32_t g8 = (uint32_t)(z >> 56) & 0x7Fu, g9 = (uint32_t)(z >> 63);
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i)
                if (i < n[q]) b8[off + i] = (uint8_t)(i + 1 < n[q] ? (lo >> (8 * i)) | 0x80 : (lo >> (8 * i)) & 0x7F);
            if (n[q] > 8) b8[off + 8] = (uint8_t)(g8 | (n[q] > 9 ? 0x80u : 0u));
            if (n[q] > 9) b8[off + 9] = (uint8_t)g9;
        }
        __syncthreads();
        const uint32_t endb = base;                          // lead + chunk bytes
        const uint64_t g0 = go & ~3ull;
        uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + g0);
        uint8_t* d8 = dst + g0;
        const uint32_t nw = (endb + 3) / 4;
        for (uint32_t kk = threadIdx.x; kk < nw; kk += kThreads) {
            const uint32_t lo = kk * 4, hi = lo + 4;
            if (lo >= lead && hi <= endb && g0 + hi <= dst_cap) {
                d32[kk] = buf[kk];
            } else {
                for (uint32_t i = lo; i < hi; ++i)
                    if (i >= lead && i < endb && g0 + i < dst_cap) d8[i] = b8[i];
            }
        }
        go += endb - lead;
        __syncthreads();                                     // buf is reassembled for the next chunk
    }
}

}  // namespace

// ---------------- host-side planning ----------------
void varint_plan(const uint64_t* blob_off, uint64_t n_blobs, VarintPlan* plan) {
    plan->blob_region.assign(n_blobs + 1, 0);
    plan->blob_tile.assign(n_blobs + 1, 0);
    plan->max_regions = 0;
    uint64_t R = 0, T = 0;
    for (uint64_t b = 0; b < n_blobs; ++b) {
        plan->blob_region[b] = R;
        plan->blob_tile[b] = T;
        const uint64_t s = blob_off[b], e = blob_off[b + 1];
        const uint64_t nr = e > s ? (e - 1) / kRegionBytes - s / kRegionBytes + 1 : 0;
        R += nr;
        T += (nr + kTileRegions - 1) / kTileRegions;
        if (nr > plan->max_regions) plan->max_regions = nr;
    }
    plan->blob_region[n_blobs] = R;
    plan->blob_tile[n_blobs] = T;
    plan->regions = R;
    plan->tiles = T;
}

// Layout of the device workspace of the decode.
struct DecodeWork {
    unsigned long long* status; unsigned int* ticket; unsigned int* err;
    uint64_t* blob_off; uint64_t* blob_tile; uint32_t* irregular; uint64_t* blob_count;
};
static DecodeWork carve(void* work, size_t R, uint64_t n_blobs) {
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char* p = static_cast<char*>(work);
    DecodeWork w;
    w.status = (unsigned long long*)p; p += up(R * 8);
    w.ticket = (unsigned int*)p; w.err = w.ticket + 1; p += 256;
    w.blob_off = (uint64_t*)p; p += up((n_blobs + 1) * 8);
    w.blob_tile = (uint64_t*)p; p += up((n_blobs + 1) * 8);
    w.irregular = (uint32_t*)p; p += up(n_blobs * 4);
    w.blob_count = (uint64_t*)p;
    return w;
}
size_t varint_decode_work_bytes(size_t regions, uint64_t n_blobs) {
    return regions * 8 + (n_blobs + 1) * 16 + n_blobs * 12 + 8 * 256;
}

hipError_t launch_varint_decode(const uint8_t* bytes, const uint64_t* blob_off_host, uint64_t n_blobs,
                                const VarintPlan& plan, void* work, int64_t* out, uint64_t out_stride,
                                uint64_t* counts_host, hipStream_t s) {
    const size_t T = plan.tiles;
    DecodeWork w = carve(work, T, n_blobs);
    hipError_t e;
    if (n_blobs == 0) return hipSuccess;
    if ((e = hipMemcpyAsync(w.blob_off, blob_off_host, (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(w.blob_tile, plan.blob_tile.data(), (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.status, 0, ((T * 8 + 255) & ~(size_t)255) + 256, s)) != hipSuccess) return e;   // + ticket, err
    if ((e = hipMemsetAsync(w.irregular, 0, n_blobs * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.blob_count, 0, n_blobs * 8, s)) != hipSuccess) return e;      // empty blobs: 0
    if (T) {
        hipLaunchKernelGGL(varint_decode_kernel, dim3((unsigned)T), dim3(kThreads), 0, s, bytes, w.blob_tile,
                           w.blob_off, n_blobs, w.status, w.ticket, w.irregular, w.blob_count, w.err, out, out_stride);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    std::vector<uint32_t> irr(n_blobs);
    uint32_t errf = 0;
    if ((e = hipMemcpyAsync(irr.data(), w.irregular, n_blobs * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&errf, w.err, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if (errf) return hipErrorUnknown;              // a look-back spin ran out (never expected)
    bool irregular_any = false;
    for (uint64_t b = 0; b < n_blobs; ++b) irregular_any |= irr[b] != 0;
    if (irregular_any) {                           // malformed blobs: the reference loop, row and count
        hipLaunchKernelGGL(varint_sequential_kernel, dim3((unsigned)((n_blobs + 63) / 64)), dim3(64), 0, s, bytes,
                           w.blob_off, (uint32_t)n_blobs, w.irregular, w.blob_count, out, out_stride, out_stride);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((e = hipMemcpyAsync(counts_host, w.blob_count, n_blobs * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

size_t varint_encode_work_bytes(uint64_t rows, uint64_t len) {
    const uint64_t chunks = (len + kEncChunk - 1) / kEncChunk;
    const uint64_t tiles = (chunks + kEncTileChunks - 1) / kEncTileChunks;
    return rows * (tiles ? tiles : 1) * 8 + rows * 8 + 1024;
}

hipError_t launch_varint_encode(const int64_t* vals, uint64_t rows, uint64_t len, uint64_t stride, uint8_t* dst,
                                uint64_t dst_cap, void* work, uint64_t* row_bytes_host, hipStream_t s) {
    const uint64_t chunks = (len + kEncChunk - 1) / kEncChunk;
    const uint64_t tiles = (chunks + kEncTileChunks - 1) / kEncTileChunks;
    if (rows == 0) return hipSuccess;
    if (tiles == 0) {
        for (uint64_t r = 0; r < rows; ++r) row_bytes_host[r] = 0;
        return hipSuccess;
    }
    if (rows * tiles >= ((uint64_t)1 << 32)) return hipErrorInvalidValue;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char* p = static_cast<char*>(work);
    unsigned long long* status = reinterpret_cast<unsigned long long*>(p);
    unsigned int* ticket = reinterpret_cast<unsigned int*>(p + up(rows * tiles * 8));
    unsigned int* err = ticket + 1;
    uint64_t* row_end = reinterpret_cast<uint64_t*>(p + up(rows * tiles * 8) + 256);
    hipError_t e;
    if ((e = hipMemsetAsync(status, 0, up(rows * tiles * 8) + 256, s)) != hipSuccess) return e;   // + ticket, err
    hipLaunchKernelGGL(varint_encode_kernel, dim3((unsigned)(rows * tiles)), dim3(kThreads), 0, s, vals, len, stride,
                       tiles, status, ticket, row_end, err, dst, dst_cap);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    std::vector<uint64_t> ends(rows);
    uint32_t errf = 0;
    if ((e = hipMemcpyAsync(ends.data(), row_end, rows * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&errf, err, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if (errf) return hipErrorUnknown;
    for (uint64_t r = 0; r < rows; ++r) row_bytes_host[r] = ends[r] - (r ? ends[r - 1] : 0);
    if (ends[rows - 1] > dst_cap) return hipErrorInvalidValue;    // nothing past dst_cap was written
    return hipSuccess;
}

}  // namespace sda
