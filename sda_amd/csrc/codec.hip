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
// stream compaction over terminator bytes (b & 0x80 == 0):
//   pass A  per 16 KiB aligned region of a blob: count terminators, flag runs of >= 11
//           continuation bytes ("irregular" blob);
//   pass B  per blob: exclusive scan of its region counts -> element base per region, total;
//   pass C  per region: each terminator byte decodes the <= 10-byte varint that ends at it (its
//           start is the previous terminator, within the 16-byte halo) into out[blob][index].
// Irregular blobs (malformed streams) are decoded by a sequential exact kernel instead.
// Roofline: HBM.  Algorithmic bytes = payload bytes read + 8 B per decoded element written.
#include "kernels.h"

namespace sda {

namespace {

constexpr int kThreads = 256;
constexpr int kWPT = 4;                       // 16-byte words per thread: word t + 256 k, k < kWPT
constexpr uint64_t kSubBytes = kThreads * 16; // one sub-region = one word per thread
constexpr uint64_t kRegionBytes = kSubBytes * kWPT;



// Inclusive prefix sum over the 64 lanes of a wave with DPP (row shifts, then the row broadcasts of
// gfx9): six VALU adds, no LDS round trips.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return x;
}

// Bits 7, 15, 23, 31 of d -> bits 0..3: the product of the masked word with 2^0 + 2^7 + 2^14 + 2^21
// moves bit 8k+7 to 28+k; every other partial product lands on a distinct lower bit (no carries).
__device__ __forceinline__ uint32_t msb_nibble(uint32_t d) {
    return ((d & 0x80808080u) * 0x00204081u) >> 28;
}

// 16 bytes as a 16-bit mask of "continuation" bytes (bit j = byte j has 0x80).
__device__ __forceinline__ uint32_t cont_mask(uint4 w) {
    return msb_nibble(w.x) | (msb_nibble(w.y) << 4) | (msb_nibble(w.z) << 8) | (msb_nibble(w.w) << 12);
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
    uint32_t valid, term, cont;
};

__device__ __forceinline__ Window make_window_cm(uint32_t cm, uint64_t word, uint64_t begin, uint64_t end) {
    Window W;
    const uint64_t a0 = word * 16;                      // byte offset of own word (aligned)
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
__device__ __forceinline__ Window make_window(uint4 prev, uint4 own, uint64_t word, uint64_t begin, uint64_t end) {
    return make_window_cm(cont_mask(prev) | (cont_mask(own) << 16), word, begin, end);
}
// A window whose 32 bytes all lie inside the blob, with the blob's last byte beyond it.
__device__ __forceinline__ Window interior_window(uint32_t cm) {
    Window W;
    W.valid = 0xFFFF0000u;
    W.cont = cm;
    W.term = ~cm;
    return W;
}

// 2-D grid: blockIdx.y = blob (+ y0), blockIdx.x = region within the blob (16 KiB aligned to the
// byte buffer).  Blocks past a blob's last region exit at once (payload blobs have near-equal sizes).
__device__ __forceinline__ bool region_of(const uint64_t* __restrict__ blob_region,
                                          const uint64_t* __restrict__ blob_off, uint32_t y0, uint32_t* blob,
                                          uint64_t* region, uint64_t* word) {
    const uint32_t b = y0 + blockIdx.y;
    const uint64_t r0 = blob_region[b], r1 = blob_region[b + 1];
    if (r0 + blockIdx.x >= r1) return false;
    *blob = b;
    *region = r0 + blockIdx.x;
    *word = (blob_off[b] / kRegionBytes + blockIdx.x) * (kRegionBytes / 16);
    return true;
}

// pass A: terminator count of each region; irregular-blob flag.
__global__ __launch_bounds__(kThreads) void varint_count_kernel(const uint8_t* __restrict__ bytes,
                                                                const uint64_t* __restrict__ blob_region,
                                                                const uint64_t* __restrict__ blob_off, uint32_t y0,
                                                                uint32_t* __restrict__ region_count,
                                                                uint32_t* __restrict__ blob_irregular) {
    uint32_t b;
    uint64_t r, word;
    if (!region_of(blob_region, blob_off, y0, &b, &r, &word)) return;
    const uint64_t begin = blob_off[b], end = blob_off[b + 1];
    // one coalesced load per word; the previous word's continuation mask (for the run check across
    // the word boundary) comes through LDS
    __shared__ uint32_t cm_l[kWPT * kThreads + 1];
    const uint4* p = reinterpret_cast<const uint4*>(bytes);
    uint4 v[kWPT];
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        const uint64_t wk = word + threadIdx.x + k * kThreads;
        v[k] = wk * 16 < end ? p[wk] : make_uint4(0, 0, 0, 0);
    }
    uint4 halo = make_uint4(0, 0, 0, 0);
    if (threadIdx.x == 0 && word * 16 > begin) halo = p[word - 1];
    Window W[kWPT];
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        const uint32_t wl = threadIdx.x + k * kThreads;
        W[k] = make_window(make_uint4(0, 0, 0, 0), v[k], word + wl, begin, end);   // own-word masks only
        cm_l[wl + 1] = W[k].cont >> 16;
    }
    if (threadIdx.x == 0) cm_l[0] = make_window(make_uint4(0, 0, 0, 0), halo, word - 1, begin, end).cont >> 16;
    __syncthreads();
    uint32_t n = 0, bad = 0;
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        const uint32_t wl = threadIdx.x + k * kThreads;
        n += __builtin_popcount(W[k].term & W[k].valid);
        // 11 continuation bytes in a row ending inside this word?
        const uint32_t cont = W[k].cont | cm_l[wl];
        uint32_t run = cont;
#pragma unroll
        for (int q = 1; q <= 10; ++q) run &= cont << q;
        bad |= run & W[k].valid;
    }
    if (bad) atomicOr(&blob_irregular[b], 1u);
    // block reduction (one value per region)
    __shared__ uint32_t red[kThreads / 64];
    for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int i = 0; i < kThreads / 64; ++i) s += red[i];
        region_count[r] = s;
    }
}

// pass B: per blob, exclusive scan of its region counts (regions of blob b are
// [blob_region[b], blob_region[b+1])) -> region_base; total -> blob_count.
__global__ __launch_bounds__(kThreads) void varint_scan_kernel(const uint32_t* __restrict__ region_count,
                                                               const uint64_t* __restrict__ blob_region,
                                                               uint64_t* __restrict__ region_base,
                                                               uint64_t* __restrict__ blob_count) {
    const uint32_t b = blockIdx.x;
    const uint64_t r0 = blob_region[b], r1 = blob_region[b + 1];
    __shared__ uint64_t part[kThreads];
    uint64_t carry = 0;
    for (uint64_t base = r0; base < r1; base += kThreads) {
        const uint64_t r = base + threadIdx.x;
        const uint64_t v = r < r1 ? region_count[r] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < kThreads; o <<= 1) {            // Hillis-Steele inclusive scan
            const uint64_t add = threadIdx.x >= (uint32_t)o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += add;
            __syncthreads();
        }
        if (r < r1) region_base[r] = carry + part[threadIdx.x] - v;
        carry += part[kThreads - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) blob_count[b] = carry;
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

// pass C: decode.  The region's bytes (plus a 16-byte halo on each side) are staged in LDS, with
// each word's 16-bit continuation mask beside them (so a window's previous-word mask is one LDS
// read).  The region is walked as kWPT sub-regions of one word per thread.  Per sub-region a
// block-wide scan of the terminator counts compacts the elements' (start, length) into LDS; then
// lane i decodes element i (balanced work, coalesced stores) from funnel-shifted dwords -- elements
// of <= 5 bytes (every field share below 2^31) on a short 32-bit path, longer ones on the general
// one.  Element index of a terminator = region base + terminators before it in the region.  Blobs
// flagged irregular are skipped here (varint_sequential_kernel).
//
// OutT = int32_t (the clerk's decode -> combine of field shares, |v| < 2^31): the values are stored
// narrowed and any value that does not fit sets *wide (the caller then decodes again as i64).
template <typename OutT>
__global__ __launch_bounds__(kThreads) void varint_decode_kernel(const uint8_t* __restrict__ bytes,
                                                                 const uint64_t* __restrict__ blob_region,
                                                                 const uint64_t* __restrict__ blob_off, uint32_t y0,
                                                                 const uint64_t* __restrict__ region_base,
                                                                 const uint32_t* __restrict__ blob_irregular,
                                                                 OutT* __restrict__ out, uint64_t out_stride,
                                                                 uint32_t* __restrict__ wide) {
    uint32_t b;
    uint64_t r, word;
    if (!region_of(blob_region, blob_off, y0, &b, &r, &word) || blob_irregular[b]) return;
    __shared__ uint32_t lb[(kRegionBytes + 32) / 4];          // [halo 16 B | region 16 KiB | tail 16 B]
    __shared__ uint32_t cml[kWPT * kThreads + 1];             // continuation mask of lb word w at [w]
    __shared__ uint32_t wsum[kThreads / 64];
    __shared__ uint32_t el[kSubBytes];                        // one sub-region's elements: start | len << 16
    const uint64_t begin = blob_off[b], end = blob_off[b + 1];
    // every window of the region inside the blob, and the blob's last byte past the region
    const bool interior = word * 16 >= begin + 16 && end > word * 16 + kRegionBytes;
    {
        const uint4* p = reinterpret_cast<const uint4*>(bytes);
        uint4 v[kWPT];
#pragma unroll
        for (int k = 0; k < kWPT; ++k) {
            const uint64_t wk = word + threadIdx.x + k * kThreads;
            v[k] = wk * 16 < end ? p[wk] : make_uint4(0, 0, 0, 0);
        }
        if (threadIdx.x == 0) {
            const uint4 h = (word * 16 > begin) ? p[word - 1] : make_uint4(0, 0, 0, 0);
            reinterpret_cast<uint4*>(lb)[0] = h;
            cml[0] = cont_mask(h);
        }
        if (threadIdx.x == kThreads - 1) reinterpret_cast<uint4*>(lb)[kWPT * kThreads + 1] = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < kWPT; ++k) {
            reinterpret_cast<uint4*>(lb)[threadIdx.x + k * kThreads + 1] = v[k];
            cml[threadIdx.x + k * kThreads + 1] = cont_mask(v[k]);
        }
    }
    __syncthreads();
    Window W[kWPT];
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        const uint32_t wl = threadIdx.x + k * kThreads;
        const uint32_t cm = cml[wl] | (cml[wl + 1] << 16);
        W[k] = interior ? interior_window(cm) : make_window_cm(cm, word + wl, begin, end);
    }
    OutT* dst = out + (uint64_t)b * out_stride + region_base[r];
    bool narrow_fail = false;
    uint32_t base = 0;                                        // elements in earlier sub-regions
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        // 1. compaction: each thread lists the (start, length) of the elements ending in its word
        const uint32_t tm = W[k].term & W[k].valid;
        const uint32_t n = __builtin_popcount(tm);
        const uint32_t incl = wave_incl_scan(n);              // exclusive scan of n over the block
        __syncthreads();                                      // lb visible; el / wsum free for reuse
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
        __syncthreads();
        uint32_t e = incl - n, total = 0;
        for (uint32_t w = 0; w < kThreads / 64; ++w) {
            if (w < (threadIdx.x >> 6)) e += wsum[w];
            total += wsum[w];
        }
        if (tm) {
            // the first element starts after the previous boundary (a terminator, or a byte outside
            // the blob); each later one right after the terminator before it
            const uint32_t boundary = W[k].term | ~(W[k].term | W[k].cont);
            const uint32_t pos0 = (threadIdx.x + k * kThreads) * 16;
            uint32_t rem = tm;
            const uint32_t below = boundary & ((1u << __builtin_ctz(rem)) - 1u);
            uint32_t st = below ? 32 - __builtin_clz(below) : 0;      // window index of the first byte
            do {
                const uint32_t j = __builtin_ctz(rem);
                rem &= rem - 1;
                el[e++] = (pos0 + st) | ((j - st + 1) << 16);
                st = j + 1;
            } while (rem);
        }
        __syncthreads();
        // 2. decode: lane i takes element i -> balanced work, coalesced stores
        for (uint32_t i = threadIdx.x; i < total; i += kThreads) {
            const uint32_t P = el[i] & 0xFFFFu;                  // byte position in lb
            const uint32_t len = el[i] >> 16;                     // 1..11 on regular blobs
            const uint32_t q = P >> 2, sh = (P & 3) * 8;
            const uint32_t d0 = lb[q], d1 = lb[q + 1], d2 = lb[q + 2];
            const uint32_t b0 = __builtin_amdgcn_alignbit(d1, d0, sh), b1 = __builtin_amdgcn_alignbit(d2, d1, sh);
            if constexpr (sizeof(OutT) < 8) {
                // int32 output: elements of <= 5 bytes whose zigzag value is below 2^32 (anything
                // else sets *wide and the caller decodes the job as i64)
                const uint32_t l4 = len < 4 ? len : 4u, cut = 32 - 8 * l4;
                uint32_t x = ((b0 << cut) >> cut) & 0x7F7F7F7Fu;
                x = (x & 0x007F007Fu) | ((x >> 1) & ~0x007F007Fu);
                x = (x & 0x00003FFFu) | ((x >> 2) & ~0x00003FFFu);
                const uint32_t g4 = len == 5 ? (b1 & 0x7Fu) : 0u;
                narrow_fail |= len > 5 || g4 > 15;
                const uint32_t zl = x | (g4 << 28);
                dst[base + i] = (OutT)((zl >> 1) ^ (0u - (zl & 1u)));
                continue;
            }
            int64_t val;
            if (len <= 5) {
                // bytes 0..3 (masked to the element) -> 4 x 7-bit groups: two bit-field merges
                const uint32_t l4 = len < 4 ? len : 4u, cut = 32 - 8 * l4;
                uint32_t x = ((b0 << cut) >> cut) & 0x7F7F7F7Fu;
                x = (x & 0x007F007Fu) | ((x >> 1) & ~0x007F007Fu);  // byte pairs -> 14-bit lanes (bit 15 junk)
                x = (x & 0x00003FFFu) | ((x >> 2) & ~0x00003FFFu);  // -> 28 bits (bits 28..31 clear)
                const uint32_t g4 = len == 5 ? (b1 & 0x7Fu) : 0u;   // group 4 at bit 28
                const uint32_t zl = x | (g4 << 28), zh = g4 >> 4;
                val = (int64_t)((((uint64_t)zh << 32) | zl) >> 1) ^ -(int64_t)(zl & 1u);
            } else {
                const uint32_t b2 = __builtin_amdgcn_alignbit(lb[q + 3], d2, sh);
                uint64_t lo = ((uint64_t)b1 << 32) | b0;
                if (len < 8) lo &= (1ull << (8 * len)) - 1;
                uint64_t z = leb_pack8(lo);
                if (len > 8) {          // groups 8, 9, 10 at shifts 56, 63, 70 & 63 = 6 (Rust release)
                    const uint32_t hb = b2 & ((len >= 11) ? 0xFFFFFFu : (len == 10 ? 0xFFFFu : 0xFFu));
                    z |= ((uint64_t)(hb & 0x7F) << 56) | ((uint64_t)((hb >> 8) & 0x7F) << 63) |
                         ((uint64_t)((hb >> 16) & 0x7F) << 6);
                }
                val = (int64_t)((z >> 1) ^ (0 - (z & 1)));
            }
            dst[base + i] = (OutT)val;
        }
        base += total;
    }
    if constexpr (sizeof(OutT) < 8) {
        if (narrow_fail) atomicOr(wide, 1u);             // rare: one atomic per lane that saw it
    }
}

// Irregular blobs: the reference loop, one lane per blob (only malformed streams get here).
// With out == nullptr it only counts.
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
        if (out && c < cap) out[(uint64_t)b * out_stride + c] = (int64_t)((z >> 1) ^ (0 - (z & 1)));
        ++c;
    }
    if (!out) blob_count[b] = c;
}

// ---------------- encode ----------------
__device__ __forceinline__ uint32_t varint_size(int64_t v) {
    const uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
    const int bits = 64 - __builtin_clzll(z | 1);
    return (uint32_t)((bits + 6) / 7);
}

constexpr uint32_t kEncChunk = 2048;          // elements per encode block
constexpr uint32_t kEncPer = kEncChunk / kThreads;
constexpr uint32_t kEncPairs = kEncPer / 2;   // size pass: rounds of one adjacent element pair per lane
#ifndef SDA_ENC_EPL
#define SDA_ENC_EPL 2
#endif
constexpr uint32_t kEncEpl = SDA_ENC_EPL;     // write pass: adjacent elements per lane per round (even)
constexpr uint32_t kEncRounds = kEncChunk / (kEncEpl * kThreads);
typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
// A full chunk whose first element is 16-byte aligned is read as element pairs (one 16-byte load per
// lane: a wave moves 1 KiB per load instruction instead of 512 B).
__device__ __forceinline__ bool enc_pairs_ok(const int64_t* rowp, uint64_t e0, uint64_t len) {
    return e0 + kEncChunk <= len && ((uintptr_t)(rowp + e0) & 15) == 0;
}

// sizes of each [row][chunk] block of elements
__global__ __launch_bounds__(kThreads) void varint_size_kernel(const int64_t* __restrict__ vals, uint64_t len,
                                                               uint64_t stride, uint32_t chunks,
                                                               uint64_t* __restrict__ chunk_bytes) {
    const uint32_t c = blockIdx.x, row = blockIdx.y;
    const uint64_t e0 = (uint64_t)c * kEncChunk;
    const int64_t* rowp = vals + (uint64_t)row * stride;
    uint64_t n = 0;
    if (enc_pairs_ok(rowp, e0, len)) {          // 16-byte loads: element pairs (order is irrelevant here)
#pragma unroll
        for (uint32_t q = 0; q < kEncPairs; ++q) {
            const i64x2 x = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(rowp + e0) + q * kThreads + threadIdx.x);
            n += varint_size(x[0]) + varint_size(x[1]);
        }
    } else {
#pragma unroll
        for (uint32_t q = 0; q < kEncPer; ++q) {
            const uint64_t e = e0 + q * kThreads + threadIdx.x;
            if (e < len) n += varint_size(rowp[e]);
        }
    }
    __shared__ uint64_t red[kThreads / 64];
    for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (int i = 0; i < kThreads / 64; ++i) s += red[i];
        chunk_bytes[(uint64_t)row * chunks + c] = s;
    }
}

// inverse of leb_pack8: 7-bit groups of z -> bytes (group i in byte i), continuation bits not set
__device__ __forceinline__ uint64_t leb_spread8(uint64_t z) {
    uint64_t x = z & 0x00FFFFFFFFFFFFFFull;
    x = (x & 0x000000000FFFFFFFull) | ((x & 0x00FFFFFFF0000000ull) << 4);
    x = (x & 0x00003FFF00003FFFull) | ((x & 0x0FFFC0000FFFC000ull) << 2);
    x = (x & 0x007F007F007F007Full) | ((x & 0x3F803F803F803F80ull) << 1);
    return x;
}

// write: coalesced 16-byte loads (lane t: kEncEpl adjacent elements per round q), one block-wide
// scan of the lane sizes per q, each element's bytes ORed into a zeroed LDS image of the chunk's output (its 8 + 2 bytes shifted
// to their byte offset: 2-4 ds_or_b32, no per-byte stores), the image aligned to the chunk's global
// byte offset mod 16 so that the interior leaves as 16-byte stores; the two partial 16-byte words at
// the ends (shared with the neighbouring chunks) are written byte-wise.
// chunk_off = row offset + exclusive scan of chunk_bytes.
__global__ __launch_bounds__(kThreads) void varint_write_kernel(const int64_t* __restrict__ vals, uint64_t len,
                                                                uint64_t stride, uint32_t chunks,
                                                                const uint64_t* __restrict__ chunk_off,
                                                                uint8_t* __restrict__ dst) {
    const uint32_t c = blockIdx.x, row = blockIdx.y;
    const uint64_t e0 = (uint64_t)c * kEncChunk;
    constexpr uint32_t kBufQuads = (kEncChunk * 10 + 32) / 16;      // lead < 16, + the shifted tail dwords
    __shared__ uint4 buf4[kBufQuads];
    __shared__ uint32_t wsum[kThreads / 64];
    uint32_t* buf = reinterpret_cast<uint32_t*>(buf4);
    const uint8_t* b8 = reinterpret_cast<const uint8_t*>(buf4);
    uint8_t* gdst = dst + chunk_off[(uint64_t)row * chunks + c];
    const uint32_t lead = (uint32_t)((uintptr_t)gdst & 15);
    for (uint32_t k = threadIdx.x; k < kBufQuads; k += kThreads) buf4[k] = make_uint4(0, 0, 0, 0);
    // round q: lane t owns the kEncEpl adjacent elements e0 + R q + kEncEpl t + j (R = kEncEpl * 256;
    // 16-byte loads when the chunk allows it), so one block-wide scan of the lane sizes places R elements
    const int64_t* rowp = vals + (uint64_t)row * stride;
    int64_t v[kEncRounds][kEncEpl];
    if (enc_pairs_ok(rowp, e0, len)) {
#pragma unroll
        for (uint32_t q = 0; q < kEncRounds; ++q)
#pragma unroll
            for (uint32_t j = 0; j < kEncEpl / 2; ++j) {
                const i64x2 x = __builtin_nontemporal_load(
                    reinterpret_cast<const i64x2*>(rowp + e0 + kEncEpl * (q * kThreads + threadIdx.x)) + j);
                v[q][2 * j] = x[0];
                v[q][2 * j + 1] = x[1];
            }
    } else {
#pragma unroll
        for (uint32_t q = 0; q < kEncRounds; ++q)
#pragma unroll
            for (uint32_t j = 0; j < kEncEpl; ++j) {
                const uint64_t e = e0 + kEncEpl * (q * kThreads + threadIdx.x) + j;
                v[q][j] = e < len ? rowp[e] : 0;
            }
    }
    uint32_t base = lead;
#pragma unroll
    for (uint32_t q = 0; q < kEncRounds; ++q) {
        const uint64_t e = e0 + kEncEpl * (q * kThreads + threadIdx.x);
        uint32_t ns[kEncEpl], pre[kEncEpl], np = 0;
#pragma unroll
        for (uint32_t j = 0; j < kEncEpl; ++j) {
            ns[j] = e + j < len ? varint_size(v[q][j]) : 0u;
            pre[j] = np;
            np += ns[j];
        }
        const uint32_t incl = wave_incl_scan(np);
        __syncthreads();                                     // wsum of the previous q consumed (and, at
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;    // q = 0, the zeroed image visible)
        __syncthreads();
        uint32_t off0 = base + incl - np, total = 0;
        for (uint32_t w = 0; w < kThreads / 64; ++w) {
            if (w < (threadIdx.x >> 6)) off0 += wsum[w];
            total += wsum[w];
        }
        base += total;
#pragma unroll
        for (uint32_t h = 0; h < kEncEpl; ++h) {
            const uint32_t n = ns[h], off = off0 + pre[h];
            const uint64_t z = ((uint64_t)v[q][h] << 1) ^ (uint64_t)(v[q][h] >> 63);
            if (n) {
                // bytes 0..7: groups 0..7, continuation bit on every byte but the element's last;
                // bytes 8, 9 (n > 8): groups 8 and 9
                const uint32_t nc = n - 1;
                const uint64_t cont = nc >= 8 ? 0x8080808080808080ull : (0x8080808080808080ull & ((1ull << (8 * nc)) - 1));
                const uint64_t W = leb_spread8(z) | cont;
                const uint32_t g8 = (uint32_t)(z >> 56) & 0x7Fu, g9 = (uint32_t)(z >> 63);
                const uint32_t E = n > 8 ? (g8 | (n > 9 ? 0x80u : 0u) | (g9 << 8)) : 0u;
                const uint32_t sh = (off & 3) * 8, dw = off >> 2;
                const uint32_t o0 = (uint32_t)W << sh;
                const uint32_t o1 = (uint32_t)(W >> (32 - sh));                          // sh = 0: W's high word
                const uint32_t o2 = (uint32_t)(((((uint64_t)E) << 32) | (uint32_t)(W >> 32)) >> (32 - sh));
                const uint32_t o3 = sh ? E >> (32 - sh) : 0u;
                atomicOr(&buf[dw], o0);                                                  // ds_or_b32
                if (o1) atomicOr(&buf[dw + 1], o1);
                if (o2) atomicOr(&buf[dw + 2], o2);
                if (o3) atomicOr(&buf[dw + 3], o3);
            }
        }
    }
    __syncthreads();
    const uint32_t end = base;                               // lead + chunk bytes
    uint4* d128 = reinterpret_cast<uint4*>(gdst - lead);
    uint8_t* d8 = gdst - lead;
    const uint32_t nq = (end + 15) / 16;
    for (uint32_t k = threadIdx.x; k < nq; k += kThreads) {
        const uint32_t lo = k * 16, hi = lo + 16;
        if (lo >= lead && hi <= end) {
            d128[k] = buf4[k];
        } else {
            for (uint32_t i = lo; i < hi; ++i)
                if (i >= lead && i < end) d8[i] = b8[i];
        }
    }
}

// exclusive scan of chunk_bytes per row (one block per row) + row base; row_bytes = total
__global__ __launch_bounds__(kThreads) void varint_offsets_kernel(const uint64_t* __restrict__ chunk_bytes,
                                                                  uint32_t chunks, const uint64_t* __restrict__ row_base,
                                                                  uint64_t* __restrict__ chunk_off,
                                                                  uint64_t* __restrict__ row_bytes) {
    const uint32_t row = blockIdx.x;
    __shared__ uint64_t part[kThreads];
    uint64_t carry = row_base ? row_base[row] : 0, total = 0;
    for (uint32_t base = 0; base < chunks; base += kThreads) {
        const uint32_t c = base + threadIdx.x;
        const uint64_t v = c < chunks ? chunk_bytes[(uint64_t)row * chunks + c] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < kThreads; o <<= 1) {
            const uint64_t add = threadIdx.x >= (uint32_t)o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += add;
            __syncthreads();
        }
        if (c < chunks) chunk_off[(uint64_t)row * chunks + c] = carry + part[threadIdx.x] - v;
        carry += part[kThreads - 1];
        total += part[kThreads - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0 && row_bytes) row_bytes[row] = total;
}

}  // namespace

// ---------------- host-side planning ----------------
void varint_plan(const uint64_t* blob_off, uint64_t n_blobs, VarintPlan* plan) {
    plan->blob_region.assign(n_blobs + 1, 0);
    plan->max_regions = 0;
    uint64_t R = 0;
    for (uint64_t b = 0; b < n_blobs; ++b) {
        plan->blob_region[b] = R;
        const uint64_t s = blob_off[b], e = blob_off[b + 1];
        const uint64_t nr = e > s ? (e - 1) / kRegionBytes - s / kRegionBytes + 1 : 0;
        R += nr;
        if (nr > plan->max_regions) plan->max_regions = nr;
    }
    plan->blob_region[n_blobs] = R;
    plan->regions = R;
}

// Layout of the device workspace for the decode passes.
struct DecodeWork {
    uint32_t* region_count; uint64_t* region_base;
    uint64_t* blob_off; uint64_t* blob_region; uint32_t* irregular; uint64_t* blob_count; uint32_t* wide;
};
static DecodeWork carve(void* work, size_t R, uint64_t n_blobs) {
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char* p = static_cast<char*>(work);
    DecodeWork w;
    w.region_base = (uint64_t*)p; p += up(R * 8);
    w.region_count = (uint32_t*)p; p += up(R * 4);
    w.blob_off = (uint64_t*)p; p += up((n_blobs + 1) * 8);
    w.blob_region = (uint64_t*)p; p += up((n_blobs + 1) * 8);
    w.irregular = (uint32_t*)p; p += up(n_blobs * 4);
    w.blob_count = (uint64_t*)p; p += up(n_blobs * 8);
    w.wide = (uint32_t*)p;
    return w;
}
size_t varint_decode_work_bytes(size_t regions, uint64_t n_blobs) {
    return regions * 12 + (n_blobs + 1) * 16 + n_blobs * 12 + 8 * 256;    // (7 x 256 B of rounding + flag)
}

hipError_t launch_varint_count(const uint8_t* bytes, const uint64_t* blob_off_host, uint64_t n_blobs,
                               const VarintPlan& plan, void* work, uint64_t* counts_host, bool* irregular_any,
                               hipStream_t s) {
    const size_t R = plan.regions;
    DecodeWork w = carve(work, R, n_blobs);
    hipError_t e;
    if ((e = hipMemcpyAsync(w.blob_off, blob_off_host, (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(w.blob_region, plan.blob_region.data(), (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.irregular, 0, n_blobs * 4, s)) != hipSuccess) return e;
    for (uint64_t y0 = 0; R && y0 < n_blobs; y0 += 65535) {
        const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
        hipLaunchKernelGGL(varint_count_kernel, dim3((unsigned)plan.max_regions, ny), dim3(kThreads), 0, s, bytes,
                           w.blob_region, w.blob_off, (uint32_t)y0, w.region_count, w.irregular);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(varint_scan_kernel, dim3((unsigned)n_blobs), dim3(kThreads), 0, s, w.region_count,
                       w.blob_region, w.region_base, w.blob_count);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(varint_sequential_kernel, dim3((unsigned)((n_blobs + 63) / 64)), dim3(64), 0, s, bytes,
                       w.blob_off, (uint32_t)n_blobs, w.irregular, w.blob_count, (int64_t*)nullptr, 0, 0);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    std::vector<uint32_t> irr(n_blobs);
    if ((e = hipMemcpyAsync(counts_host, w.blob_count, n_blobs * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(irr.data(), w.irregular, n_blobs * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *irregular_any = false;
    for (uint64_t b = 0; b < n_blobs; ++b) *irregular_any |= irr[b] != 0;
    return hipSuccess;
}

hipError_t launch_varint_decode(const uint8_t* bytes, uint64_t n_blobs, const VarintPlan& plan, void* work,
                                int64_t* out, uint64_t out_stride, uint64_t len, bool irregular_any,
                                hipStream_t s) {
    const size_t R = plan.regions;
    DecodeWork w = carve(work, R, n_blobs);
    hipError_t e;
    for (uint64_t y0 = 0; R && y0 < n_blobs; y0 += 65535) {
        const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
        hipLaunchKernelGGL(varint_decode_kernel<int64_t>, dim3((unsigned)plan.max_regions, ny), dim3(kThreads), 0, s,
                           bytes, w.blob_region, w.blob_off, (uint32_t)y0, w.region_base, w.irregular, out, out_stride,
                           w.wide);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (irregular_any) {
        hipLaunchKernelGGL(varint_sequential_kernel, dim3((unsigned)((n_blobs + 63) / 64)), dim3(64), 0, s, bytes,
                           w.blob_off, (uint32_t)n_blobs, w.irregular, w.blob_count, out, out_stride, len);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_varint_decode_narrow(const uint8_t* bytes, uint64_t n_blobs, const VarintPlan& plan, void* work,
                                       int32_t* out, uint64_t out_stride, bool* wide_host, hipStream_t s) {
    const size_t R = plan.regions;
    DecodeWork w = carve(work, R, n_blobs);
    hipError_t e;
    if ((e = hipMemsetAsync(w.wide, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    for (uint64_t y0 = 0; R && y0 < n_blobs; y0 += 65535) {
        const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
        hipLaunchKernelGGL(varint_decode_kernel<int32_t>, dim3((unsigned)plan.max_regions, ny), dim3(kThreads), 0, s,
                           bytes, w.blob_region, w.blob_off, (uint32_t)y0, w.region_base, w.irregular, out, out_stride,
                           w.wide);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    uint32_t flag = 0;
    if ((e = hipMemcpyAsync(&flag, w.wide, sizeof(flag), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *wide_host = flag != 0;
    return hipSuccess;
}

size_t varint_encode_work_bytes(uint64_t rows, uint64_t len) {
    const uint64_t chunks = (len + kEncChunk - 1) / kEncChunk;
    return 2 * rows * (chunks ? chunks : 1) * 8 + 2 * rows * 8 + 1024;
}

hipError_t launch_varint_encode(const int64_t* vals, uint64_t rows, uint64_t len, uint64_t stride, uint8_t* dst,
                                uint64_t dst_cap, void* work, uint64_t* row_bytes_host, hipStream_t s) {
    const uint64_t chunks = (len + kEncChunk - 1) / kEncChunk;
    if (rows == 0) return hipSuccess;
    uint64_t* chunk_bytes = static_cast<uint64_t*>(work);
    uint64_t* chunk_off = chunk_bytes + rows * (chunks ? chunks : 1);
    uint64_t* row_base = chunk_off + rows * (chunks ? chunks : 1);
    uint64_t* rbytes = row_base + rows;
    hipError_t e;
    if (chunks == 0) {
        for (uint64_t r = 0; r < rows; ++r) row_bytes_host[r] = 0;
        return hipSuccess;
    }
    hipLaunchKernelGGL(varint_size_kernel, dim3((unsigned)chunks, (unsigned)rows), dim3(kThreads), 0, s, vals, len,
                       stride, (uint32_t)chunks, chunk_bytes);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // per-row totals first (row_base = nullptr), then the host places rows back to back
    hipLaunchKernelGGL(varint_offsets_kernel, dim3((unsigned)rows), dim3(kThreads), 0, s, chunk_bytes,
                       (uint32_t)chunks, (const uint64_t*)nullptr, chunk_off, rbytes);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(row_bytes_host, rbytes, rows * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    std::vector<uint64_t> base(rows);
    uint64_t acc = 0;
    for (uint64_t r = 0; r < rows; ++r) { base[r] = acc; acc += row_bytes_host[r]; }
    if (acc > dst_cap) return hipErrorInvalidValue;
    if ((e = hipMemcpyAsync(row_base, base.data(), rows * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(varint_offsets_kernel, dim3((unsigned)rows), dim3(kThreads), 0, s, chunk_bytes,
                       (uint32_t)chunks, (const uint64_t*)row_base, chunk_off, (uint64_t*)nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(varint_write_kernel, dim3((unsigned)chunks, (unsigned)rows), dim3(kThreads), 0, s, vals, len,
                       stride, (uint32_t)chunks, chunk_off, dst);
    return hipGetLastError();
}

}  // namespace sda
