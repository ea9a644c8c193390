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
//
// The clerk's decode -> combine (clerk.rs:79-86) decodes into an int32 matrix and runs the exact combine.
// An opt-in variant (SDA_CODEC_PATH=fused; measured slower -- VALU-bound, profiles/r02d/ab_codec_fused.txt)
// fuses pass C with the combine instead of writing the [N][len] matrix: pass A also counts the
// terminators of every 256-byte sub-chunk; a plan kernel locates, per (column tile of kDcTile
// elements, blob), the sub-chunk holding the terminator that ends
// the previous tile and how many of its terminators precede the tile; then one workgroup per column
// tile walks the blobs in order, decodes its tile's slice of each payload (read once, plus at most a
// sub-chunk per tile edge) and folds it into combiner.rs:16-28's exact recurrence in registers.
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"

namespace sda {

namespace {

constexpr int kThreads = 256;
constexpr int kWPT = 4;                       // 16-byte words per thread: word t + 256 k, k < kWPT
constexpr uint64_t kSubBytes = kThreads * 16; // one sub-region = one word per thread
constexpr uint64_t kRegionBytes = kSubBytes * kWPT;
// Slots per region of the clerk's slot decode: a region of 16 KiB holds at most 4096 elements of >= 4
// bytes (a field share below 2^31 takes 4-5).  A region with more (short elements) raises *wide, and the
// job takes the matrix path; the slot buffer has kRegionBytes - kSlotCap slots of slack at its end, so the
// last region's overflowing stores stay inside it.
constexpr uint64_t kSlotCap = 4096;



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

// Sum over each row of 16 lanes, in the row's last lane (the first four steps of wave_incl_scan).
__device__ __forceinline__ uint32_t row16_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
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
    // (natural order: the XCD-chunked order of xcd.h made the clerk's decode -> combine 3 % slower,
    // profiles/r04f)
    const uint32_t b = y0 + blockIdx.y;
    const uint64_t r0 = blob_region[b], r1 = blob_region[b + 1];
    if (r0 + blockIdx.x >= r1) return false;
    *blob = b;
    *region = r0 + blockIdx.x;
    *word = (blob_off[b] / kRegionBytes + blockIdx.x) * (kRegionBytes / 16);
    return true;
}

// pass A: terminator count of each region; irregular-blob flag.  With sub_count (the clerk's fused
// decode -> combine) also the count of every 256-byte sub-chunk (16 words = one row of 16 lanes):
// sub_count[region * 64 + sub-chunk].
constexpr uint32_t kSubChunk = 256;
constexpr uint32_t kSubPerRegion = (uint32_t)(kRegionBytes / kSubChunk);
__global__ __launch_bounds__(kThreads) void varint_count_kernel(const uint8_t* __restrict__ bytes,
                                                                const uint64_t* __restrict__ blob_region,
                                                                const uint64_t* __restrict__ blob_off, uint32_t y0,
                                                                uint32_t* __restrict__ region_count,
                                                                uint32_t* __restrict__ blob_irregular,
                                                                uint16_t* __restrict__ sub_count) {
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
    // every word of the region inside the blob and the blob's last byte past it (most regions): the
    // masks need no blob-edge clipping
    const bool interior = word * 16 >= begin + 16 && end > word * 16 + kRegionBytes;
    uint32_t term[kWPT], cont[kWPT], valid[kWPT];        // 16-bit masks of the own word
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        const uint32_t wl = threadIdx.x + k * kThreads;
        const uint32_t cm = cont_mask(v[k]);
        if (interior) {
            term[k] = ~cm & 0xFFFFu;
            cont[k] = cm;
            valid[k] = 0xFFFFu;
        } else {
            const Window W = make_window_cm(cm << 16, word + wl, begin, end);
            term[k] = (W.term & W.valid) >> 16;
            cont[k] = W.cont >> 16;
            valid[k] = W.valid >> 16;
        }
        cm_l[wl + 1] = cont[k];
    }
    if (threadIdx.x == 0) cm_l[0] = make_window(make_uint4(0, 0, 0, 0), halo, word - 1, begin, end).cont >> 16;
    __syncthreads();
    uint32_t n = 0, bad = 0, lng = 0;
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        const uint32_t wl = threadIdx.x + k * kThreads;
        const uint32_t nk = __builtin_popcount(term[k]);
        n += nk;
        if (sub_count) {
            const uint32_t rs = row16_incl_scan(nk);
            if ((threadIdx.x & 15) == 15) sub_count[r * kSubPerRegion + (wl >> 4)] = (uint16_t)rs;
        }
        // runs of continuation bytes ending inside this word (bit j of rK: bytes j-K+1 .. j all continue):
        // 11 in a row = an irregular blob, 5 = an element of >= 6 bytes
        const uint32_t c = (cont[k] << 16) | cm_l[wl];
        const uint32_t r2 = c & (c << 1), r4 = r2 & (r2 << 2), r5 = r4 & (c << 4);
        const uint32_t r8 = r4 & (r4 << 4), r11 = r8 & (r4 << 7);
        bad |= r11 & (valid[k] << 16);
        lng |= r5 & (valid[k] << 16);
    }
    // bit 0: irregular (sequential decoder); bit 1: an element of >= 6 bytes (the fused decode -> combine
    // then takes its multi-round variant)
    if (bad || lng) atomicOr(&blob_irregular[b], (bad ? 1u : 0u) | (lng ? 2u : 0u));
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
                                                               uint64_t* __restrict__ blob_count,
                                                               uint32_t b0 = 0) {
    const uint32_t b = b0 + blockIdx.x;
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

// The element of `len` bytes (1..11, a regular blob) that starts at byte P of the LDS image lb (read
// as funnel-shifted dwords; lb holds at least 12 readable bytes past P): zigzag + LEB128 -> i64.
__device__ __forceinline__ int64_t varint_value_at(const uint32_t* lb, uint32_t P, uint32_t len) {
    const uint32_t q = P >> 2, sh = (P & 3) * 8;
    const uint32_t d0 = lb[q], d1 = lb[q + 1], d2 = lb[q + 2];
    const uint32_t b0 = __builtin_amdgcn_alignbit(d1, d0, sh), b1 = __builtin_amdgcn_alignbit(d2, d1, sh);
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
    return val;
}

// pass C: decode.  Each thread loads its kWPT words of the region up front (all in flight); the region
// is then walked as kWPT sub-regions of one word per thread, each staged in LDS with a 16-byte halo
// (the previous word) and every word's 16-bit continuation mask beside it.  Per sub-region a
// block-wide scan of the terminator counts compacts the elements' starts into LDS; then lane i decodes
// element i (balanced work, coalesced stores) from funnel-shifted dwords -- elements of <= 5 bytes
// (every field share below 2^31) on a short 32-bit path, longer ones on the general one.  Element
// index of a terminator = region base + terminators before it in the region.  Blobs flagged irregular
// are skipped here (varint_sequential_kernel).
//
// OutT = int32_t (the clerk's decode -> combine of field shares, |v| < 2^31): the values are stored
// narrowed and any value that does not fit sets *wide (the caller then decodes again as i64).
//
// SPARSE (the clerk's decode -> combine without a count pass): region r's elements go to its own slots
// out + r * kSlotCap, and the region's element count to region_count[r]; region_base and blob_irregular
// are not read.  A region with more than kSlotCap elements sets *wide, and so does a malformed blob (a run
// of >= 11 continuation bytes always holds an element longer than 5 bytes).
template <typename OutT, bool SPARSE = false, bool NT = false>
__global__ __launch_bounds__(kThreads) void varint_decode_kernel(const uint8_t* __restrict__ bytes,
                                                                 const uint64_t* __restrict__ blob_region,
                                                                 const uint64_t* __restrict__ blob_off, uint32_t y0,
                                                                 const uint64_t* __restrict__ region_base,
                                                                 const uint32_t* __restrict__ blob_irregular,
                                                                 OutT* __restrict__ out, uint64_t out_stride,
                                                                 uint32_t* __restrict__ wide,
                                                                 uint32_t* __restrict__ region_count = nullptr,
                                                                 const uint32_t* __restrict__ skip = nullptr) {
    uint32_t b;
    uint64_t r, word;
    if (skip && *skip) return;                                // a blob exceeds the output row: write nothing
    if (!region_of(blob_region, blob_off, y0, &b, &r, &word)) return;
    if (!SPARSE && (blob_irregular[b] & 1u)) return;
    // LDS holds one sub-region at a time (the region's other words wait in registers): 12.9 KB per
    // workgroup instead of 26.7, so LDS no longer caps the waves per SIMD
    __shared__ uint32_t lb[(kSubBytes + 32) / 4];             // [halo 16 B | sub-region 4 KiB | tail 16 B]
    __shared__ uint16_t cml[kThreads + 1];                    // continuation mask (16 bits) of lb word w at [w]
    __shared__ uint32_t wsum[kThreads / 64];
    // one sub-region's element starts (byte positions in lb) and, after the last, its end: an element
    // ends where the next one starts (the blob's elements are contiguous), so a u16 per element suffices
    __shared__ uint16_t el[kSubBytes + 1];
    uint4* lb4 = reinterpret_cast<uint4*>(lb);
    const uint64_t begin = blob_off[b], end = blob_off[b + 1];
    // every window of the region inside the blob, and the blob's last byte past the region
    const bool interior = word * 16 >= begin + 16 && end > word * 16 + kRegionBytes;
    const uint4* p = reinterpret_cast<const uint4*>(bytes);
    uint4 v[kWPT];
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        const uint64_t wk = word + threadIdx.x + k * kThreads;
        v[k] = wk * 16 < end ? p[wk] : make_uint4(0, 0, 0, 0);
    }
    uint4 h = make_uint4(0, 0, 0, 0);                         // the word before the region (thread 0)
    if (threadIdx.x == 0 && word * 16 > begin) h = p[word - 1];
    if (threadIdx.x == kThreads - 1) lb4[kThreads + 1] = make_uint4(0, 0, 0, 0);
    OutT* dst = SPARSE ? out + r * kSlotCap : out + (uint64_t)b * out_stride + region_base[r];
    bool narrow_fail = false;
    uint32_t base = 0;                                        // elements in earlier sub-regions
#pragma unroll
    for (int k = 0; k < kWPT; ++k) {
        const uint32_t wl = threadIdx.x + k * kThreads;
        const uint32_t cmk = cont_mask(v[k]);
        // terminators of the own word (they do not depend on the previous word) and their block scan
        const Window Wo = interior ? interior_window(cmk << 16) : make_window_cm(cmk << 16, word + wl, begin, end);
        const uint32_t tm = Wo.term & Wo.valid;
        const uint32_t n = __builtin_popcount(tm);
        const uint32_t incl = wave_incl_scan(n);
        if (k > 0) __syncthreads();                           // the previous sub-region's decode is done
        lb4[threadIdx.x + 1] = v[k];
        cml[threadIdx.x + 1] = (uint16_t)cmk;
        if (k == 0 && threadIdx.x == 0) { lb4[0] = h; cml[0] = (uint16_t)cont_mask(h); }
        if (k > 0 && threadIdx.x == kThreads - 1) { lb4[0] = v[k - 1]; cml[0] = (uint16_t)cont_mask(v[k - 1]); }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
        __syncthreads();
        // 1. compaction: each thread lists the starts of the elements ending in its word
        uint32_t e = incl - n, total = 0;
        for (uint32_t w = 0; w < kThreads / 64; ++w) {
            if (w < (threadIdx.x >> 6)) e += wsum[w];
            total += wsum[w];
        }
        if (tm) {
            // the first element starts after the previous boundary (a terminator, or a byte outside
            // the blob); each later one right after the terminator before it
            const uint32_t cm = (uint32_t)cml[threadIdx.x] | (cmk << 16);
            const Window W = interior ? interior_window(cm) : make_window_cm(cm, word + wl, begin, end);
            const uint32_t boundary = W.term | ~(W.term | W.cont);
            const uint32_t pos0 = threadIdx.x * 16;
            uint32_t rem = tm;
            const uint32_t below = boundary & ((1u << __builtin_ctz(rem)) - 1u);
            uint32_t st = below ? 32 - __builtin_clz(below) : 0;      // window index of the first byte
            do {
                const uint32_t j = __builtin_ctz(rem);
                rem &= rem - 1;
                el[e++] = (uint16_t)(pos0 + st);
                st = j + 1;
            } while (rem);
            if (e == total) el[total] = (uint16_t)(pos0 + st);    // end of the sub-region's last element
        }
        __syncthreads();
        // 2. decode: lane i takes element i -> balanced work, coalesced stores
        for (uint32_t i = threadIdx.x; i < total; i += kThreads) {
            const uint32_t P = el[i];                             // byte position in lb
            const uint32_t len = el[i + 1] - P;                   // 1..11 on regular blobs
            if constexpr (sizeof(OutT) < 8) {
                const uint32_t q = P >> 2, sh = (P & 3) * 8;
                const uint32_t d0 = lb[q], d1 = lb[q + 1], d2 = lb[q + 2];
                const uint32_t b0 = __builtin_amdgcn_alignbit(d1, d0, sh), b1 = __builtin_amdgcn_alignbit(d2, d1, sh);
                // int32 output: elements of <= 5 bytes whose zigzag value is below 2^32 (anything
                // else sets *wide and the caller decodes the job as i64)
                const uint32_t l4 = len < 4 ? len : 4u, cut = 32 - 8 * l4;
                uint32_t x = ((b0 << cut) >> cut) & 0x7F7F7F7Fu;
                x = (x & 0x007F007Fu) | ((x >> 1) & ~0x007F007Fu);
                x = (x & 0x00003FFFu) | ((x >> 2) & ~0x00003FFFu);
                const uint32_t g4 = len == 5 ? (b1 & 0x7Fu) : 0u;
                narrow_fail |= len > 5 || g4 > 15;
                const uint32_t zl = x | (g4 << 28);
                const OutT val = (OutT)((zl >> 1) ^ (0u - (zl & 1u)));
                if constexpr (NT) __builtin_nontemporal_store(val, dst + base + i);
                else dst[base + i] = val;
                continue;
            }
            const OutT val = (OutT)varint_value_at(lb, P, len);
            if constexpr (NT) __builtin_nontemporal_store(val, dst + base + i);
            else dst[base + i] = val;
        }
        base += total;
    }
    if constexpr (sizeof(OutT) < 8) {
        if (narrow_fail) atomicOr(wide, 1u);             // rare: one atomic per lane that saw it
    }
    if constexpr (SPARSE) {
        if (threadIdx.x == 0) {
            region_count[r] = base;
            if (base > kSlotCap) atomicOr(wide, 1u);
        }
    }
}

// Nontemporal element stores for the clerk's slots (SPARSE): decode -> combine -1.5 % in-process (2.625 ->
// 2.586 ms at 1000 x 1M); the i64 matrix decode ran 3.5 % slower with them (3.288 -> 3.403 ms) and keeps cached
// stores (profiles/r06ae).  SDA_DEC_NT (read per call; A/B knob) = 0 / 1 forces cached / nontemporal everywhere.
template <typename OutT, bool SPARSE = false>
static auto dec_kernel() {
    const char* e = getenv("SDA_DEC_NT");
    const bool nt = e && (e[0] == '0' || e[0] == '1') ? e[0] == '1' : SPARSE;
    return nt ? varint_decode_kernel<OutT, SPARSE, true> : varint_decode_kernel<OutT, SPARSE, false>;
}

// ---------------- the clerk's decode -> combine over region slots ----------------
// After the SPARSE decode and varint_scan_kernel (region_base = the blob's elements before region r),
// element j of blob b sits in the region r of b with region_base[r] <= j < region_base[r] + count[r],
// at slot r * kSlotCap + (j - region_base[r]).  The combine walks column tiles of `tile` elements.
// A tile's elements lie in at most two regions: every element of this path has <= 5 bytes (any longer
// one sets the wide flag and the job takes the matrix path), so a region the blob covers whole holds
// >= kRegionBytes / 5 > tile elements, and a partial region is the blob's first or last.  The plan
// entry of (tile t, blob b) is therefore self-contained -- no dependent load in the combine:
//   bits  0..38  s0  = slot of the tile's first element (r * kSlotCap + local offset)
//   bits 39..49  c0  = min(elements of the tile in region r, tile)
//   bits 50..63  gap = kSlotCap - count[r]: element o >= c0 of the tile sits at s0 + o + gap
// One thread per (region, blob) emits the entries of the tiles whose first element it holds.
//
// CPL columns per lane: lane l of a tile owns columns CPL*l .. CPL*l + CPL - 1 and reads them with one
// CPL x 4-byte load per blob (tile = CPL x kThreads columns).  The slot index of a tile's first element
// has no alignment, so the loads are only dword-aligned (global loads allow it).
constexpr uint32_t kScMaxTile = 4 * kThreads;
static_assert(kRegionBytes / 5 > kScMaxTile && kSlotCap <= (1u << 14) && kScMaxTile < 2048, "slot plan packing");
__device__ __forceinline__ uint64_t slot_plan_entry(uint64_t s0, uint64_t c0, uint64_t gap) {
    return s0 | (c0 << 39) | (gap << 50);      // s0: 39 bits, c0: 11 bits, gap: 14 bits
}
// The plan and the combine run right behind the decode, before the host has seen the element counts; both
// exit at once when `flags` is set (bit 0: an element the slots cannot hold -- the job takes the matrix
// path; bit 1: the blobs decode to different lengths -- "Wrong dimension"), and the combine also when the
// dimension exceeds the output's capacity.  The host reports those cases after the call's final wait.
// sda_varint_decode_dev's capacity check on the device: *flag = some blob decodes to more than cap values.
__global__ __launch_bounds__(kThreads) void varint_cap_kernel(const uint64_t* __restrict__ blob_count, uint64_t n_blobs,
                                                              uint64_t cap, uint32_t* __restrict__ flag) {
    bool over = false;
    for (uint64_t b = threadIdx.x; b < n_blobs; b += kThreads) over |= blob_count[b] > cap;
    if (over) atomicOr(flag, 1u);
}

// blobs [b0, b1) against blob 0's count
__global__ __launch_bounds__(kThreads) void slot_dims_kernel(const uint64_t* __restrict__ blob_count, uint64_t b1,
                                                             uint32_t* __restrict__ flags, uint64_t b0 = 0) {
    bool bad = false;
    for (uint64_t b = b0 + threadIdx.x; b < b1; b += kThreads) bad |= blob_count[b] != blob_count[0];
    if (bad) atomicOr(flags, 2u);
}

__global__ __launch_bounds__(kThreads) void slot_plan_kernel(const uint64_t* __restrict__ blob_region,
                                                             const uint64_t* __restrict__ region_base,
                                                             const uint32_t* __restrict__ region_count, uint32_t y0,
                                                             uint64_t n_blobs, uint64_t ntiles, uint32_t tile,
                                                             const uint32_t* __restrict__ flags,
                                                             uint64_t* __restrict__ plan, uint64_t pb0 = 0,
                                                             uint64_t rbase = 0) {
    // grouped job (pb0, rbase > 0): blob b of the group [pb0, pb0 + n_blobs) is plan column b - pb0, and its
    // region r sits at slot (r - rbase) * kSlotCap of the group's slot buffer
    if (*flags) return;
    const uint64_t b = pb0 + y0 + blockIdx.y;
    const uint64_t r0 = blob_region[b], r1 = blob_region[b + 1];
    const uint64_t r = r0 + (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (r >= r1) return;
    const uint32_t cnt = region_count[r];
    const uint64_t E0 = region_base[r], E1 = E0 + cnt;
    const uint64_t gap = kSlotCap - cnt;
    for (uint64_t t = (E0 + tile - 1) / tile; t < ntiles && t * tile < E1; ++t) {
        const uint64_t local = t * tile - E0;
        const uint64_t c0 = E1 - t * tile < tile ? E1 - t * tile : tile;
        plan[t * n_blobs + (b - pb0)] = slot_plan_entry((r - rbase) * kSlotCap + local, c0, gap);
    }
}

// One workgroup per column tile: lane l owns CPL adjacent columns and walks the blobs in reference order
// through combiner.rs:16-28's exact recurrence (add_trem).  Blobs go UNROLL at a time: their plan entries
// are uniform (scalar loads) and give every slot address directly, so all UNROLL slot loads are issued
// before the dependent chain.  The one lane whose columns straddle the region boundary (c0) also loads
// them past the gap and merges.  dim = blob 0's element count, read on the device; the grid covers the
// host's bound (blob 0's bytes), and runs only when every blob decoded to dim elements (flags clear); a
// lane's load may run past the blob's last element into unused slots (never past the buffer: the tile
// plan follows the slots).
template <int CPL, int UNROLL, bool SMALL_M>
__global__ __launch_bounds__(kThreads) void slot_combine_kernel(const int32_t* __restrict__ slots,
                                                                const uint64_t* __restrict__ plan,
                                                                uint64_t n_blobs, const uint64_t* __restrict__ dim_p,
                                                                const uint32_t* __restrict__ flags, uint64_t out_cap,
                                                                int64_t* __restrict__ out, Mod64 M,
                                                                const int64_t* __restrict__ acc_in = nullptr) {
    typedef typename std::conditional<CPL == 1, int32_t,
            int32_t __attribute__((ext_vector_type(CPL == 1 ? 2 : CPL)))>::type V;
    constexpr uint32_t kTile = CPL * kThreads;
    const uint64_t dim = *dim_p;
    if (*flags || dim > out_cap) return;
    // natural order: the XCD-chunked order (xcd.h) made this read-only walk 1.6x slower (profiles/r04d)
    const uint64_t tile = blockIdx.x;
    const uint64_t e0 = tile * kTile;
    const uint32_t o = CPL * threadIdx.x;
    if (e0 + o >= dim) return;
    const uint64_t* pl = plan + tile * n_blobs;
    auto get = [&](const V& v, int i) -> int32_t {
        if constexpr (CPL == 1) return v; else return v[i];
    };
    auto load = [&](uint64_t pe) -> V {
        const uint64_t s0 = pe & ((1ull << 39) - 1);
        const uint32_t c0 = (uint32_t)(pe >> 39) & 2047u, gap = (uint32_t)(pe >> 50);
        V v = __builtin_nontemporal_load(reinterpret_cast<const V*>(slots + s0 + o + (o >= c0 ? gap : 0u)));
        if constexpr (CPL > 1) {
            if (o < c0 && o + CPL > c0) {          // the lane straddling the region boundary
                const V w = __builtin_nontemporal_load(reinterpret_cast<const V*>(slots + s0 + o + gap));
#pragma unroll
                for (int i = 0; i < CPL; ++i)
                    if (o + i >= c0) v[i] = w[i];
            }
        }
        return v;
    };
    int64_t acc[CPL];     // the recurrence's state: 0, or where the previous group of blobs left it
#pragma unroll
    for (int i = 0; i < CPL; ++i) acc[i] = (acc_in && e0 + o + i < dim) ? acc_in[e0 + o + i] : 0;
    uint64_t b = 0;
    for (; b + UNROLL <= n_blobs; b += UNROLL) {
        V v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = load(pl[b + u]);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int i = 0; i < CPL; ++i) acc[i] = add_trem(acc[i], get(v[u], i), M, SMALL_M);
    }
    for (; b < n_blobs; ++b) {
        const V v = load(pl[b]);
#pragma unroll
        for (int i = 0; i < CPL; ++i) acc[i] = add_trem(acc[i], get(v, i), M, SMALL_M);
    }
#pragma unroll
    for (int i = 0; i < CPL; ++i)
        if (e0 + o + i < dim) out[e0 + o + i] = acc[i];
}

// grouped slot path: the finished state goes to out only when no flag is set and the dimension fits
__global__ __launch_bounds__(kThreads) void slot_commit_kernel(const int64_t* __restrict__ acc,
                                                               const uint64_t* __restrict__ dim_p,
                                                               const uint32_t* __restrict__ flags, uint64_t out_cap,
                                                               int64_t* __restrict__ out) {
    const uint64_t dim = *dim_p;
    if (*flags || dim > out_cap) return;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < dim; i += (uint64_t)gridDim.x * kThreads)
        out[i] = acc[i];
}

// ---------------- the clerk's fused decode -> combine ----------------
// Column tile of the fused decode -> combine: 1,536 columns = 3 per lane of a 512-lane workgroup.  With
// elements of <= 5 bytes (every field share: |v| < 2^31) a tile's slice of a payload is at most
// 256 + 5 x 1536 + 256 = 8 KiB = one 16-byte word per lane.
constexpr uint32_t kDcThreads = 512;
constexpr uint32_t kDcTile = 3 * kDcThreads;

// Per (column tile t >= 1, blob b): the 256-byte sub-chunk holding the terminator of element t*kDcTile - 1
// (the previous tile's last element) and the number of the blob's terminators in that sub-chunk up to
// and including it; tile 0 starts at the blob's first byte.  plan[t * n_blobs + b] = byte << 16 | skip.
// One thread per (region, blob) (grid.y = blob): it emits the entries of every tile whose boundary
// element falls in its region, walking the region's 64 sub-chunk counts once (no search).
__global__ __launch_bounds__(kThreads) void varint_tile_plan_kernel(const uint64_t* __restrict__ blob_off,
                                                                    const uint64_t* __restrict__ blob_region,
                                                                    const uint64_t* __restrict__ region_base,
                                                                    const uint16_t* __restrict__ sub_count,
                                                                    uint32_t y0, uint64_t n_blobs, uint64_t ntiles,
                                                                    uint64_t* __restrict__ plan) {
    const uint64_t b = y0 + blockIdx.y;
    const uint64_t r0 = blob_region[b], r1 = blob_region[b + 1];
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    const uint64_t beg = blob_off[b];
    if (i == 0) plan[b] = (beg & ~(uint64_t)15) << 16;              // tile 0
    if (r0 + i >= r1) return;
    const uint64_t r = r0 + i;
    const uint64_t E0 = region_base[r];
    const uint64_t E1 = r + 1 < r1 ? region_base[r + 1] : ~(uint64_t)0;   // last region: to the blob's end
    // tiles t >= 1 whose boundary element t*T - 1 lies in [E0, E1)
    uint64_t t = E0 / kDcTile + 1;
    if (t >= ntiles || t * kDcTile - 1 >= E1) return;
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    const u32x4_t* sc4 = reinterpret_cast<const u32x4_t*>(sub_count + r * kSubPerRegion);
    u32x4_t w[kSubPerRegion / 8];
    static_for<0, kSubPerRegion / 8>([&](auto j) { w[j] = sc4[j]; });
    const uint64_t rbyte = (beg / kRegionBytes + i) * kRegionBytes;
    uint64_t E = E0, e = t * kDcTile - 1;
    static_for<0, kSubPerRegion>([&](auto s) {
        const uint32_t c = (w[s / 8][(s % 8) / 2] >> (16 * (s % 2))) & 0xFFFFu;
        while (e < E + c && e < E1 && t < ntiles) {                 // boundary e in sub-chunk s
            plan[t * n_blobs + b] = ((rbyte + (uint64_t)s * kSubChunk) << 16) | (e - E + 1);
            ++t;
            e += kDcTile;
        }
        E += c;
    });
}

// make_window_cm in 32-bit offsets relative to a slice start: own word at byte w0 (>= 0), the blob at
// [lo_b, hi_b) (clamped to +-2^30 by the caller).
__device__ __forceinline__ Window window_rel(uint32_t cm, int32_t w0, int32_t lo_b, int32_t hi_b) {
    Window W;
    const int32_t lo = lo_b - (w0 - 16), hi = hi_b - (w0 - 16);
    const int l = lo < 0 ? 0 : (lo > 32 ? 32 : lo);
    const int h = hi < 0 ? 0 : (hi > 32 ? 32 : hi);
    uint32_t in = 0;
    if (h > l) in = (h - l == 32 ? 0xFFFFFFFFu : ((1u << (h - l)) - 1u)) << l;
    W.valid = in & 0xFFFF0000u;
    const uint32_t lastbit = (hi >= 1 && hi <= 32) ? 1u << (hi - 1) : 0u;
    W.cont = cm & in;
    W.term = (~cm & in) | (lastbit & in);
    return W;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_word(const uint8_t* bytes, uint64_t w) {      // read once: non-temporal
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(bytes) + w);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// One workgroup (512 lanes) per column tile [e0, e0 + kDcTile): for every blob in order, its tile slice
// -- the words from the plan's sub-chunk to the end of the sub-chunk the next tile's plan points at, one
// per lane -- is staged in LDS, one block scan ranks its terminators, the ones with rank in
// [skip, skip + tile) are compacted as (start, length), and lane l decodes elements l, l + 512, l + 1024
// (its own columns) straight into combiner.rs:16-28's recurrence (add_trem: exact for signed shares,
// reference order).  LDS images are double-buffered by round parity, so a round takes two barriers.
// MULTI (the job has an element of >= 6 bytes): a slice longer than 512 words takes further rounds, the
// previous round's last word as the halo; otherwise the body is straight-line, which keeps hipcc's load
// counters exact.  Each lane's round-0 word is loaded DEPTH blobs ahead (register ring), so DEPTH blobs'
// loads are in flight while one is decoded.  Regular blobs only (no run of 11 continuation bytes).
template <int DEPTH, bool MULTI>
__global__ __launch_bounds__(kDcThreads) __attribute__((amdgpu_waves_per_eu(6, 8)))
void varint_decode_combine_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ blob_off,
                                  uint64_t n_blobs, const uint64_t* __restrict__ plan, uint64_t ntiles,
                                  uint64_t dim, int64_t* __restrict__ out, Mod64 M, bool small_m) {
    constexpr uint32_t NT = kDcThreads, NW = kDcThreads, TILE = kDcTile, COLS = TILE / NT;
    __shared__ uint4 lb4[2][NW + 2];                      // [halo word | NW words | zero tail] per parity
    __shared__ uint32_t cml[2][NW + 1];                   // continuation mask of lb4[.][w] at [w]
    __shared__ uint32_t wsum[NT / 64];
    __shared__ uint32_t el[2][TILE];                      // element i of the tile: start | len << 16
    __shared__ uint4 halo4;                               // the last word of the previous round (MULTI)
    __shared__ uint32_t halo_cm;
    const uint32_t tid = threadIdx.x;
    const uint64_t t = blockIdx.x;
    const uint64_t e0 = t * TILE;
    const uint32_t tile = (uint32_t)(dim - e0 < TILE ? dim - e0 : TILE);
    if (tid < 2) lb4[tid][NW + 1] = make_uint4(0, 0, 0, 0);
    uint32_t par = 0;                                     // LDS parity of the current round

    // the tile's slice of blob b: words [a / 16, (end + 15) / 16); terminators of rank < skip end the
    // previous tile's elements
    struct Slice { uint64_t wa, nw, beg, bend; uint32_t skip; };
    auto slice = [&](uint64_t b) {
        Slice S;
        const uint64_t pe = plan[t * n_blobs + b];
        S.wa = pe >> 20;
        S.skip = (uint32_t)(pe & 0xFFFF);
        S.beg = blob_off[b];
        S.bend = blob_off[b + 1];
        uint64_t end = S.bend;
        if (t + 1 < ntiles) {
            const uint64_t an = (plan[(t + 1) * n_blobs + b] >> 16) + kSubChunk;
            end = an < S.bend ? an : S.bend;
        }
        S.nw = ((end + 15) >> 4) - S.wa;
        return S;
    };
    // unconditional load (clamped into the slice): a load under a lane branch leaves the wait counter
    // unknown at the join, and hipcc then drains every load in flight (vmcnt(0)) at the ring's use
    auto load_word = [&](uint64_t wa, uint64_t nw, uint64_t r0) {
        const uint64_t w = r0 + tid;
        return nt_word(bytes, wa + (w < nw ? w : nw - 1));
    };

    int64_t acc[COLS];
    static_for<0, COLS>([&](auto c) { acc[c] = 0; });

    // One round over words [r0, r0 + NW) of slice S (v: this lane's word, zero past the slice): stage in
    // LDS, rank the terminators, compact the tile's elements among them, decode this lane's columns.
    // `staged()` runs once the word is in LDS (the ring slot it came from may be refilled).  Returns the
    // round's terminator count.
    auto round = [&](const Slice& S, int32_t lo_b, int32_t hi_b, uint64_t r0, uint32_t rank, const uint4& v,
                     auto&& staged) __attribute__((always_inline)) {
        const uint32_t skip = S.skip;
        uint4* L4 = lb4[par];
        uint32_t* CM = cml[par];
        uint32_t* EL = el[par];
        const uint32_t cm = cont_mask(v);
        L4[tid + 1] = v;
        CM[tid + 1] = cm;
        const int32_t w0 = (int32_t)((r0 + tid) * 16);
        const Window Wo = window_rel(cm << 16, w0, lo_b, hi_b);
        const uint32_t tm = Wo.term & Wo.valid;
        const uint32_t n = __builtin_popcount(tm);
        staged();
        if (tid == 0) {
            if (!MULTI || r0 == 0) { L4[0] = make_uint4(0, 0, 0, 0); CM[0] = 0; }
            else { L4[0] = halo4; CM[0] = halo_cm; }
        }
        const uint32_t incl = wave_incl_scan(n);
        if ((tid & 63) == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        uint32_t q = rank + incl - n, total = 0;
        static_for<0, NT / 64>([&](auto w) {
            const uint32_t x = wsum[w];
            if ((uint32_t)w < (tid >> 6)) q += x;
            total += x;
        });
        if (tm && q + n > skip && q < skip + tile) {
            // element starts as in pass C (previous boundary in the 32-byte window)
            const Window W = window_rel(CM[tid] | (cm << 16), w0, lo_b, hi_b);
            const uint32_t boundary = W.term | ~(W.term | W.cont);
            const uint32_t pos0 = tid * 16;
            uint32_t rem = tm;
            const uint32_t below = boundary & ((1u << __builtin_ctz(rem)) - 1u);
            uint32_t st = below ? 32 - __builtin_clz(below) : 0;
            do {
                const uint32_t j = __builtin_ctz(rem);
                rem &= rem - 1;
                const uint32_t i = q - skip;              // wraps (huge) below skip
                if (i < tile) EL[i] = (pos0 + st) | ((j - st + 1) << 16);
                ++q;
                st = j + 1;
            } while (rem);
        }
        if (MULTI && tid == 0 && r0 + NW < S.nw) { halo4 = L4[NW]; halo_cm = CM[NW]; }
        __syncthreads();
        // elements [ilo, ihi) of the tile end in this round; lane l owns columns l + 512 c
        const uint32_t ilo = rank > skip ? (rank - skip < tile ? rank - skip : tile) : 0u;
        const uint32_t ihi = rank + total > skip ? (rank + total - skip < tile ? rank + total - skip : tile) : 0u;
        const uint32_t* lb = reinterpret_cast<const uint32_t*>(L4);
        static_for<0, COLS>([&](auto c) {
            const uint32_t i = tid + c * NT;
            if (i >= ilo && i < ihi) {
                const uint32_t e = EL[i];
                acc[c] = add_trem(acc[c], varint_value_at(lb, e & 0xFFFFu, e >> 16), M, small_m);
            }
        });
        par ^= 1u;
        return total;
    };

    // blob b: round 0 straight from its ring slot (refilled with blob `next`'s word as soon as it is
    // staged); further rounds (MULTI) load their words synchronously
    auto blob = [&](uint64_t b, uint4& slot, bool refill, uint64_t next) __attribute__((always_inline)) {
        const Slice S = slice(b);
        auto rel = [&](uint64_t x) {                      // blob bounds in bytes from the slice start
            const int64_t d = (int64_t)(x - (S.wa << 4));
            return (int32_t)(d < -(1ll << 30) ? -(1ll << 30) : (d > (1ll << 30) ? (1ll << 30) : d));
        };
        const int32_t lo_b = rel(S.beg), hi_b = rel(S.bend);
        const uint4 v = tid < S.nw ? slot : make_uint4(0, 0, 0, 0);
        uint32_t rank = round(S, lo_b, hi_b, 0, 0, v, [&] {
            if (refill) { const Slice N = slice(next); slot = load_word(N.wa, N.nw, 0); }
        });
        if constexpr (MULTI) {
            for (uint64_t r0 = NW; r0 < S.nw && rank < S.skip + tile; r0 += NW) {
                const uint4 w = load_word(S.wa, S.nw, r0);
                rank += round(S, lo_b, hi_b, r0, rank, r0 + tid < S.nw ? w : make_uint4(0, 0, 0, 0), [] {});
            }
        }
    };

    // The ring's loads and refills are unconditional (a refill past the last blob re-reads the last
    // blob's slice): a load on one side of a branch makes hipcc's counter state at the join treat it as
    // the newest, and the slot's use then waits for every load in flight.
    uint4 ring[DEPTH];
    static_for<0, DEPTH>([&](auto u) {
        const Slice S = slice((uint64_t)u < n_blobs ? (uint64_t)u : n_blobs - 1);
        ring[u] = load_word(S.wa, S.nw, 0);
    });
    uint64_t b0 = 0;
    for (; b0 + DEPTH <= n_blobs; b0 += DEPTH) {
        static_for<0, DEPTH>([&](auto u) {
            const uint64_t nb = b0 + u + DEPTH;
            blob(b0 + u, ring[u], true, nb < n_blobs ? nb : n_blobs - 1);
        });
    }
    static_for<0, DEPTH>([&](auto u) {                  // the last n_blobs % DEPTH blobs
        if (b0 + u < n_blobs) blob(b0 + u, ring[u], false, 0);
    });
    static_for<0, COLS>([&](auto c) {
        if (tid + c * NT < tile) out[e0 + tid + c * NT] = acc[c];
    });
}

// Irregular blobs: the reference loop, one lane per blob (only malformed streams get here).
// With out == nullptr it only counts.
__global__ void varint_sequential_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ blob_off,
                                         uint32_t n_blobs, const uint32_t* __restrict__ blob_irregular,
                                         uint64_t* __restrict__ blob_count, int64_t* __restrict__ out,
                                         uint64_t out_stride, uint64_t cap, const uint32_t* __restrict__ skip = nullptr) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_blobs || !(blob_irregular[b] & 1u) || (out && skip && *skip)) return;
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
// Chunk (c, row) starts at dst + row_base[row] + chunk_off (the exclusive scan of the row's chunk_bytes);
// nothing is written when *too_big (the rows do not fit dst_cap).
template <bool NT>
__global__ __launch_bounds__(kThreads) void varint_write_kernel(const int64_t* __restrict__ vals, uint64_t len,
                                                                uint64_t stride, uint32_t chunks,
                                                                const uint64_t* __restrict__ chunk_off,
                                                                const uint64_t* __restrict__ row_base,
                                                                const uint32_t* __restrict__ too_big,
                                                                uint8_t* __restrict__ dst) {
    const uint32_t c = blockIdx.x, row = blockIdx.y;
    if (*too_big) return;
    const uint64_t e0 = (uint64_t)c * kEncChunk;
    constexpr uint32_t kBufQuads = (kEncChunk * 10 + 32) / 16;      // lead < 16, + the shifted tail dwords
    __shared__ uint4 buf4[kBufQuads];
    __shared__ uint32_t wsum[kThreads / 64];
    uint32_t* buf = reinterpret_cast<uint32_t*>(buf4);
    const uint8_t* b8 = reinterpret_cast<const uint8_t*>(buf4);
    uint8_t* gdst = dst + row_base[row] + chunk_off[(uint64_t)row * chunks + c];
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
            if constexpr (NT)
                __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(buf4)[k], reinterpret_cast<u32x4*>(d128) + k);
            else d128[k] = buf4[k];
        } else {
            for (uint32_t i = lo; i < hi; ++i)
                if (i >= lead && i < end) d8[i] = b8[i];
        }
    }
}

// exclusive scan of chunk_bytes per row (one block per row) + row base; row_bytes = total
// One workgroup: rows placed back to back -- row_base = exclusive scan of row_bytes; *too_big = the total
// exceeds cap (the write pass then writes nothing and the host reports it).
__global__ __launch_bounds__(kThreads) void varint_rows_kernel(const uint64_t* __restrict__ row_bytes, uint64_t rows,
                                                               uint64_t cap, uint64_t* __restrict__ row_base,
                                                               uint32_t* __restrict__ too_big) {
    __shared__ uint64_t part[kThreads];
    uint64_t carry = 0;
    for (uint64_t base = 0; base < rows; base += kThreads) {
        const uint64_t r = base + threadIdx.x;
        const uint64_t v = r < rows ? row_bytes[r] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < kThreads; o <<= 1) {
            const uint64_t add = threadIdx.x >= (uint32_t)o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += add;
            __syncthreads();
        }
        if (r < rows) row_base[r] = carry + part[threadIdx.x] - v;
        carry += part[kThreads - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) *too_big = carry > cap ? 1u : 0u;
}

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
    uint16_t* sub_count;
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
    w.wide = (uint32_t*)p; p += 256;
    w.sub_count = (uint16_t*)p;
    return w;
}
size_t varint_decode_work_bytes(size_t regions, uint64_t n_blobs) {
    // (7 x 256 B of rounding + flag) + the sub-chunk counts of the fused decode -> combine
    return regions * 12 + (n_blobs + 1) * 16 + n_blobs * 12 + 8 * 256 + regions * 2 * kSubPerRegion;
}
uint64_t varint_tile_plan_bytes(uint64_t n_blobs, uint64_t dim) {
    return n_blobs * ((dim + kDcTile - 1) / kDcTile) * 8;
}
uint64_t varint_fused_tiles(uint64_t dim) { return (dim + kDcTile - 1) / kDcTile; }

hipError_t launch_varint_count(const uint8_t* bytes, const uint64_t* blob_off_host, uint64_t n_blobs,
                               const VarintPlan& plan, void* work, uint64_t* counts_host, bool* irregular_any,
                               hipStream_t s, bool sub_counts, bool* long_any) {
    const size_t R = plan.regions;
    DecodeWork w = carve(work, R, n_blobs);
    hipError_t e;
    if ((e = hipMemcpyAsync(w.blob_off, blob_off_host, (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(w.blob_region, plan.blob_region.data(), (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.irregular, 0, n_blobs * 4, s)) != hipSuccess) return e;
    for (uint64_t y0 = 0; R && y0 < n_blobs; y0 += 65535) {
        const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
        hipLaunchKernelGGL(varint_count_kernel, dim3((unsigned)plan.max_regions, ny), dim3(kThreads), 0, s, bytes,
                           w.blob_region, w.blob_off, (uint32_t)y0, w.region_count, w.irregular,
                           sub_counts ? w.sub_count : nullptr);
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
    bool lng = false;
    for (uint64_t b = 0; b < n_blobs; ++b) {
        *irregular_any |= (irr[b] & 1u) != 0;
        lng |= (irr[b] & 2u) != 0;
    }
    if (long_any) *long_any = lng;
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
        hipLaunchKernelGGL(dec_kernel<int64_t>(), dim3((unsigned)plan.max_regions, ny), dim3(kThreads), 0, s,
                           bytes, w.blob_region, w.blob_off, (uint32_t)y0, w.region_base, w.irregular, out, out_stride,
                           w.wide, (uint32_t*)nullptr, (const uint32_t*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (irregular_any) {
        hipLaunchKernelGGL(varint_sequential_kernel, dim3((unsigned)((n_blobs + 63) / 64)), dim3(64), 0, s, bytes,
                           w.blob_off, (uint32_t)n_blobs, w.irregular, w.blob_count, out, out_stride, len);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_varint_decode_one_wait(const uint8_t* bytes, const uint64_t* blob_off_host, uint64_t n_blobs,
                                        const VarintPlan& plan, void* work, int64_t* out, uint64_t out_stride,
                                        uint64_t* counts_host, bool* too_long, hipStream_t s) {
    const size_t R = plan.regions;
    DecodeWork w = carve(work, R, n_blobs);
    hipError_t e;
    if ((e = hipMemcpyAsync(w.blob_off, blob_off_host, (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(w.blob_region, plan.blob_region.data(), (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.irregular, 0, n_blobs * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.wide, 0, sizeof(uint32_t), s)) != hipSuccess) return e;      // the capacity flag
    for (uint64_t y0 = 0; R && y0 < n_blobs; y0 += 65535) {
        const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
        hipLaunchKernelGGL(varint_count_kernel, dim3((unsigned)plan.max_regions, ny), dim3(kThreads), 0, s, bytes,
                           w.blob_region, w.blob_off, (uint32_t)y0, w.region_count, w.irregular, (uint16_t*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(varint_scan_kernel, dim3((unsigned)n_blobs), dim3(kThreads), 0, s, w.region_count,
                       w.blob_region, w.region_base, w.blob_count);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const unsigned seq_grid = (unsigned)((n_blobs + 63) / 64);
    hipLaunchKernelGGL(varint_sequential_kernel, dim3(seq_grid), dim3(64), 0, s, bytes, w.blob_off, (uint32_t)n_blobs,
                       w.irregular, w.blob_count, (int64_t*)nullptr, 0, 0, (const uint32_t*)nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(varint_cap_kernel, dim3(1), dim3(kThreads), 0, s, (const uint64_t*)w.blob_count, n_blobs,
                       out_stride, w.wide);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    for (uint64_t y0 = 0; R && y0 < n_blobs; y0 += 65535) {
        const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
        hipLaunchKernelGGL(dec_kernel<int64_t>(), dim3((unsigned)plan.max_regions, ny), dim3(kThreads), 0, s,
                           bytes, w.blob_region, w.blob_off, (uint32_t)y0, w.region_base, w.irregular, out, out_stride,
                           (uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)w.wide);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(varint_sequential_kernel, dim3(seq_grid), dim3(64), 0, s, bytes, w.blob_off, (uint32_t)n_blobs,
                       w.irregular, w.blob_count, out, out_stride, out_stride, (const uint32_t*)w.wide);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the call's one wait: the counts and the capacity flag, after the whole job
    uint32_t flag = 0;
    if ((e = hipMemcpyAsync(counts_host, w.blob_count, n_blobs * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&flag, w.wide, sizeof(flag), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *too_long = flag != 0;
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
        hipLaunchKernelGGL(dec_kernel<int32_t>(), dim3((unsigned)plan.max_regions, ny), dim3(kThreads), 0, s,
                           bytes, w.blob_region, w.blob_off, (uint32_t)y0, w.region_base, w.irregular, out, out_stride,
                           w.wide, (uint32_t*)nullptr, (const uint32_t*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    uint32_t flag = 0;
    if ((e = hipMemcpyAsync(&flag, w.wide, sizeof(flag), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *wide_host = flag != 0;
    return hipSuccess;
}

// Columns per lane of the slot combine (SDA_SLOT_CPL = 1, 2 or 4: A/B knob; default 4).
static uint32_t slot_cpl() {
    const char* e = getenv("SDA_SLOT_CPL");
    const int v = e ? atoi(e) : 4;
    return (v == 1 || v == 2) ? (uint32_t)v : 4u;
}

// Blobs per group of the slot path (SDA_CODEC_GROUP; 0 = the whole job in one pass).  Grouped, each group
// is decoded into one reused slot buffer and combined from it at once, while its slots may still sit in the
// caches, the recurrence's state carried from group to group in a scratch row.
static uint64_t slot_group() {
    const char* e = getenv("SDA_CODEC_GROUP");
    return e ? strtoull(e, nullptr, 10) : 0;
}
struct SlotGroups {
    uint64_t G;            // blobs per group (0: one pass)
    uint64_t regions;      // slot regions of the largest group (all regions in one pass)
};
static SlotGroups slot_groups(const VarintPlan& plan, uint64_t n_blobs) {
    const uint64_t G = std::min<uint64_t>(slot_group(), 65535);     // grid.y of a group's launches
    if (G == 0 || G >= n_blobs) return {0, plan.regions};
    uint64_t mx = 0;
    for (uint64_t g0 = 0; g0 < n_blobs; g0 += G) {
        const uint64_t g1 = g0 + G < n_blobs ? g0 + G : n_blobs;
        mx = std::max<uint64_t>(mx, plan.blob_region[g1] - plan.blob_region[g0]);
    }
    return {G, mx};
}
// slot buffer layout: [slots | tile plan | (grouped) the recurrence's state, dim i64]
static size_t slot_area_bytes(uint64_t regions) { return (regions * kSlotCap + (kRegionBytes - kSlotCap)) * sizeof(int32_t); }

size_t varint_slot_bytes(const VarintPlan& plan, uint64_t n_blobs, uint64_t dim) {
    const uint64_t ntiles = (dim + kThreads - 1) / kThreads;          // plan room for the smallest tile
    const SlotGroups sg = slot_groups(plan, n_blobs);
    return slot_area_bytes(sg.regions) + ntiles * (sg.G ? sg.G : n_blobs) * 8 + (sg.G ? dim * 8 : 0) + 256;
}

hipError_t launch_varint_decode_slots_combine(const uint8_t* bytes, const uint64_t* blob_off_host, uint64_t n_blobs,
                                              const VarintPlan& plan, void* work, void* slot_buf, int64_t* out,
                                              uint64_t out_cap, int64_t modulus, uint64_t* counts_host,
                                              uint32_t* flags_host, hipStream_t s) {
    const size_t R = plan.regions;
    DecodeWork w = carve(work, R, n_blobs);
    const SlotGroups sg = slot_groups(plan, n_blobs);
    int32_t* slots = static_cast<int32_t*>(slot_buf);
    uint64_t* tplan = reinterpret_cast<uint64_t*>(static_cast<char*>(slot_buf) + slot_area_bytes(sg.regions));
    const uint32_t cpl = slot_cpl(), tile = cpl * kThreads;
    // the grid's bound: blob 0 decodes to at most one element per byte
    const uint64_t ntiles = (blob_off_host[1] - blob_off_host[0] + tile - 1) / tile;
    if (ntiles > 0x7FFFFFFFull || R * kSlotCap >= (1ull << 39)) return hipErrorInvalidValue;
    hipError_t e;
    if ((e = hipMemcpyAsync(w.blob_off, blob_off_host, (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(w.blob_region, plan.blob_region.data(), (n_blobs + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.wide, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    const Mod64 M = make_mod64(modulus > 0 ? modulus : 1);
    const bool small_m = modulus <= ((int64_t)1 << 62);
#define SLOT_COMBINE(C, SM, NB, DST, ACC_IN)                                                                       \
    hipLaunchKernelGGL((slot_combine_kernel<C, 8, SM>), dim3((unsigned)ntiles), dim3(kThreads), 0, s, slots,         \
                       (const uint64_t*)tplan, NB, (const uint64_t*)w.blob_count, (const uint32_t*)w.wide, out_cap, \
                       DST, M, ACC_IN)
#define SLOT_COMBINE_ANY(NB, DST, ACC_IN)                                                                            \
    do {                                                                                                             \
        if (cpl == 4) { if (small_m) SLOT_COMBINE(4, true, NB, DST, ACC_IN); else SLOT_COMBINE(4, false, NB, DST, ACC_IN); } \
        else if (cpl == 2) { if (small_m) SLOT_COMBINE(2, true, NB, DST, ACC_IN); else SLOT_COMBINE(2, false, NB, DST, ACC_IN); } \
        else { if (small_m) SLOT_COMBINE(1, true, NB, DST, ACC_IN); else SLOT_COMBINE(1, false, NB, DST, ACC_IN); } \
    } while (0)
    if (sg.G) {
        // grouped: decode, scan, check and combine one group of blobs at a time through the one slot buffer
        // (region r of the group starting at blob g0 sits at slot (r - blob_region[g0]) * kSlotCap); the
        // state carried between groups lives in `acc`, and reaches out only if the whole job is clean
        int64_t* acc = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(tplan) + ntiles * sg.G * 8);
        for (uint64_t g0 = 0; g0 < n_blobs; g0 += sg.G) {
            const uint64_t g1 = g0 + sg.G < n_blobs ? g0 + sg.G : n_blobs;
            const uint64_t ng = g1 - g0, R0 = plan.blob_region[g0];
            if (plan.blob_region[g1] > R0) {
                hipLaunchKernelGGL((dec_kernel<int32_t, true>()), dim3((unsigned)plan.max_regions, (unsigned)ng),
                                   dim3(kThreads), 0, s, bytes, w.blob_region, w.blob_off, (uint32_t)g0,
                                   (const uint64_t*)nullptr, (const uint32_t*)nullptr, slots - R0 * kSlotCap, 0, w.wide,
                                   w.region_count, (const uint32_t*)nullptr);
                if ((e = hipGetLastError()) != hipSuccess) return e;
            }
            hipLaunchKernelGGL(varint_scan_kernel, dim3((unsigned)ng), dim3(kThreads), 0, s, w.region_count,
                               w.blob_region, w.region_base, w.blob_count, (uint32_t)g0);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            hipLaunchKernelGGL(slot_dims_kernel, dim3(1), dim3(kThreads), 0, s, (const uint64_t*)w.blob_count, g1,
                               w.wide, g0);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            if (ntiles && modulus > 0) {
                hipLaunchKernelGGL(slot_plan_kernel, dim3((unsigned)((plan.max_regions + kThreads - 1) / kThreads),
                                   (unsigned)ng), dim3(kThreads), 0, s, w.blob_region, w.region_base, w.region_count,
                                   0u, ng, ntiles, tile, (const uint32_t*)w.wide, tplan, g0, R0);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                SLOT_COMBINE_ANY(ng, acc, g0 ? (const int64_t*)acc : (const int64_t*)nullptr);
                if ((e = hipGetLastError()) != hipSuccess) return e;
            }
        }
        if (ntiles && modulus > 0) {
            hipLaunchKernelGGL(slot_commit_kernel, dim3(2048), dim3(kThreads), 0, s, (const int64_t*)acc,
                               (const uint64_t*)w.blob_count, (const uint32_t*)w.wide, out_cap, out);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        if ((e = hipMemcpyAsync(counts_host, w.blob_count, n_blobs * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(flags_host, w.wide, sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        return hipStreamSynchronize(s);
    }
    for (uint64_t y0 = 0; R && y0 < n_blobs; y0 += 65535) {
        const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
        hipLaunchKernelGGL((dec_kernel<int32_t, true>()), dim3((unsigned)plan.max_regions, ny), dim3(kThreads),
                           0, s, bytes, w.blob_region, w.blob_off, (uint32_t)y0, (const uint64_t*)nullptr,
                           (const uint32_t*)nullptr, slots, 0, w.wide, w.region_count, (const uint32_t*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(varint_scan_kernel, dim3((unsigned)n_blobs), dim3(kThreads), 0, s, w.region_count,
                       w.blob_region, w.region_base, w.blob_count);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(slot_dims_kernel, dim3(1), dim3(kThreads), 0, s, (const uint64_t*)w.blob_count, n_blobs, w.wide);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ntiles && modulus > 0) {       // modulus 0: invalid -- no combine (an error if the dimension is > 0)
        for (uint64_t y0 = 0; y0 < n_blobs; y0 += 65535) {
            const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
            hipLaunchKernelGGL(slot_plan_kernel, dim3((unsigned)((plan.max_regions + kThreads - 1) / kThreads), ny),
                               dim3(kThreads), 0, s, w.blob_region, w.region_base, w.region_count, (uint32_t)y0,
                               n_blobs, ntiles, tile, (const uint32_t*)w.wide, tplan);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        SLOT_COMBINE_ANY(n_blobs, out, (const int64_t*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
#undef SLOT_COMBINE_ANY
#undef SLOT_COMBINE
    // the call's one wait: the counts and the flags, after the whole job
    if ((e = hipMemcpyAsync(counts_host, w.blob_count, n_blobs * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(flags_host, w.wide, sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

hipError_t launch_varint_decode_combine(const uint8_t* bytes, uint64_t n_blobs, const VarintPlan& plan, void* work,
                                        uint64_t* tile_plan, uint64_t dim, int64_t* out, int64_t modulus,
                                        bool multi, hipStream_t s) {
    if (dim == 0 || n_blobs == 0) return hipSuccess;
    const size_t R = plan.regions;
    DecodeWork w = carve(work, R, n_blobs);
    const uint64_t ntiles = varint_fused_tiles(dim);
    if (ntiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipError_t e;
    for (uint64_t y0 = 0; y0 < n_blobs; y0 += 65535) {
        const unsigned ny = (unsigned)(n_blobs - y0 < 65535 ? n_blobs - y0 : 65535);
        hipLaunchKernelGGL(varint_tile_plan_kernel, dim3((unsigned)((plan.max_regions + kThreads - 1) / kThreads), ny),
                           dim3(kThreads), 0, s, w.blob_off, w.blob_region, w.region_base, w.sub_count, (uint32_t)y0,
                           n_blobs, ntiles, tile_plan);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const Mod64 M = make_mod64(modulus);
    const bool small_m = modulus <= ((int64_t)1 << 62);
    const char* env = getenv("SDA_DC_DEPTH");                  // A/B knob: blobs prefetched ahead
    const int depth = env ? atoi(env) : 4;
    const dim3 grid((unsigned)ntiles), block(kDcThreads);
    const uint64_t* tp = tile_plan;
    if (multi)
        hipLaunchKernelGGL((varint_decode_combine_kernel<2, true>), grid, block, 0, s, bytes, w.blob_off, n_blobs,
                           tp, ntiles, dim, out, M, small_m);
    else if (depth == 2)
        hipLaunchKernelGGL((varint_decode_combine_kernel<2, false>), grid, block, 0, s, bytes, w.blob_off, n_blobs,
                           tp, ntiles, dim, out, M, small_m);
    else if (depth == 8)
        hipLaunchKernelGGL((varint_decode_combine_kernel<8, false>), grid, block, 0, s, bytes, w.blob_off, n_blobs,
                           tp, ntiles, dim, out, M, small_m);
    else
        hipLaunchKernelGGL((varint_decode_combine_kernel<4, false>), grid, block, 0, s, bytes, w.blob_off, n_blobs,
                           tp, ntiles, dim, out, M, small_m);
    return hipGetLastError();
}

size_t varint_encode_work_bytes(uint64_t rows, uint64_t len) {
    const uint64_t chunks = (len + kEncChunk - 1) / kEncChunk;
    return 2 * rows * (chunks ? chunks : 1) * 8 + 2 * rows * 8 + 1024 + 256;
}

hipError_t launch_varint_encode(const int64_t* vals, uint64_t rows, uint64_t len, uint64_t stride, uint8_t* dst,
                                uint64_t dst_cap, void* work, uint64_t* row_bytes_host, hipStream_t s) {
    const uint64_t chunks = (len + kEncChunk - 1) / kEncChunk;
    if (rows == 0) return hipSuccess;
    uint64_t* chunk_bytes = static_cast<uint64_t*>(work);
    uint64_t* chunk_off = chunk_bytes + rows * (chunks ? chunks : 1);
    uint64_t* row_base = chunk_off + rows * (chunks ? chunks : 1);
    uint64_t* rbytes = row_base + rows;
    uint32_t* too_big = reinterpret_cast<uint32_t*>(rbytes + rows);
    hipError_t e;
    if (chunks == 0) {
        for (uint64_t r = 0; r < rows; ++r) row_bytes_host[r] = 0;
        return hipSuccess;
    }
    hipLaunchKernelGGL(varint_size_kernel, dim3((unsigned)chunks, (unsigned)rows), dim3(kThreads), 0, s, vals, len,
                       stride, (uint32_t)chunks, chunk_bytes);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // per row: its chunks' offsets and its total; then the rows back to back -- all on the device, so the
    // only host wait is the row sizes' copy at the end
    hipLaunchKernelGGL(varint_offsets_kernel, dim3((unsigned)rows), dim3(kThreads), 0, s, chunk_bytes,
                       (uint32_t)chunks, (const uint64_t*)nullptr, chunk_off, rbytes);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(varint_rows_kernel, dim3(1), dim3(kThreads), 0, s, (const uint64_t*)rbytes, rows, dst_cap,
                       row_base, too_big);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // nontemporal payload stores: encode -5.5 % in-process (3.770 -> 3.563 ms at 1000 x 1M, profiles/r06ad);
    // SDA_ENC_NT=0 (read per call) keeps cached stores for A/B
    const char* nt = getenv("SDA_ENC_NT");
    if (!(nt && nt[0] == '0'))
        hipLaunchKernelGGL(varint_write_kernel<true>, dim3((unsigned)chunks, (unsigned)rows), dim3(kThreads), 0, s,
                           vals, len, stride, (uint32_t)chunks, (const uint64_t*)chunk_off,
                           (const uint64_t*)row_base, (const uint32_t*)too_big, dst);
    else
        hipLaunchKernelGGL(varint_write_kernel<false>, dim3((unsigned)chunks, (unsigned)rows), dim3(kThreads), 0, s,
                           vals, len, stride, (uint32_t)chunks, (const uint64_t*)chunk_off,
                           (const uint64_t*)row_base, (const uint32_t*)too_big, dst);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(row_bytes_host, rbytes, rows * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    uint64_t acc = 0;
    for (uint64_t r = 0; r < rows; ++r) acc += row_bytes_host[r];
    return acc > dst_cap ? hipErrorInvalidValue : hipSuccess;     // nothing was written (too_big)
}

}  // namespace sda
