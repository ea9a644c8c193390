// kernels.h -- internal launchers (not part of the C ABI).  Each returns hipSuccess or the
// launch error; all of them only enqueue on `stream`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "modarith.h"

namespace sda {

// ---- combine.hip ----
// Exact clerk combine: out[j] = fold over rows of (r + v) % m  (combiner.rs:22-25).
// accumulate: continue from the values in `out` (a previous result, |r| < m) instead of 0.
hipError_t launch_combine_exact(const int64_t* in, uint64_t n, uint64_t dim, uint64_t stride,
                                int64_t* out, int64_t modulus, hipStream_t s, bool accumulate = false);
// The same recurrence over int32 rows (decoded field shares: the clerk's decode -> combine).
hipError_t launch_combine_exact32(const int32_t* in, uint64_t n, uint64_t dim, uint64_t stride,
                                  int64_t* out, int64_t modulus, hipStream_t s);
// Canonical residue of the int64 sums of the ranks' results (multi-GPU finalize; signed sums allowed).
hipError_t launch_mod_canonical(const int64_t* sums, uint64_t dim, int64_t* out, int64_t modulus,
                                hipStream_t s);
// Participation split.  Pass 1: the exact recurrence continued from inout that also sets
// flags[0] = 1 (an input < 0) / flags[1] = 1 (an input outside [-(2^63 - m), 2^63 - m]).
hipError_t launch_combine_split(const int64_t* in, uint64_t n, uint64_t dim, uint64_t stride, int64_t* inout,
                                int64_t modulus, int64_t* flags, hipStream_t s);
// Pass 2 (signed inputs): replay the canonical trajectory from state (c_in), recording the last sign
// event in code (reset_code = 2 rank + 1 on a reset, + 1 on a set; unchanged without an event).
hipError_t launch_combine_replay(const int64_t* in, uint64_t n, uint64_t dim, uint64_t stride, int64_t* state,
                                 int32_t* code, int32_t reset_code, int64_t modulus, hipStream_t s);
hipError_t launch_split_prefix(const int64_t* gathered, uint64_t world, uint64_t rank, uint64_t dim, int64_t* c_in,
                               int64_t* total, int32_t* code, int64_t modulus, hipStream_t s);
hipError_t launch_split_resolve(const int64_t* total, const int32_t* code, uint64_t dim, int64_t* out,
                                int64_t modulus, hipStream_t s);

// ---- elementwise.hip ----
hipError_t launch_additive_generate(const int64_t* secrets, uint64_t D, const int64_t* draws,
                                    uint64_t n, int64_t* out, int64_t modulus, hipStream_t s);
// out[i] = (a[i] + sign * b[i]) % m   (sign = +1: mask, -1: unmask)
hipError_t launch_addsub_trem(const int64_t* a, const int64_t* b, int sign, uint64_t D,
                              int64_t* out, int64_t modulus, hipStream_t s);
hipError_t launch_positive(const int64_t* v, uint64_t D, int64_t* out, int64_t modulus,
                           hipStream_t s);
// out = positive((ms - mask) % q, pos_m); mask == nullptr: no unmask; pos_m == 0: no positive()
hipError_t launch_unmask_positive(const int64_t* ms, const int64_t* mask, uint64_t D, int64_t q, int64_t pos_m,
                                  int64_t* out, hipStream_t s);
hipError_t launch_synth_fill(int64_t* dst, uint64_t rows, uint64_t cols, uint64_t seed,
                             int64_t lo, int64_t hi, hipStream_t s);

// ---- packed_gen.hip / packed_reveal.hip ----
// Engine-owned device copy of a precomputed, data-independent table (twiddles, Newton inverses,
// Lagrange weights).  Rebuilt and uploaded only when its key (the parameters it depends on) changes.
struct DeviceTable {
    std::vector<uint8_t> key;
    void* dev = nullptr;
    size_t cap = 0;
    void* ws = nullptr;           // packed_wide.hip: per-lane transform workspace (grows, never shrinks)
    size_t ws_cap = 0;
    uint32_t flags = 0;           // per-table launch choices (packed_gen.hip: bit 0 = sign-bit kernel)
};
hipError_t ensure_table(DeviceTable& t, const std::vector<uint8_t>& key, const void* host, size_t bytes);
void free_table(DeviceTable& t);

struct PackedGenArgs {
    const int64_t* secrets; uint64_t dimension; uint64_t n_vectors;
    const int64_t* draws; int64_t* out;
    bool canonical = false;       // shares as canonical residues in [0, p) instead of tss' signed values
    uint32_t prime = 0;           // set by launch_packed_generate (selects the lazy-truncation kernel)
    bool signbit = false;         // set by launch_packed_generate (sign-bit radix-2 half, packed_gen.hip)
    bool xcd_order = true;        // set by launch_packed_generate: XCD-chunked tile order (xcd.h)
};
// A/B knob: SDA_XCD_ORDER=0 runs the streaming kernels in natural workgroup order (xcd.h).
bool xcd_order_enabled();
// Exact share-gen uses lazy truncation (packed_gen.hip: Trunc<true>) for primes at least this big.
constexpr uint32_t kLazyTruncMinP = 1u << 24;
// Batches whose inputs fall outside (-p, p) are logged by the fast kernel and recomputed by a
// generic exact fix-up kernel.  `log_buf` is device memory of packed_gen_log_bytes() bytes.
constexpr uint32_t kGenLogCap = 1u << 16;
struct GenFixupLog {
    unsigned int* count;
    uint64_t* list;        // vec * B + batch
    uint32_t cap;
};
size_t packed_gen_log_bytes();
hipError_t launch_packed_generate(const PackedGenArgs& a, uint32_t k, uint32_t t, uint32_t n, uint32_t p,
                                  uint32_t omega_secrets, uint32_t omega_shares, DeviceTable& tab, void* log_buf,
                                  hipStream_t s);
struct PackedRevealArgs {
    const int64_t* shares; uint64_t dimension; uint64_t n_vectors; int64_t* out;
};
// The register reveal kernels take up to kRevealMaxPoints - 1 clerk shares per batch (n + 1 <= 81
// gives n <= 80 clerks; they keep n_idx + 1 Newton points in registers).
constexpr int kRevealMaxPoints = 96;
// Past these sizes (k + t + 1 > 64, n + 1 > 81, more than kRevealMaxPoints - 1 shares) the packed
// calls take packed_wide.hip's workspace kernels, up to the engine's domain limits below.
constexpr uint32_t kWideMaxL = 1024;       // k + t + 1
constexpr uint32_t kWideMaxN3 = 729;       // n + 1
constexpr uint32_t kRevealMaxShares = 1023;
hipError_t launch_packed_generate_wide(const PackedGenArgs& a, uint32_t k, uint32_t t, uint32_t n, uint32_t p,
                                       uint32_t omega_secrets, uint32_t omega_shares, DeviceTable& tab,
                                       hipStream_t s);
// returns hipErrorInvalidValue for CANONICAL mode with duplicate clerk points.  `log_buf`: device
// memory of packed_gen_log_bytes() bytes (batches the exact kernel hands to its generic fix-up).
hipError_t launch_packed_reveal(const PackedRevealArgs& a, const uint64_t* indices, uint32_t n_idx, uint32_t k,
                                uint32_t p, uint32_t omega_secrets, uint32_t omega_shares, int mode,
                                DeviceTable& tab, void* log_buf, hipStream_t s);
hipError_t launch_packed_reveal_wide(const PackedRevealArgs& a, const uint64_t* indices, uint32_t n_idx, uint32_t k,
                                     uint32_t p, uint32_t omega_secrets, uint32_t omega_shares, int mode,
                                     DeviceTable& tab, hipStream_t s);

// ---- codec.hip (share payload codec: sodium.rs:36-41 / :82-88, integer-encoding 1.0 VarInt) ----
// Host-side plan of the decode: blobs are split into 4 KiB regions aligned to the (16-byte
// aligned) byte buffer; a region shared by two blobs appears once per blob.
struct VarintPlan {
    std::vector<uint64_t> blob_region;   // [n_blobs + 1] first region of each blob (prefix sum)
    uint64_t regions = 0;
    uint64_t max_regions = 0;            // regions of the largest blob (grid.x)
};
void varint_plan(const uint64_t* blob_off, uint64_t n_blobs, VarintPlan* plan);
size_t varint_decode_work_bytes(size_t regions, uint64_t n_blobs);
// element count of every blob (synchronous: copies n_blobs counts to the host); long_any: some element
// has >= 6 bytes (sub_counts: also the 256-byte sub-chunk counts of the fused decode -> combine)
hipError_t launch_varint_count(const uint8_t* bytes, const uint64_t* blob_off_host, uint64_t n_blobs,
                               const VarintPlan& plan, void* work, uint64_t* counts_host, bool* irregular_any,
                               hipStream_t s, bool sub_counts = false, bool* long_any = nullptr);
// decode every blob into out + blob * out_stride (after launch_varint_count on the same work)
hipError_t launch_varint_decode(const uint8_t* bytes, uint64_t n_blobs, const VarintPlan& plan, void* work,
                                int64_t* out, uint64_t out_stride, uint64_t len, bool irregular_any,
                                hipStream_t s);
// the same decode into int32 (regular blobs only: the caller checked irregular_any == false); *wide_host
// (synchronous) tells whether some value did not fit, in which case out holds garbage
// sda_varint_decode_dev in one pass of launches: count, scan, a device capacity check (some blob
// decodes to more than out_stride values: nothing is written, *too_long), decode; counts_host[n_blobs]
// and the flag are read at the end of the call (its only wait).
hipError_t launch_varint_decode_one_wait(const uint8_t* bytes, const uint64_t* blob_off_host, uint64_t n_blobs,
                                        const VarintPlan& plan, void* work, int64_t* out, uint64_t out_stride,
                                        uint64_t* counts_host, bool* too_long, hipStream_t s);
hipError_t launch_varint_decode_narrow(const uint8_t* bytes, uint64_t n_blobs, const VarintPlan& plan, void* work,
                                       int32_t* out, uint64_t out_stride, bool* wide_host, hipStream_t s);
// The clerk's fused decode -> combine (after launch_varint_count with sub_counts on the same work; regular
// blobs of equal element count dim): out[dim] = combiner.rs:16-28 over the decoded blobs in order, each
// payload read once.  tile_plan: device scratch of varint_tile_plan_bytes(n_blobs, dim).
uint64_t varint_tile_plan_bytes(uint64_t n_blobs, uint64_t dim);
uint64_t varint_fused_tiles(uint64_t dim);
hipError_t launch_varint_decode_combine(const uint8_t* bytes, uint64_t n_blobs, const VarintPlan& plan, void* work,
                                        uint64_t* tile_plan, uint64_t dim, int64_t* out, int64_t modulus,
                                        bool multi, hipStream_t s);
// The clerk's decode -> combine over region slots (no count pass), in one pass of launches: the payload is
// decoded once into int32 slots per 16 KiB region (slot buffer: varint_slot_bytes), region counts are
// scanned, and combiner.rs:16-28 runs over the slots into out -- unless *flags_host comes back nonzero
// (bit 0: an element longer than 5 bytes or not a field share: use the matrix path; bit 1: the blobs
// decode to different lengths), or blob 0's count exceeds out_cap, or modulus (|m|) is 0: then out is
// untouched.  counts_host[n_blobs] and *flags_host are read at the end of the call (its only wait).
size_t varint_slot_bytes(const VarintPlan& plan, uint64_t n_blobs, uint64_t dim);
hipError_t launch_varint_decode_slots_combine(const uint8_t* bytes, const uint64_t* blob_off_host, uint64_t n_blobs,
                                              const VarintPlan& plan, void* work, void* slot_buf, int64_t* out,
                                              uint64_t out_cap, int64_t modulus, uint64_t* counts_host,
                                              uint32_t* flags_host, hipStream_t s);
size_t varint_encode_work_bytes(uint64_t rows, uint64_t len);
// encode rows [rows][stride] (first len elements) back to back into dst; row_bytes_host gets each
// row's byte count (synchronous).  hipErrorInvalidValue if dst_cap is too small.
hipError_t launch_varint_encode(const int64_t* vals, uint64_t rows, uint64_t len, uint64_t stride, uint8_t* dst,
                                uint64_t dst_cap, void* work, uint64_t* row_bytes_host, hipStream_t s);

// ---- chacha.hip ----
// Combine of n_seeds ChaCha mask streams (chacha.rs:57-76), two implementations:
//  * fast path: counter mode, canonical sums, rejections logged and fixed up.  `work` must hold
//    chacha_work_bytes(D, n_seeds).  Valid when !chacha_needs_stream_path(m); sets *overflow (and writes
//    nothing) when more rejections occur than its log holds -- rerun on the stream path.
//  * stream path: the draws of a tile of streams expanded exactly (any rejection rate) into rows,
//    then the exact sequential combine recurrence (wrapping i64 add for m > 2^62, as the reference).
//    `work` must hold chacha_stream_work_bytes(D, n_seeds, m).  Host-synchronous per tile.
size_t chacha_work_bytes(uint64_t dimension, uint64_t n_seeds);
bool chacha_needs_stream_path(int64_t modulus);
size_t chacha_stream_work_bytes(uint64_t dimension, uint64_t n_seeds, int64_t modulus);
hipError_t launch_chacha_mask_combine(int64_t modulus, uint64_t dimension, const uint32_t* seeds,
                                      uint32_t w, uint64_t n_seeds, int64_t* out, void* work,
                                      hipStream_t s, bool* overflow, int* fixups_out);
// The same fast path in two halves, for pipelines that keep queueing work behind it: _async enqueues
// the combine (canonical draws' sums in out, before any fix-up) and copies its rejection count to
// count_host (PINNED host memory, valid once the stream has drained); resolve_ then applies the
// fix-ups for that count (host-synchronous, rare) or sets *overflow (rerun on the stream path).  The
// caller redoes whatever it queued on `out` when the count was nonzero.
hipError_t launch_chacha_mask_combine_async(int64_t modulus, uint64_t dimension, const uint32_t* seeds, uint32_t w,
                                            uint64_t n_seeds, int64_t* out, void* work, hipStream_t s,
                                            unsigned long long* count_host);
// One stream's masked secrets in one pass (chacha.rs:36-45): masked = (secrets + draw) % m, the rejection
// count to count_host (pinned).  A nonzero count means `masked` used rejected draws: the caller redoes
// the mask exactly (launch_chacha_mask_combine, then the add).
hipError_t launch_chacha_mask_add_async(int64_t modulus, uint64_t dimension, const uint32_t* seed, uint32_t w,
                                        const int64_t* secrets, int64_t* masked, void* work, hipStream_t s,
                                        unsigned long long* count_host);
hipError_t resolve_chacha_mask_combine(int64_t modulus, uint64_t dimension, const uint32_t* seeds, uint32_t w,
                                       uint64_t n_seeds, int64_t* out, void* work, hipStream_t s,
                                       unsigned long long n_rej, bool* overflow, int* fixups_out);
hipError_t launch_chacha_streams_combine(int64_t modulus, uint64_t dimension, const uint32_t* seeds, uint32_t w,
                                         uint64_t n_seeds, int64_t* out, void* work, hipStream_t s);
// mask[i] = gen_range draw i of one stream (chacha.rs:36-39); `work`: chacha_stream_work_bytes(D, 1, m)
hipError_t launch_chacha_stream(int64_t modulus, uint64_t dimension, const uint32_t* seed, uint32_t w,
                                int64_t* mask, void* work, hipStream_t s);

// ---- snapshot.hip ----
// One blob of the snapshot transposition: len bytes from src offset to dst offset.
struct SnapshotCopy {
    uint64_t src, dst, len;
};
uint64_t snapshot_chunk_bytes();
// blobs[n_blobs] (each len >= 1), chunk_start[n_blobs + 1] = exclusive prefix of ceil(len / chunk);
// src/dst 16-byte aligned, src readable 32 bytes past the last blob's end.
hipError_t launch_snapshot_transpose(const uint8_t* src, uint8_t* dst, const SnapshotCopy* blobs,
                                     const uint64_t* chunk_start, uint64_t n_blobs, uint64_t total_chunks,
                                     hipStream_t s);

}  // namespace sda
