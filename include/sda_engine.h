/*
 * sda_engine.h -- C ABI of the MI355X (gfx950) SDA secret-sharing engine.
 *
 * This is the drop-in boundary for the reference client's sharing and masking
 * traits (baajur/sda, client/src/crypto/{sharing,masking}/mod.rs).  A Rust FFI
 * shim implements the six traits on top of these entry points
 * and is selected in the factories at client/src/crypto/sharing/mod.rs:35-96
 * and client/src/crypto/masking/mod.rs:33-94.
 *
 * Conventions
 *   - sda_share_combine, the Full sda_mask_combine, the Additive sda_secret_reconstruct and
 *     sda_clerk_decode_combine stream their inputs through pinned double buffers in row tiles of
 *     SDA_HOST_STAGE_MB (default 256) MiB, so a job larger than HBM runs (bit-identical to one pass).
 *     The other host entry points (packed and additive generate, packed reconstruct, ChaCha mask
 *     combine, sda_recipient_reveal) stage their whole job -- or, on a multi-device handle, each
 *     device's share of it -- in device memory, and return OUT_OF_MEMORY past it.
 *   - Elements are i64 (client/src/crypto/mod.rs:33-36); arithmetic follows
 *     Rust: truncated `%`, wrapping `+` (release builds).
 *   - The caller owns every buffer.  Host entry points are synchronous (they
 *     return when results are in host memory), like the Rust trait calls.
 *   - Entry points suffixed `_dev` take DEVICE pointers and a hipStream_t
 *     (passed as void*; NULL = the HIP null stream, the same convention as the
 *     ROCm math libraries); they only enqueue work, except for the few host
 *     values they return: the ChaCha combine waits for its rejection log (a few
 *     bytes) mid-call; the recipient and participant pipelines with ChaCha
 *     masking, and the varint encode (row sizes), wait for their stream at the
 *     end of the call instead, so no GPU idle gap opens inside them.
 *   - Randomness is explicit.  Where the reference draws from OsRng the caller
 *     passes the drawn values (or, for ChaCha masking, the seed words).
 *   - Every function returns an sda_status; 0 = OK.  The codes 1..6 map 1:1 to
 *     the reference's error strings; sda_last_error_message() gives details.
 *   - A handle may be used from one thread at a time (the Rust trait objects
 *     are not Sync either); distinct handles are independent.  The handle's
 *     scratch buffers are shared by its calls: a `_dev` call on a different
 *     stream than the handle's previous call first makes its stream wait (an
 *     event recorded when the previous call returned, no host sync) for the
 *     work queued by the previous one, so calls on one handle never race
 *     however the caller mixes streams.  The previous call's stream is not
 *     touched again: it may be destroyed once that call has returned.
 */
#ifndef SDA_ENGINE_H
#define SDA_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDA_ENGINE_ABI_VERSION 1

typedef enum {
    SDA_OK = 0,
    SDA_ERR_BATCH_INPUT_WRONG_LENGTH = 1,     /* "Batch input wrong length"          additive.rs:33      */
    SDA_ERR_PACKED_SHARING_FAILED = 2,        /* "Sharing failed for packed secret sharing scheme" packed_shamir.rs:41 */
    SDA_ERR_WRONG_DIMENSION = 3,              /* "Wrong dimension"                   combiner.rs:21      */
    SDA_ERR_MISMATCHING_DIMENSION = 4,        /* "Mismatching dimension"             additive.rs:64      */
    SDA_ERR_INPUTS_MUST_HAVE_SAME_LENGTH = 5, /* "Inputs must have same length"      packed_shamir.rs:74 */
    SDA_ERR_NOT_ENOUGH_SHARES = 6,            /* "Not enough shares to reconstruct"  packed_shamir.rs:75 */
    SDA_ERR_PRECONDITION = 64,   /* where the reference panics (assert!/assert_eq!, chacha.rs:26 ...)   */
    SDA_ERR_INVALID_ARGUMENT = 65, /* null handle/pointer, buffer too small                              */
    SDA_ERR_UNSUPPORTED = 66,    /* scheme parameters outside the engine's domain       */
    SDA_ERR_DEVICE = 67,         /* HIP runtime / kernel failure                                        */
    SDA_ERR_OUT_OF_MEMORY = 68
} sda_status;

/* protocol/src/crypto.rs:79-114  LinearSecretSharingScheme */
typedef enum { SDA_SHARING_ADDITIVE = 0, SDA_SHARING_PACKED_SHAMIR = 1 } sda_sharing_kind;
typedef struct {
    int32_t kind;                /* sda_sharing_kind                                  */
    uint64_t share_count;        /* Additive.share_count / PackedShamir.share_count   */
    int64_t modulus;             /* Additive.modulus     / PackedShamir.prime_modulus */
    uint64_t secret_count;       /* PackedShamir only                                 */
    uint64_t privacy_threshold;  /* PackedShamir only                                 */
    int64_t omega_secrets;       /* PackedShamir only                                 */
    int64_t omega_shares;        /* PackedShamir only                                 */
} sda_sharing_scheme;

/* protocol/src/crypto.rs:43-64  LinearMaskingScheme */
typedef enum { SDA_MASKING_NONE = 0, SDA_MASKING_FULL = 1, SDA_MASKING_CHACHA = 2 } sda_masking_kind;
typedef struct {
    int32_t kind;                /* sda_masking_kind                    */
    int64_t modulus;             /* Full.modulus / ChaCha.modulus       */
    uint64_t dimension;          /* ChaCha.dimension                    */
    uint64_t seed_bitsize;       /* ChaCha.seed_bitsize                 */
} sda_masking_scheme;

/* Packed-Shamir reveal representation. */
typedef enum {
    SDA_REVEAL_EXACT = 0,        /* bit-exact signed representatives of tss reconstruct (Newton) */
    SDA_REVEAL_CANONICAL = 1     /* canonical residues in [0,p) (Lagrange weights); equal mod p  */
} sda_reveal_mode;

typedef struct sda_engine sda_engine;

/* ---------------- lifecycle / diagnostics ---------------- */
int sda_abi_version(void);
sda_status sda_engine_create(int device_ordinal, sda_engine** out);
void sda_engine_destroy(sda_engine* h);
sda_status sda_engine_synchronize(sda_engine* h);
/* One handle over n_devices devices ("1-8 GPUs are used internally").  The host entry
 * points split their work over the devices and still return when the result is in host memory:
 *   sda_share_combine / Full sda_mask_combine / Additive sda_secret_reconstruct: by columns (each device
 *     walks every row in order over its slice: exact, signed inputs included, no exchange);
 *   ChaCha sda_mask_combine: by seeds, one RCCL ncclReduce(SUM, int64) onto ordinals[0] + the device
 *     finalize (RCCL is loaded on first use; moduli above 2^62, or repeated ordinals, run on ordinals[0]);
 *   sda_share_generate / PackedShamir sda_secret_reconstruct: by batches (Additive generate: by columns).
 * The `_dev` entry points run on ordinals[0].  Ordinals may repeat (several slices on one device: a
 * rehearsal of the split on fewer GPUs).  n_devices = 1 gives a one-device handle whose ChaCha mask
 * combine still reduces through a one-rank RCCL communicator. */
sda_status sda_engine_create_multi(const int* ordinals, int n_devices, sda_engine** out);
int sda_engine_device_count(const sda_engine* h);     /* devices the host entry points use; 0 for NULL */
const char* sda_last_error_message(void);          /* thread-local; never NULL */
const char* sda_status_string(int status);         /* reference error string for 1..6 */

/* ---------------- derived scheme sizes: protocol/src/crypto.rs:117-155 ---------------- */
uint64_t sda_scheme_input_size(const sda_sharing_scheme* s);              /* :120-126 */
uint64_t sda_scheme_output_size(const sda_sharing_scheme* s);             /* :129-135 */
uint64_t sda_scheme_privacy_threshold(const sda_sharing_scheme* s);       /* :138-144 */
uint64_t sda_scheme_reconstruction_threshold(const sda_sharing_scheme* s);/* :147-153 */
/* number of batches per clerk vector: ceil(dimension / input_size) (batched.rs:21-23) */
uint64_t sda_share_length(const sda_sharing_scheme* s, uint64_t dimension);

/* ---------------- trait mirrors (host buffers, synchronous) ---------------- */

/* ShareGenerator::generate  (sharing/mod.rs:14-17; batched.rs:19-53)
 *   secrets[dimension];  draws: the values OsRng produced, in draw order:
 *     Additive     [dimension][share_count-1]   gen_range(0, modulus)   additive.rs:42-44
 *     PackedShamir [B][privacy_threshold]       tss Range(0, p-1) sample
 *   out: [share_count][B] clerk-major, B = sda_share_length(s, dimension). */
sda_status sda_share_generate(sda_engine* h, const sda_sharing_scheme* s,
                              const int64_t* secrets, uint64_t dimension,
                              const int64_t* draws, uint64_t n_draws,
                              int64_t* out, uint64_t out_cap);

/* ShareCombiner::combine  (sharing/mod.rs:23-25; combiner.rs:16-28)
 *   rows[i] has lens[i] elements (a Vec<Vec<i64>>).  out_len = lens[0] (0 if n_rows == 0). */
sda_status sda_share_combine(sda_engine* h, const sda_sharing_scheme* s,
                             const int64_t* const* rows, const uint64_t* lens, uint64_t n_rows,
                             int64_t* out, uint64_t out_cap, uint64_t* out_len);

/* SecretReconstructor::reconstruct  (sharing/mod.rs:31-33; additive.rs:56-72; batched.rs:69-97)
 *   indexed shares = (indices[i], rows[i][lens[i]]);  dimension = factory argument (mod.rs:76). */
sda_status sda_secret_reconstruct(sda_engine* h, const sda_sharing_scheme* s, uint64_t dimension,
                                  const uint64_t* indices, const int64_t* const* rows,
                                  const uint64_t* lens, uint64_t n_rows,
                                  int64_t* out, uint64_t out_cap, uint64_t* out_len);

/* SecretMasker::mask  (masking/mod.rs:13-15)
 *   None:   mask_len = 0, masked = secrets                        (none.rs:14-19)
 *   Full:   full_masks[dimension] = the OsRng draws; mask = them  (full.rs:22-35)
 *   ChaCha: seed[seed_words] = the OsRng seed words; mask = seed as i64 (chacha.rs:25-53)
 *   mask_out needs room for dimension (Full) or seed_words (ChaCha) values. */
sda_status sda_secret_mask(sda_engine* h, const sda_masking_scheme* s,
                           const int64_t* secrets, uint64_t dimension,
                           const uint32_t* seed, uint64_t seed_words,
                           const int64_t* full_masks,
                           int64_t* mask_out, uint64_t mask_cap, uint64_t* mask_len,
                           int64_t* masked_out);

/* MaskCombiner::combine  (masking/mod.rs:21-23)
 *   Full: rows are masks (full.rs:38-50); ChaCha: rows are seeds-as-i64 (chacha.rs:57-76);
 *   None: every row must be empty, out_len = 0 (none.rs:22-25). */
sda_status sda_mask_combine(sda_engine* h, const sda_masking_scheme* s,
                            const int64_t* const* rows, const uint64_t* lens, uint64_t n_rows,
                            int64_t* out, uint64_t out_cap, uint64_t* out_len);

/* SecretUnmasker::unmask  (masking/mod.rs:29-31; chacha.rs:80-91; full.rs:55-66; none.rs:28-32)
 *   For ChaCha, `mask` is the COMBINED mask (the recipient's mask_combiner output). */
sda_status sda_secret_unmask(sda_engine* h, const sda_masking_scheme* s,
                             const int64_t* mask, uint64_t mask_len,
                             const int64_t* masked, uint64_t masked_len,
                             int64_t* out, uint64_t out_cap, uint64_t* out_len);

/* RecipientOutput::positive  (receive.rs:14-20) */
sda_status sda_recipient_positive(sda_engine* h, int64_t modulus, const int64_t* values,
                                  uint64_t n, int64_t* out);

/* ---------------- device-resident entry points (HBM-resident inputs) ---------------- */

/* Exact clerk combine of a dense [n][dim] matrix with row stride `row_stride` elements:
 * out[j] = combiner.rs:22-25 applied over rows 0..n-1 in order. */
sda_status sda_combine_dev(sda_engine* h, int64_t modulus, const int64_t* shares,
                           uint64_t n, uint64_t dim, uint64_t row_stride,
                           int64_t* out, void* stream);

/* The same recurrence continued from inout[dim] (a previous combine result, |r| < m, or zeros):
 * a clerk job streamed through HBM in row tiles is bit-identical to one pass over all rows. */
sda_status sda_combine_accumulate_dev(sda_engine* h, int64_t modulus, const int64_t* shares,
                                      uint64_t n, uint64_t dim, uint64_t row_stride,
                                      int64_t* inout, void* stream);

/* Multi-GPU finalize: `sums` are the int64 sums (RCCL-reduced; |sum| <= 2^63 - 1, signed allowed)
 * of per-GPU combine results; out = their canonical residue in [0, m).  Exact w.r.t. the reference
 * when all combined inputs were non-negative. */
sda_status sda_combine_finalize_dev(sda_engine* h, int64_t modulus, const int64_t* sums,
                                    uint64_t dim, int64_t* out, void* stream);

/* ---- participation split of the clerk combine over G ranks ----
 * The reference's result (combiner.rs:16-28) is order dependent when inputs are negative (Additive
 * last shares are signed, additive.rs:46), so rank g (rows of participations g's contiguous range):
 *  1. sda_combine_split_dev: the exact recurrence continued from inout (zeros before the first row
 *     tile), which also sets flags[0] = 1 if an input is < 0 and flags[1] = 1 if an input lies outside
 *     [-(2^63 - m), 2^63 - m] (the reference's `r + v` may wrap there: no split reproduces that, refuse
 *     the split).  flags: device int64[2], zeroed by the caller, only ever set to 1.
 *  2. no rank flagged a negative input: all-reduce(SUM) the G results, sda_combine_finalize_dev.
 *  3. otherwise: all-gather the G results into gathered[G][dim]; sda_combine_split_prefix_dev gives
 *     c_in (canonical sum of ranks < g), total (canonical sum of all) and the initial code;
 *     sda_combine_split_replay_dev replays this rank's row tiles from c_in (state in/out) recording the
 *     last sign event in code (0 none, 2g+1 reset, 2g+2 set); all-reduce(MAX) the codes over the ranks;
 *     sda_combine_split_resolve_dev writes the reference's signed result. */
sda_status sda_combine_split_dev(sda_engine* h, int64_t modulus, const int64_t* shares, uint64_t n,
                                 uint64_t dim, uint64_t row_stride, int64_t* inout, int64_t* flags,
                                 void* stream);
sda_status sda_combine_split_prefix_dev(sda_engine* h, int64_t modulus, const int64_t* gathered,
                                        uint64_t world, uint64_t rank, uint64_t dim, int64_t* c_in,
                                        int64_t* total, int32_t* code, void* stream);
sda_status sda_combine_split_replay_dev(sda_engine* h, int64_t modulus, const int64_t* shares, uint64_t n,
                                        uint64_t dim, uint64_t row_stride, uint64_t rank, int64_t* state,
                                        int32_t* code, void* stream);
sda_status sda_combine_split_resolve_dev(sda_engine* h, int64_t modulus, const int64_t* total,
                                         const int32_t* code, uint64_t dim, int64_t* out, void* stream);

/* Packed-Shamir share generation for `n_vectors` participant vectors at once:
 * secrets [n_vectors][dimension], draws [n_vectors][B][t], out [n_vectors][n][B]. */
sda_status sda_packed_generate_dev(sda_engine* h, const sda_sharing_scheme* s,
                                   const int64_t* secrets, uint64_t dimension, uint64_t n_vectors,
                                   const int64_t* draws, int64_t* out, void* stream);

/* The same with a representation mode: SDA_REVEAL_EXACT = tss' signed shares (as above),
 * SDA_REVEAL_CANONICAL = their canonical residues in [0, p).  Canonical shares are equal to the
 * reference's mod p, so combine -> reveal -> unmask -> positive() ends in the identical output
 * when the masking modulus is the sharing prime. */
sda_status sda_packed_generate_mode_dev(sda_engine* h, const sda_sharing_scheme* s,
                                        const int64_t* secrets, uint64_t dimension, uint64_t n_vectors,
                                        const int64_t* draws, int64_t* out, int32_t mode, void* stream);

/* Packed-Shamir reveal: shares [n_vectors][n_idx][B] at clerk `indices` (host array),
 * out [n_vectors][dimension].  All n_idx shares are used (batched.rs:75); n_idx <= 1023. */
sda_status sda_packed_reconstruct_dev(sda_engine* h, const sda_sharing_scheme* s, uint64_t dimension,
                                      const uint64_t* indices, uint64_t n_idx, uint64_t n_vectors,
                                      const int64_t* shares, int64_t* out, int32_t mode, void* stream);

/* Additive share generation: secrets [dimension], draws [dimension][n-1], out [n][dimension]. */
sda_status sda_additive_generate_dev(sda_engine* h, int64_t modulus, uint64_t share_count,
                                     const int64_t* secrets, uint64_t dimension,
                                     const int64_t* draws, int64_t* out, void* stream);

/* ChaCha mask expansion + combine (chacha.rs:57-76) over n_seeds seeds of w words
 * (seeds [n_seeds][w] u32, device), out [dimension].  Exact including gen_range rejections
 * (fix-up pass; moduli with a high rejection rate expand each stream exactly instead) and the
 * reference's wrapping i64 sum for moduli above 2^62 (the result is then signed and
 * order-dependent, as in the reference).  Waits for its rejection log before returning. */
sda_status sda_chacha_mask_combine_dev(sda_engine* h, int64_t modulus, uint64_t dimension,
                                       const uint32_t* seeds, uint64_t w, uint64_t n_seeds,
                                       int64_t* out, void* stream);

/* ---------------- share payload codec ----------------
 * Encryptor::encrypt encodes shares with integer-encoding 1.0 VarInt before sealing
 * (client/src/crypto/encryption/sodium.rs:36-41); Decryptor::decrypt decodes after opening
 * (:82-88): zigzag + LEB128, a run of >= 11 continuation bytes forms one 11-byte element and a
 * truncated final varint yields its partial value.  The sealed box itself stays on the host. */

/* Encryptor::encrypt's encoding step: out[*out_len] bytes (at most 10 per value). */
sda_status sda_varint_encode(sda_engine* h, const int64_t* vals, uint64_t n,
                             uint8_t* out, uint64_t out_cap, uint64_t* out_len);
/* Decryptor::decrypt's decoding step for one opened blob. */
sda_status sda_varint_decode(sda_engine* h, const uint8_t* bytes, uint64_t n_bytes,
                             int64_t* out, uint64_t out_cap, uint64_t* out_len);
/* Clerk job after the sealed-box opens (clerk.rs:79-86): decode every participation's blob,
 * then ShareCombiner::combine -- "Wrong dimension" if a blob decodes to a different length. */
sda_status sda_clerk_decode_combine(sda_engine* h, const sda_sharing_scheme* s,
                                    const uint8_t* const* blobs, const uint64_t* blob_lens,
                                    uint64_t n_blobs, int64_t* out, uint64_t out_cap,
                                    uint64_t* out_len);
/* Device forms.  `bytes`: device, 16-byte aligned, readable up to blob_off[n_blobs] rounded up to
 * 16 plus 16 bytes; blob i = bytes[blob_off[i], blob_off[i+1]) with blob_off a HOST array.
 * decode: out [n_blobs][out_stride] (device), counts[n_blobs] (host) = values per blob. */
sda_status sda_varint_decode_dev(sda_engine* h, const uint8_t* bytes, const uint64_t* blob_off,
                                 uint64_t n_blobs, int64_t* out, uint64_t out_stride,
                                 uint64_t* counts, void* stream);
/* decode + exact combine (combiner.rs:16-28); out (device) gets *out_len values. */
sda_status sda_clerk_decode_combine_dev(sda_engine* h, int64_t modulus, const uint8_t* bytes,
                                        const uint64_t* blob_off, uint64_t n_blobs,
                                        int64_t* out, uint64_t out_cap, uint64_t* out_len,
                                        void* stream);
/* encode rows [rows][stride] (first len values of each) back to back into dst (device);
 * row_bytes[rows] (host) = bytes per row. */
sda_status sda_varint_encode_dev(sda_engine* h, const int64_t* vals, uint64_t rows, uint64_t len,
                                 uint64_t stride, uint8_t* dst, uint64_t dst_cap,
                                 uint64_t* row_bytes, void* stream);

/* ---------------- snapshot transposition ----------------
 * Replaces AggregationsStore::iter_snapshot_clerk_jobs_data (server/src/stores.rs:86-101; the Mongo
 * store's $unwind/$group at server-store-mongodb/src/aggregations.rs:164-195): the snapshot's
 * participations [participation][clerk] regrouped as clerking jobs [clerk][participation], each
 * clerk's blobs in snapshot order.  Blobs are opaque bytes (sealed boxes or opened payloads).
 *   src (device, 16-byte aligned, readable 32 bytes past part_off[P*n]): participation p's payload
 *     for clerk c = src[part_off[p*n + c], part_off[p*n + c + 1]); part_off is a HOST array [P*n + 1].
 *   dst (device, 16-byte aligned): clerk c's job starts at dst + clerk_base[c] (16-byte aligned) and
 *     its blob p = [clerk_off[c*(P+1) + p], clerk_off[c*(P+1) + p + 1]) relative to that start, followed
 *     by >= 16 readable bytes -- exactly the (bytes, blob_off) pair sda_clerk_decode_combine_dev takes.
 *   clerk_base [n], clerk_off [n][P+1] (HOST, written); *dst_len = bytes of dst used.
 *   dst == NULL: sizing query (offsets and *dst_len only, nothing launched).
 *   Runs on `stream` and returns once the copy has completed (the copy plan is uploaded per call). */
sda_status sda_snapshot_transpose_dev(sda_engine* h, const uint8_t* src, const uint64_t* part_off,
                                      uint64_t n_participations, uint64_t n_clerks, uint8_t* dst,
                                      uint64_t dst_cap, uint64_t* dst_len, uint64_t* clerk_base,
                                      uint64_t* clerk_off, void* stream);

/* ---------------- fused role pipelines ---------------- */

/* Recipient reveal (receive.rs:80-157) + RecipientOutput::positive (:14-20) as one device
 * pipeline: mask combine -> reconstruct -> fused unmask+positive, no host round trip between.
 *   mask_in: Full = masks [n_masks][mask_width] i64; ChaCha = seeds [n_masks][mask_width] u32
 *            (1..8 words); None = n_masks rows of width 0.
 *   shares [n_idx][share_len] at clerk `indices` (host array); dimension = the reconstructor's
 *   factory argument (vector_dimension); output_modulus = aggregation.modulus for positive().
 *   Errors as the reference: Not enough shares (6), Mismatching dimension (4), assert -> 64.
 *   With ChaCha masking the call drains its stream before returning: the mask's gen_range rejection
 *   count is read then (the rare rejected draws are fixed and the unmask redone). */
sda_status sda_recipient_reveal_dev(sda_engine* h, const sda_masking_scheme* ms, const void* mask_in,
                                    uint64_t n_masks, uint64_t mask_width, const sda_sharing_scheme* ss,
                                    uint64_t dimension, const uint64_t* indices, const int64_t* shares,
                                    uint64_t n_idx, uint64_t share_len, int64_t output_modulus,
                                    int32_t mode, int64_t* out, uint64_t out_cap, uint64_t* out_len,
                                    void* stream);
/* Host form: mask rows as MaskCombiner::combine takes them (Full masks / ChaCha seeds-as-i64),
 * share rows as SecretReconstructor::reconstruct takes them.  On a multi-device handle the ChaCha mask
 * combine is split over the devices (as sda_mask_combine), the rest runs on ordinals[0]. */
sda_status sda_recipient_reveal(sda_engine* h, const sda_masking_scheme* ms,
                                const int64_t* const* mask_rows, const uint64_t* mask_lens, uint64_t n_masks,
                                const sda_sharing_scheme* ss, uint64_t dimension, const uint64_t* indices,
                                const int64_t* const* share_rows, const uint64_t* share_lens, uint64_t n_idx,
                                int64_t output_modulus, int32_t mode,
                                int64_t* out, uint64_t out_cap, uint64_t* out_len);

/* Participant (participate.rs:53-76): SecretMasker::mask -> ShareGenerator::generate -> per-clerk
 * payload encoding (sodium.rs:36-41) on device.  seed: host words (ChaCha); full_masks: device [D]
 * (Full); secrets [D], draws (as sda_share_generate) and shares_out [n][B] are device buffers.
 * mode: packed shares as tss' signed values (SDA_REVEAL_EXACT) or canonical residues
 * (SDA_REVEAL_CANONICAL, see sda_packed_generate_mode_dev); ignored for Additive.
 * payload (device, may be NULL): the n clerk payloads back to back, payload_row_bytes[n] (host).
 * With ChaCha masking, or with payloads, the call drains its stream before returning (the mask's
 * rejection count; the payload sizes). */
sda_status sda_participant_share_dev(sda_engine* h, const sda_masking_scheme* ms, const uint32_t* seed,
                                     uint64_t seed_words, const int64_t* full_masks,
                                     const sda_sharing_scheme* ss, const int64_t* secrets, uint64_t dimension,
                                     const int64_t* draws, int32_t mode, int64_t* shares_out, uint8_t* payload,
                                     uint64_t payload_cap, uint64_t* payload_row_bytes, void* stream);

/* Synthetic benchmark input: dst[r*cols + c] = lo + splitmix64(seed, r, c) % (hi - lo). */
sda_status sda_synth_fill_dev(sda_engine* h, int64_t* dst, uint64_t rows, uint64_t cols,
                              uint64_t seed, int64_t lo, int64_t hi, void* stream);

/* HBM for the resident hot-path buffers (no reference counterpart: the reference's buffers are Rust
 * Vec<i64> on the host, batched.rs:25-28).  `bytes` of device memory on `device`, one virtual range
 * mapped from physical chunks of SDA_HBM_CHUNK_MB (default 64) MiB, so its backing never depends on how
 * fragmented the driver's free VRAM is.  The request is rounded up to whole chunks, and
 * belongs to a size class (n chunks: n up to 4, then 4..7 x 2^e, at most 25 % more): the buffer reserves
 * its class's virtual range and maps the chunks asked for.
 * sda_hbm_free does not wait: the buffer returns to a per-process pool, still mapped, and a later
 * sda_hbm_alloc of the same size class gets it back (after a device-wide sync if none has completed since
 * the free; extra chunks, if it needs more, are mapped at the range's never-mapped tail).  The pool holds
 * at most SDA_HBM_POOL_MB (default 32768) MiB per device: an allocation that finds no pooled buffer of its
 * class trims the oldest pooled buffers down to that bound, and trims the whole pool and retries once when
 * the device is out of memory.  Trimming syncs the device and releases the physical chunks; the virtual
 * range stays reserved and is never mapped again (DESIGN.md §2 gives the cause).  NULL is a no-op; a
 * pointer not returned by sda_hbm_alloc, or freed twice, is INVALID_ARGUMENT.  Thread-safe; no lock is
 * held across a device sync. */
sda_status sda_hbm_alloc(int device, uint64_t bytes, void** out);
sda_status sda_hbm_free(void* ptr);
/* Release pooled buffers of `device` (oldest first) until at most keep_bytes stay pooled.
 * Destroying the last live engine handle of a device trims that device's pool to 0. */
sda_status sda_hbm_trim(int device, uint64_t keep_bytes);
/* Bytes of `device` handed out and pooled (mapped chunks), and retired (virtual ranges kept reserved
 * after a trim; a steady stream of jobs whose buffers fit the pool retires none); any pointer may be
 * NULL. */
sda_status sda_hbm_stats(int device, uint64_t* live_bytes, uint64_t* pooled_bytes, uint64_t* retired_bytes);

#ifdef __cplusplus
}
#endif
#endif /* SDA_ENGINE_H */
