/*
 * sda_oracle.h -- CPU restatement of the SDA secret-sharing hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X engine (sda_amd/libsda_engine.so).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path never links it.
 *
 * Every function restates one piece of the reference (baajur/sda, Rust) with
 * the same operation order and Rust's integer semantics:
 *   - `%` is truncated remainder (sign of the dividend) -- identical to C99 `%`;
 *   - i64 `+`/`-`/`*` wrap on overflow (Rust release builds) -- done here on
 *     uint64_t and cast back, so no C undefined behaviour.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - combine / additive / masking / positive: fully specified by in-tree source
 *     (cited per function) and pinned by integration-tests/tests/full_loop.rs:148
 *     and README.md:157.
 *   - ChaCha20 block: pinned by RFC 7539 A.1 test vectors.
 *   - rand-0.3 ChaChaRng stream layout and gen_range zone rule, and the
 *     threshold-secret-sharing 0.2 FFT / Newton operation order: third-party
 *     crates absent from /root/reference; restated from their published
 *     algorithms.  Their canonical (mod p) results are pinned by the full_loop
 *     KATs; their exact signed representatives are "parity unpinned".
 */
#ifndef SDA_ORACLE_H
#define SDA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- element arithmetic (client/src/crypto/mod.rs:33-36: all i64) ---- */
int64_t or_rem(int64_t a, int64_t m);               /* Rust a % m            */
int64_t or_wadd(int64_t a, int64_t b);              /* Rust wrapping a + b   */

/* ---- combine: client/src/crypto/sharing/combiner.rs:16-28 ----
 * rows: n_rows pointers, lens[i] = length of row i.  Returns 0, or
 * 3 ("Wrong dimension") exactly where the reference would Err. */
int or_combine_rows(int64_t m, const int64_t* const* rows, const size_t* lens,
                    size_t n_rows, int64_t* out, size_t* out_len);
/* dense [n][dim] row-major form of the same loop */
void or_combine(int64_t m, const int64_t* shares, size_t n, size_t dim, int64_t* out);
int or_combine_mt(int64_t m, const int64_t* shares, size_t n, size_t dim, int64_t* out, int threads);

/* ---- additive: client/src/crypto/sharing/additive.rs:32-51 via batched.rs:19-53 ----
 * draws: [D][n-1] values that OsRng.gen_range(0, m) returned, in draw order.
 * out: [n][D] clerk-major (batched.rs:25-28, 46-48). */
void or_additive_generate(int64_t m, size_t n, const int64_t* secrets, size_t D,
                          const int64_t* draws, int64_t* out);

/* ---- packed Shamir: threshold-secret-sharing 0.2 (packed.rs, fft.rs, numtheory.rs) ---- */
typedef struct {
    size_t secret_count;       /* k */
    size_t share_count;        /* n */
    size_t privacy_threshold;  /* t */
    int64_t prime;             /* p */
    int64_t omega_secrets;     /* order k+t+1 (power of two) */
    int64_t omega_shares;      /* order n+1   (power of three) */
} or_packed_params;

int64_t or_mod_pow(int64_t x, uint32_t e, int64_t p);
int64_t or_mod_inverse(int64_t k, int64_t p);
/* one batch: k secrets + t randomness -> n shares (signed, tss op order) */
void or_packed_share(const or_packed_params* pp, const int64_t* secrets,
                     const int64_t* randomness, int64_t* shares);
/* batched.rs:19-53 over tss share: secrets[D] (tail zero-padded), rand [B][t], out [n][B] */
void or_packed_generate(const or_packed_params* pp, const int64_t* secrets, size_t D,
                        const int64_t* randomness, int64_t* out);
/* one batch: |I| shares at clerk indices -> k secrets (Newton, tss op order) */
void or_packed_reconstruct_batch(const or_packed_params* pp, const size_t* indices,
                                 size_t n_idx, const int64_t* shares, int64_t* secrets);
/* batched.rs:69-97: shares [n_idx][B] with B = ceil(dimension/k); out [dimension].
 * Returns 0, 5 ("Inputs must have same length") or 6 ("Not enough shares"). */
int or_packed_reconstruct(const or_packed_params* pp, size_t dimension,
                          const size_t* indices, size_t n_idx,
                          const int64_t* shares, int64_t* out);

/* ---- ChaCha20 / rand-0.3 ChaChaRng ---- */
/* core(): 20 rounds over a 16-word input state, then add the input (RFC 7539 2.3) */
void or_chacha20_core(const uint32_t in[16], uint32_t out[16]);
typedef struct {
    uint32_t state[16];
    uint32_t buffer[16];
    size_t index;
} or_chacha_rng;
void or_chacha_rng_from_seed(or_chacha_rng* r, const uint32_t* seed, size_t n_words);
uint32_t or_chacha_next_u32(or_chacha_rng* r);
uint64_t or_chacha_next_u64(or_chacha_rng* r);
int64_t or_chacha_gen_range(or_chacha_rng* r, int64_t low, int64_t high);

/* ---- masking: client/src/crypto/masking/{chacha,full}.rs ---- */
/* chacha.rs:25-53 with the OsRng seed replaced by `seed` */
void or_chacha_mask(int64_t m, const uint32_t* seed, size_t n_words,
                    const int64_t* secrets, size_t D, int64_t* masked);
/* chacha.rs:57-76: seeds [N][w] (i64 -> u32 as in :62-64) */
void or_chacha_mask_combine(int64_t m, size_t dimension, const int64_t* seeds,
                            size_t w, size_t N, int64_t* out);
/* chacha.rs:80-91 == full.rs:55-66: (ms - mask) % q */
void or_unmask(int64_t q, const int64_t* masks, const int64_t* masked, size_t D, int64_t* out);
/* full.rs:22-35 with OsRng draws supplied */
void or_full_mask(int64_t m, const int64_t* masks, const int64_t* secrets, size_t D, int64_t* out);
/* receive.rs:14-20 */
void or_positive(int64_t m, const int64_t* vals, size_t D, int64_t* out);

/* ---- share payload codec (sodium.rs:36-41, :78-90; integer-encoding 1.0 VarInt for i64) ---- */
size_t or_varint_encode(const int64_t* vals, size_t n, uint8_t* out);
size_t or_varint_decode(const uint8_t* in, size_t n_bytes, int64_t* out, size_t cap);

/* server/src/stores.rs:86-101 iter_snapshot_clerk_jobs_data: [participation][clerk] blobs regrouped
 * per clerk in snapshot order.  in blob (p, c) = in[part_off[p*n+c], part_off[p*n+c+1]); out gets
 * clerk 0's blobs back to back, then clerk 1's, ...; clerk_off [n][P+1] absolute offsets into out. */
void or_snapshot_transpose(const uint8_t* in, const uint64_t* part_off, size_t P, size_t n,
                           uint8_t* out, uint64_t* clerk_off);

#ifdef __cplusplus
}
#endif
#endif
