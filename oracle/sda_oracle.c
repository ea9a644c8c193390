/*
 * sda_oracle.c -- CPU restatement of the SDA secret-sharing hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline "port").  See
 * sda_oracle.h for the pinning status of each part.  Paths below are relative
 * to the reference tree (baajur/sda).
 */
#include "sda_oracle.h"

#include <stdlib.h>
#include <pthread.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* element arithmetic                                                        */
/* ------------------------------------------------------------------------ */

int64_t or_rem(int64_t a, int64_t m) {
    /* Rust `%` on i64 == C99 `%` (truncated).  i64::MIN % -1 would panic in
     * Rust; not reachable with the positive moduli used by the schemes. */
    return a % m;
}

int64_t or_wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static int64_t or_wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static int64_t or_wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

/* ------------------------------------------------------------------------ */
/* combine -- client/src/crypto/sharing/combiner.rs:16-28                   */
/* ------------------------------------------------------------------------ */

int or_combine_rows(int64_t m, const int64_t* const* rows, const size_t* lens,
                    size_t n_rows, int64_t* out, size_t* out_len) {
    /* combiner.rs:17  dimension = shares.get(0).map_or(0, Vec::len) */
    size_t dim = n_rows ? lens[0] : 0;
    *out_len = dim;
    /* combiner.rs:19  result = vec![0; dimension] */
    for (size_t j = 0; j < dim; ++j) out[j] = 0;
    for (size_t i = 0; i < n_rows; ++i) {
        /* combiner.rs:21  if share.len() != dimension { Err("Wrong dimension")? } */
        if (lens[i] != dim) return 3;
        const int64_t* row = rows[i];
        /* combiner.rs:22-25  result[ix] += *value; result[ix] %= self.modulus; */
        for (size_t j = 0; j < dim; ++j) out[j] = or_rem(or_wadd(out[j], row[j]), m);
    }
    return 0;
}

void or_combine(int64_t m, const int64_t* shares, size_t n, size_t dim, int64_t* out) {
    for (size_t j = 0; j < dim; ++j) out[j] = 0;
    for (size_t i = 0; i < n; ++i) {
        const int64_t* row = shares + i * dim;
        for (size_t j = 0; j < dim; ++j) out[j] = or_rem(or_wadd(out[j], row[j]), m);
    }
}

/* The same loop split over `threads` POSIX threads by column range (the CPU baseline's all-cores
 * mode): columns are independent, so every thread runs combiner.rs:22-25
 * over all rows, in order, for its own columns -- the result is identical to or_combine. */
typedef struct {
    int64_t m;
    const int64_t* shares;
    size_t n, dim, c0, c1;
    int64_t* out;
} or_combine_part;

static void* or_combine_worker(void* arg) {
    const or_combine_part* a = (const or_combine_part*)arg;
    for (size_t j = a->c0; j < a->c1; ++j) a->out[j] = 0;
    for (size_t i = 0; i < a->n; ++i) {
        const int64_t* row = a->shares + i * a->dim;
        for (size_t j = a->c0; j < a->c1; ++j) a->out[j] = or_rem(or_wadd(a->out[j], row[j]), a->m);
    }
    return NULL;
}

int or_combine_mt(int64_t m, const int64_t* shares, size_t n, size_t dim, int64_t* out, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    or_combine_part part[256];
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        /* 64-column aligned ranges: no two threads write one cache line of `out` */
        const size_t blocks = (dim + 63) / 64;
        const size_t b0 = blocks * (size_t)t / (size_t)threads, b1 = blocks * (size_t)(t + 1) / (size_t)threads;
        part[t] = (or_combine_part){m, shares, n, dim, b0 * 64 < dim ? b0 * 64 : dim, b1 * 64 < dim ? b1 * 64 : dim, out};
        if (pthread_create(&tid[t], NULL, or_combine_worker, &part[t]) != 0) break;
        ++started;
    }
    for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
    for (int t = started; t < threads; ++t) or_combine_worker(&part[t]);   /* could not start: run inline */
    return started;
}

/* ------------------------------------------------------------------------ */
/* additive -- client/src/crypto/sharing/additive.rs:32-51, batched.rs:19-53 */
/* ------------------------------------------------------------------------ */

void or_additive_generate(int64_t m, size_t n, const int64_t* secrets, size_t D,
                          const int64_t* draws, int64_t* out) {
    /* batched.rs:21-23: secrets_per_batch = 1, number_of_batches = D */
    for (size_t b = 0; b < D; ++b) {
        const int64_t secret = secrets[b];
        const int64_t* r = draws + b * (n - 1);
        /* additive.rs:42-44: n-1 draws gen_range(0, m) (supplied) */
        int64_t last = secret;
        for (size_t j = 0; j + 1 < n; ++j) {
            out[j * D + b] = r[j];
            /* additive.rs:47: fold(secret, |sum, &x| (sum - x) % modulus) */
            last = or_rem(or_wsub(last, r[j]), m);
        }
        out[(n - 1) * D + b] = last;   /* additive.rs:48 push; batched.rs:46-48 scatter */
    }
}

/* ------------------------------------------------------------------------ */
/* threshold-secret-sharing 0.2 numtheory / fft / packed [ext, restated]    */
/* ------------------------------------------------------------------------ */

int64_t or_mod_pow(int64_t x, uint32_t e, int64_t p) {
    /* numtheory::mod_pow: square-and-multiply, `%` after every product */
    int64_t acc = 1;
    while (e > 0) {
        if (e & 1u) acc = or_rem(or_wmul(acc, x), p);
        x = or_rem(or_wmul(x, x), p);
        e >>= 1;
    }
    return acc;
}

/* numtheory::gcd (extended Euclid, recursive): returns (g, s, t) with g = s*a + t*b */
static void or_egcd(int64_t a, int64_t b, int64_t* g, int64_t* s, int64_t* t) {
    if (b == 0) { *g = a; *s = 1; *t = 0; return; }
    int64_t n = a / b, c = a % b, g1, s1, t1;
    or_egcd(b, c, &g1, &s1, &t1);
    *g = g1; *s = t1; *t = s1 - t1 * n;
}

int64_t or_mod_inverse(int64_t k, int64_t p) {
    /* numtheory::mod_inverse */
    int64_t k2 = k % p, g, s, t, r;
    if (k2 < 0) { or_egcd(p, -k2, &g, &s, &t); r = -t; }
    else        { or_egcd(p, k2, &g, &s, &t); r = t; }
    return (p + r) % p;
}

/* fft::fft2 -- recursive radix-2 DIT, tss combine order:
 *   a[i]       = (b[i] + omega^i * c[i]) % p
 *   a[i + h]   = (b[i] - omega^i * c[i]) % p                                   */
static void or_fft2(const int64_t* a, size_t len, int64_t omega, int64_t p, int64_t* out) {
    if (len == 1) { out[0] = a[0]; return; }
    size_t h = len / 2;
    int64_t* tmp = (int64_t*)calloc(2 * len, sizeof(int64_t));
    int64_t *bc = tmp, *cc = tmp + h, *bp = tmp + len, *cp = tmp + len + h;
    for (size_t i = 0; i < h; ++i) { bc[i] = a[2 * i]; cc[i] = a[2 * i + 1]; }
    int64_t o2 = or_mod_pow(omega, 2, p);
    or_fft2(bc, h, o2, p, bp);
    or_fft2(cc, h, o2, p, cp);
    for (size_t i = 0; i < h; ++i) {
        int64_t w = or_mod_pow(omega, (uint32_t)i, p);
        out[i]     = or_rem(or_wadd(bp[i], or_wmul(w, cp[i])), p);
        out[i + h] = or_rem(or_wsub(bp[i], or_wmul(w, cp[i])), p);
    }
    free(tmp);
}

/* fft::fft2_inverse: fft2 with omega^-1, then `x * len_inv % p` */
static void or_fft2_inverse(const int64_t* a, size_t len, int64_t omega, int64_t p, int64_t* out) {
    int64_t omega_inv = or_mod_inverse(omega, p);
    int64_t len_inv = or_mod_inverse((int64_t)len, p);
    or_fft2(a, len, omega_inv, p, out);
    for (size_t i = 0; i < len; ++i) out[i] = or_rem(or_wmul(out[i], len_inv), p);
}

/* fft::fft3 -- recursive radix-3 DIT, tss combine order:
 *   a[j] = (b[i] + x * c[i] + x^2 * d[i]) % p,  x = omega^j, x^2 = x * x % p,
 *   j in {i, i + len/3, i + 2 len/3}                                            */
static void or_fft3(const int64_t* a, size_t len, int64_t omega, int64_t p, int64_t* out) {
    if (len == 1) { out[0] = a[0]; return; }
    size_t th = len / 3;
    int64_t* tmp = (int64_t*)calloc(2 * len, sizeof(int64_t));
    int64_t *bc = tmp, *cc = tmp + th, *dc = tmp + 2 * th;
    int64_t *bp = tmp + len, *cp = tmp + len + th, *dp = tmp + len + 2 * th;
    for (size_t i = 0; i < th; ++i) { bc[i] = a[3 * i]; cc[i] = a[3 * i + 1]; dc[i] = a[3 * i + 2]; }
    int64_t o3 = or_mod_pow(omega, 3, p);
    or_fft3(bc, th, o3, p, bp);
    or_fft3(cc, th, o3, p, cp);
    or_fft3(dc, th, o3, p, dp);
    for (size_t i = 0; i < th; ++i) {
        for (size_t q = 0; q < 3; ++q) {
            size_t j = i + q * th;
            int64_t x = or_mod_pow(omega, (uint32_t)j, p);
            int64_t x2 = or_rem(or_wmul(x, x), p);
            int64_t v = or_wadd(or_wadd(bp[i], or_wmul(x, cp[i])), or_wmul(x2, dp[i]));
            out[j] = or_rem(v, p);
        }
    }
    free(tmp);
}

void or_packed_share(const or_packed_params* pp, const int64_t* secrets,
                     const int64_t* randomness, int64_t* shares) {
    const size_t k = pp->secret_count, t = pp->privacy_threshold, n = pp->share_count;
    const size_t L = k + t + 1;           /* reconstruct_limit() + 1 */
    int64_t* values = (int64_t*)malloc(sizeof(int64_t) * (n + 1 > L ? n + 1 : L) * 3);
    int64_t* coeffs = values + (n + 1 > L ? n + 1 : L);
    int64_t* points = coeffs + (n + 1 > L ? n + 1 : L);
    /* packed::recover_polynomial: values = [0] ++ secrets ++ randomness */
    values[0] = 0;
    for (size_t i = 0; i < k; ++i) values[1 + i] = secrets[i];
    for (size_t i = 0; i < t; ++i) values[1 + k + i] = randomness[i];
    or_fft2_inverse(values, L, pp->omega_secrets, pp->prime, coeffs);
    /* packed::share: extend with zeros to share_count + 1 */
    for (size_t i = L; i < n + 1; ++i) coeffs[i] = 0;
    /* packed::evaluate_polynomial: fft3 over n+1 points */
    or_fft3(coeffs, n + 1, pp->omega_shares, pp->prime, points);
    /* drop points[0] (always 0) */
    for (size_t j = 0; j < n; ++j) shares[j] = points[j + 1];
    free(values);
}

void or_packed_generate(const or_packed_params* pp, const int64_t* secrets, size_t D,
                        const int64_t* randomness, int64_t* out) {
    const size_t k = pp->secret_count, t = pp->privacy_threshold, n = pp->share_count;
    /* batched.rs:21-23 */
    const size_t B = (D + k - 1) / k;
    int64_t* batch = (int64_t*)malloc(sizeof(int64_t) * (k + n));
    int64_t* sh = batch + k;
    for (size_t b = 0; b < B; ++b) {
        /* batched.rs:32-43: full batch, or zero-padded tail */
        for (size_t i = 0; i < k; ++i) {
            size_t idx = b * k + i;
            batch[i] = idx < D ? secrets[idx] : 0;
        }
        or_packed_share(pp, batch, randomness + b * t, sh);
        /* batched.rs:46-48: scatter to [clerk][batch] */
        for (size_t j = 0; j < n; ++j) out[j * B + b] = sh[j];
    }
    free(batch);
}

void or_packed_reconstruct_batch(const or_packed_params* pp, const size_t* indices,
                                 size_t n_idx, const int64_t* shares, int64_t* secrets) {
    const int64_t p = pp->prime;
    const size_t m = n_idx + 1;
    int64_t* points = (int64_t*)malloc(sizeof(int64_t) * m * 3);
    int64_t* store = points + m;       /* divided differences (value column of tss' store) */
    int64_t* np = store + m;
    size_t* lo = (size_t*)malloc(sizeof(size_t) * m * 2);
    size_t* hi = lo + m;
    /* packed::reconstruct: points = omega_shares^(idx+1), then insert (1, 0) in front */
    points[0] = 1;
    store[0] = 0;
    for (size_t i = 0; i < n_idx; ++i) {
        points[i + 1] = or_mod_pow(pp->omega_shares, (uint32_t)(indices[i] + 1), p);
        store[i + 1] = shares[i];
    }
    for (size_t i = 0; i < m; ++i) { lo[i] = i; hi[i] = i; }
    /* numtheory::compute_newton_coefficients */
    for (size_t j = 1; j < m; ++j) {
        for (size_t i = m - 1; i >= j; --i) {
            size_t index_lower = lo[i - 1], index_upper = hi[i];
            int64_t point_diff = or_rem(or_wsub(points[index_upper], points[index_lower]), p);
            int64_t point_diff_inverse = or_mod_inverse(point_diff, p);
            int64_t coef_diff = or_rem(or_wsub(store[i], store[i - 1]), p);
            int64_t fraction = or_rem(or_wmul(coef_diff, point_diff_inverse), p);
            lo[i] = index_lower; hi[i] = index_upper; store[i] = fraction;
            if (i == j) break;
        }
    }
    /* evaluate at omega_secrets^e, e = 1..k (numtheory::newton_evaluate) */
    for (size_t e = 1; e <= pp->secret_count; ++e) {
        int64_t point = or_mod_pow(pp->omega_secrets, (uint32_t)e, p);
        np[0] = 1;
        for (size_t i = 0; i + 1 < m; ++i) {
            int64_t diff = or_rem(or_wsub(point, points[i]), p);
            np[i + 1] = or_rem(or_wmul(np[i], diff), p);
        }
        int64_t acc = 0;
        for (size_t i = 0; i < m; ++i) acc = or_rem(or_wadd(acc, or_rem(or_wmul(store[i], np[i]), p)), p);
        secrets[e - 1] = acc;
    }
    free(points);
    free(lo);
}

int or_packed_reconstruct(const or_packed_params* pp, size_t dimension,
                          const size_t* indices, size_t n_idx,
                          const int64_t* shares, int64_t* out) {
    const size_t k = pp->secret_count;
    /* batched.rs:75-77: batch_input_size = |I|; B from output_size (= dimension) */
    const size_t B = (dimension + k - 1) / k;
    int64_t* col = (int64_t*)malloc(sizeof(int64_t) * (n_idx + k + 1));
    int64_t* sec = col + n_idx;
    size_t w = 0;
    for (size_t b = 0; b < B; ++b) {
        /* packed_shamir.rs:74-75 error checks (per batch; identical for all batches) */
        /* :74 batch_shares.len() != indices.len() cannot differ in this layout */
        if (n_idx < pp->privacy_threshold + pp->secret_count) { free(col); return 6; }
        for (size_t i = 0; i < n_idx; ++i) col[i] = shares[i * B + b];   /* batched.rs:83-85 */
        or_packed_reconstruct_batch(pp, indices, n_idx, col, sec);
        for (size_t e = 0; e < k; ++e, ++w)
            if (w < dimension) out[w] = sec[e];                          /* batched.rs:94 truncate */
    }
    free(col);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* ChaCha20 core + rand-0.3 ChaChaRng [ext, restated]                      */
/* ------------------------------------------------------------------------ */

static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define QR(a, b, c, d)                         \
    a += b; d ^= a; d = rotl32(d, 16);         \
    c += d; b ^= c; b = rotl32(b, 12);         \
    a += b; d ^= a; d = rotl32(d, 8);          \
    c += d; b ^= c; b = rotl32(b, 7);

void or_chacha20_core(const uint32_t in[16], uint32_t out[16]) {
    uint32_t x[16];
    memcpy(x, in, sizeof(x));
    for (int r = 0; r < 10; ++r) {
        QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

void or_chacha_rng_from_seed(or_chacha_rng* r, const uint32_t* seed, size_t n_words) {
    /* ChaChaRng::from_seed -> reseed: init(&[0; 8]) then key words = seed (zip: at most 8) */
    r->state[0] = 0x61707865u; r->state[1] = 0x3320646Eu;
    r->state[2] = 0x79622D32u; r->state[3] = 0x6B206574u;
    for (int i = 0; i < 8; ++i) r->state[4 + i] = 0;
    for (size_t i = 0; i < n_words && i < 8; ++i) r->state[4 + i] = seed[i];
    for (int i = 12; i < 16; ++i) r->state[i] = 0;
    r->index = 16;
}

static void or_chacha_update(or_chacha_rng* r) {
    or_chacha20_core(r->state, r->buffer);
    r->index = 0;
    /* 128-bit block counter in state words 12..15 */
    if (++r->state[12] != 0) return;
    if (++r->state[13] != 0) return;
    if (++r->state[14] != 0) return;
    ++r->state[15];
}

uint32_t or_chacha_next_u32(or_chacha_rng* r) {
    if (r->index == 16) or_chacha_update(r);
    return r->buffer[r->index++ % 16];
}

uint64_t or_chacha_next_u64(or_chacha_rng* r) {
    /* Rng::next_u64 default: (next_u32 << 32) | next_u32 -- high word drawn first */
    uint64_t hi = or_chacha_next_u32(r);
    uint64_t lo = or_chacha_next_u32(r);
    return (hi << 32) | lo;
}

int64_t or_chacha_gen_range(or_chacha_rng* r, int64_t low, int64_t high) {
    /* distributions::range integer_impl for i64/u64 */
    uint64_t range = (uint64_t)high - (uint64_t)low;
    uint64_t zone = UINT64_MAX - UINT64_MAX % range;
    for (;;) {
        uint64_t v = or_chacha_next_u64(r);
        if (v < zone) return (int64_t)((uint64_t)low + v % range);
    }
}

/* ------------------------------------------------------------------------ */
/* masking -- client/src/crypto/masking/{chacha,full}.rs, receive.rs        */
/* ------------------------------------------------------------------------ */

void or_chacha_mask(int64_t m, const uint32_t* seed, size_t n_words,
                    const int64_t* secrets, size_t D, int64_t* masked) {
    or_chacha_rng r;
    or_chacha_rng_from_seed(&r, seed, n_words);               /* chacha.rs:36 */
    for (size_t i = 0; i < D; ++i) {
        int64_t mask = or_chacha_gen_range(&r, 0, m);         /* chacha.rs:37-39 */
        masked[i] = or_rem(or_wadd(secrets[i], mask), m);     /* chacha.rs:42-45 */
    }
}

void or_chacha_mask_combine(int64_t m, size_t dimension, const int64_t* seeds,
                            size_t w, size_t N, int64_t* out) {
    uint32_t seed[64];
    for (size_t i = 0; i < dimension; ++i) out[i] = 0;        /* chacha.rs:58 */
    for (size_t s = 0; s < N; ++s) {
        size_t nw = w < 64 ? w : 64;
        for (size_t j = 0; j < nw; ++j) seed[j] = (uint32_t)seeds[s * w + j];   /* :62-64 */
        or_chacha_rng r;
        or_chacha_rng_from_seed(&r, seed, nw);                /* :67 */
        for (size_t i = 0; i < dimension; ++i) {              /* :68-72 */
            int64_t mk = or_chacha_gen_range(&r, 0, m);
            out[i] = or_rem(or_wadd(out[i], mk), m);
        }
    }
}

void or_unmask(int64_t q, const int64_t* masks, const int64_t* masked, size_t D, int64_t* out) {
    for (size_t i = 0; i < D; ++i) out[i] = or_rem(or_wsub(masked[i], masks[i]), q);
}

void or_full_mask(int64_t m, const int64_t* masks, const int64_t* secrets, size_t D, int64_t* out) {
    for (size_t i = 0; i < D; ++i) out[i] = or_rem(or_wadd(secrets[i], masks[i]), m);
}

void or_positive(int64_t m, const int64_t* vals, size_t D, int64_t* out) {
    for (size_t i = 0; i < D; ++i) out[i] = vals[i] < 0 ? vals[i] + m : vals[i];
}

/* ------------------------------------------------------------------------ */
/* varint codec -- integer-encoding 1.0 VarInt for i64 (zigzag + LEB128)    */
/* ------------------------------------------------------------------------ */

size_t or_varint_encode(const int64_t* vals, size_t n, uint8_t* out) {
    size_t w = 0;
    for (size_t i = 0; i < n; ++i) {
        uint64_t z = ((uint64_t)vals[i] << 1) ^ (uint64_t)(vals[i] >> 63);
        while (z >= 0x80) { out[w++] = (uint8_t)(z | 0x80); z >>= 7; }
        out[w++] = (uint8_t)z;
    }
    return w;
}

/* Decryptor::decrypt's loop (sodium.rs:82-88):
 *     while reader.len() > 0 { let (i, size) = Share::decode_var(reader); push(i); reader = &reader[size..] }
 * with integer-encoding 1.0 u64::decode_var (then zigzag for i64):
 *     for b in src { result |= ((b & 0x7f) as u64) << shift; shift += 7;
 *                    if b & 0x80 == 0 || shift > 10 * 7 { break } }      size = shift / 7
 * Rust release builds mask an over-wide shift (`<< 70` == `<< 6`), reproduced with `& 63`, so a
 * run of >= 11 continuation bytes becomes an 11-byte element, and a truncated final varint
 * yields the partial value. */
size_t or_varint_decode(const uint8_t* in, size_t n_bytes, int64_t* out, size_t cap) {
    size_t r = 0, c = 0;
    while (r < n_bytes && c < cap) {
        uint64_t z = 0;
        unsigned shift = 0;
        while (r < n_bytes) {
            const uint8_t b = in[r++];
            z |= (uint64_t)(b & 0x7f) << (shift & 63);
            shift += 7;
            if (!(b & 0x80) || shift > 70) break;
        }
        out[c++] = (int64_t)((z >> 1) ^ (0 - (z & 1)));
    }
    return c;
}

/* server/src/stores.rs:86-101: shares[ix].push(share) for every participation in snapshot order. */
void or_snapshot_transpose(const uint8_t* in, const uint64_t* part_off, size_t P, size_t n,
                           uint8_t* out, uint64_t* clerk_off) {
    uint64_t w = 0;
    for (size_t c = 0; c < n; ++c)
        for (size_t p = 0; p <= P; ++p) {
            clerk_off[c * (P + 1) + p] = w;
            if (p == P) break;
            const uint64_t b = part_off[p * n + c], e = part_off[p * n + c + 1];
            memcpy(out + w, in + b, e - b);
            w += e - b;
        }
}
