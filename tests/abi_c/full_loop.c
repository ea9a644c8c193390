/*
 * full_loop.c -- a plain C consumer of include/sda_engine.h (no torch, no Python in the process).
 *
 * Runs one aggregation of integration-tests/tests/full_loop.rs:30-150 through the host entry
 * points, in the order of the reference workflows (tests/pipeline.py documents the same flow):
 *   participate.rs:53-76  sda_secret_mask, sda_share_generate          (per participant)
 *   clerk.rs:79-86        sda_share_combine                             (per clerk, snapshot order)
 *   receive.rs:102-152    sda_mask_combine, sda_secret_reconstruct, sda_secret_unmask
 *   receive.rs:14-20      sda_recipient_positive
 * plus the fused sda_recipient_reveal.  The OsRng draws come from stdin (the golden fixture's
 * trace, written by tests/test_abi_c.py); every stage is printed as "key: v v v" for the test to
 * compare with the golden trace.
 *
 * stdin:  mkind mmod mdim mbits
 *         skind n mod k t ws wn
 *         dimension output_modulus participants
 *         per participant:  secrets[dimension]  mask_len masks[mask_len]  n_draws draws[n_draws]
 *         n_order order[n_order]
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sda_engine.h"

#define MAXP 16
#define MAXN 64
#define MAXV 4096

static int64_t rd(void) {
    long long v;
    if (scanf("%lld", &v) != 1) {
        fprintf(stderr, "bad input\n");
        exit(2);
    }
    return (int64_t)v;
}

static void put(const char* key, const int64_t* v, uint64_t n) {
    printf("%s:", key);
    for (uint64_t i = 0; i < n; ++i) printf(" %" PRId64, v[i]);
    printf("\n");
}

static void check(sda_status st, const char* what) {
    if (st != SDA_OK) {
        fprintf(stderr, "%s failed: %s (%s)\n", what, sda_status_string(st), sda_last_error_message());
        exit(1);
    }
}

static int64_t secrets[MAXP][MAXV], masks[MAXP][MAXV], masked[MAXP][MAXV], draws[MAXP][MAXV];
static int64_t shares[MAXP][MAXN * MAXV], clerk[MAXN][MAXV], tmp[MAXV], tmp2[MAXV], outv[MAXV];
static uint64_t mask_len[MAXP];

int main(void) {
    sda_masking_scheme ms;
    sda_sharing_scheme ss;
    memset(&ms, 0, sizeof ms);
    memset(&ss, 0, sizeof ss);
    ms.kind = (int32_t)rd(); ms.modulus = rd(); ms.dimension = (uint64_t)rd(); ms.seed_bitsize = (uint64_t)rd();
    ss.kind = (int32_t)rd(); ss.share_count = (uint64_t)rd(); ss.modulus = rd();
    ss.secret_count = (uint64_t)rd(); ss.privacy_threshold = (uint64_t)rd();
    ss.omega_secrets = rd(); ss.omega_shares = rd();
    const uint64_t D = (uint64_t)rd();
    const int64_t out_mod = rd();
    const uint64_t P = (uint64_t)rd();
    const uint64_t n = sda_scheme_output_size(&ss), B = sda_share_length(&ss, D);
    if (P > MAXP || n > MAXN || D > MAXV || n * B > MAXN * MAXV) return 2;

    /* SDA_TEST_DEVICES="0,0,..." opens one handle over those ordinals (sda_engine_create_multi): the host
     * trait calls then split over them (a one-device list reduces ChaCha masks through a one-rank RCCL
     * communicator) */
    sda_engine* h = NULL;
    const char* devs = getenv("SDA_TEST_DEVICES");
    if (devs && *devs) {
        int ord[16], nd = 0;
        for (const char* c = devs; *c && nd < 16;) {
            ord[nd++] = atoi(c);
            while (*c && *c != ',') ++c;
            if (*c == ',') ++c;
        }
        check(sda_engine_create_multi(ord, nd, &h), "sda_engine_create_multi");
        if (sda_engine_device_count(h) != nd) {
            fprintf(stderr, "sda_engine_device_count: %d != %d\n", sda_engine_device_count(h), nd);
            return 1;
        }
    } else {
        check(sda_engine_create(0, &h), "sda_engine_create");
    }
    printf("abi_version: %d\n", sda_abi_version());

    char key[64];
    for (uint64_t p = 0; p < P; ++p) {
        for (uint64_t i = 0; i < D; ++i) secrets[p][i] = rd();
        const uint64_t ml = (uint64_t)rd();
        for (uint64_t i = 0; i < ml; ++i) tmp[i] = rd();
        const uint64_t nd = (uint64_t)rd();
        for (uint64_t i = 0; i < nd; ++i) draws[p][i] = rd();
        /* SecretMasker::mask: Full takes the drawn masks, ChaCha the drawn seed words */
        uint32_t seed[16];
        for (uint64_t i = 0; i < ml && i < 16; ++i) seed[i] = (uint32_t)tmp[i];
        const int full = ms.kind == SDA_MASKING_FULL, chacha = ms.kind == SDA_MASKING_CHACHA;
        check(sda_secret_mask(h, &ms, secrets[p], D, chacha ? seed : NULL, chacha ? ml : 0, full ? tmp : NULL,
                              masks[p], MAXV, &mask_len[p], masked[p]),
              "sda_secret_mask");
        snprintf(key, sizeof key, "masks %" PRIu64, p);
        put(key, masks[p], mask_len[p]);
        snprintf(key, sizeof key, "masked %" PRIu64, p);
        put(key, masked[p], D);
        /* ShareGenerator::generate: [n][B] clerk-major */
        check(sda_share_generate(h, &ss, masked[p], D, draws[p], nd, shares[p], MAXN * MAXV), "sda_share_generate");
        for (uint64_t c = 0; c < n; ++c) {
            snprintf(key, sizeof key, "shares %" PRIu64 " %" PRIu64, p, c);
            put(key, shares[p] + c * B, B);
        }
    }
    /* clerks: ShareCombiner::combine over the participations in snapshot order */
    const int64_t* rows[MAXP];
    uint64_t lens[MAXP], len = 0;
    for (uint64_t c = 0; c < n; ++c) {
        for (uint64_t p = 0; p < P; ++p) { rows[p] = shares[p] + c * B; lens[p] = B; }
        check(sda_share_combine(h, &ss, rows, lens, P, clerk[c], MAXV, &len), "sda_share_combine");
        snprintf(key, sizeof key, "clerk %" PRIu64, c);
        put(key, clerk[c], len);
    }
    /* recipient: MaskCombiner::combine, SecretReconstructor::reconstruct, SecretUnmasker::unmask */
    uint64_t mlen = 0;
    if (ms.kind != SDA_MASKING_NONE) {
        for (uint64_t p = 0; p < P; ++p) { rows[p] = masks[p]; lens[p] = mask_len[p]; }
        check(sda_mask_combine(h, &ms, rows, lens, P, tmp, MAXV, &mlen), "sda_mask_combine");
        put("combined_mask", tmp, mlen);
    }
    const uint64_t n_order = (uint64_t)rd();
    uint64_t idx[MAXN];
    const int64_t* srows[MAXN];
    uint64_t slens[MAXN];
    for (uint64_t i = 0; i < n_order; ++i) {
        idx[i] = (uint64_t)rd();
        srows[i] = clerk[idx[i]];
        slens[i] = B;
    }
    uint64_t olen = 0;
    check(sda_secret_reconstruct(h, &ss, D, idx, srows, slens, n_order, tmp2, MAXV, &olen), "sda_secret_reconstruct");
    put("masked_output", tmp2, olen);
    uint64_t ulen = 0;
    check(sda_secret_unmask(h, &ms, tmp, mlen, tmp2, olen, outv, MAXV, &ulen), "sda_secret_unmask");
    put("output", outv, ulen);
    check(sda_recipient_positive(h, out_mod, outv, ulen, tmp2), "sda_recipient_positive");
    put("positive", tmp2, ulen);
    /* the same reveal as one fused device pipeline */
    for (uint64_t p = 0; p < P; ++p) { rows[p] = masks[p]; lens[p] = mask_len[p]; }
    check(sda_recipient_reveal(h, &ms, rows, lens, ms.kind == SDA_MASKING_NONE ? 0 : P, &ss, D, idx, srows, slens,
                               n_order, out_mod, SDA_REVEAL_EXACT, outv, MAXV, &ulen),
          "sda_recipient_reveal");
    put("fused_reveal", outv, ulen);
    sda_engine_destroy(h);
    return 0;
}
