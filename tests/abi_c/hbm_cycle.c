/*
 * hbm_cycle.c -- sda_hbm_alloc / sda_hbm_free / sda_hbm_trim from a plain C program on the ROCm runtime the
 * engine was built against (/opt/rocm/lib/libamdhip64, as the Rust shim of INTEGRATION.md would load it; no
 * torch in the process).  tests/test_abi_c.py runs each mode and checks its output lines.
 *
 *   hbm_cycle seq      the trim / re-allocate sequence of tests/test_gpu_hbm.py (the round-4 corruption:
 *                      a filled buffer freed and released, a foreign hipMalloc block, new buffers, share-gen
 *                      into one of them), three rounds with every free releasing at once (SDA_HBM_POOL_MB=0):
 *                      share-gen into the sda_hbm buffer equals share-gen into a hipMalloc buffer (read twice),
 *                      no new buffer lies in a retired range, the foreign block is untouched.
 *   hbm_cycle gen      configs[2] (PackedShamir k=8 n=26 t=7, p = 2147482801) at 1M-dim: inputs from the
 *                      splitmix64 generator (sda_synth_fill_dev), shares through the host entry point and
 *                      through the _dev one into an sda_hbm buffer; prints both checksums, which must equal
 *                      tests/golden/abi_c_sharegen.json (the oracle's tss shares, tests/golden/make_golden.py).
 *   hbm_cycle cycle N  N alloc / free cycles of mixed job sizes (1-3 buffers of 2-192 MiB each, 2 MiB chunks,
 *                      each touched by a memset): prints the bytes retired, pooled and live, and the pool's peak.
 *                      With the default pool bound nothing is retired (size-class reuse).
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "sda_engine.h"

static void check(sda_status st, const char* what) {
    if (st != SDA_OK) {
        fprintf(stderr, "%s failed: %s (%s)\n", what, sda_status_string(st), sda_last_error_message());
        exit(1);
    }
}

static void hcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        fprintf(stderr, "%s failed: %s\n", what, hipGetErrorString(e));
        exit(1);
    }
}

static uint64_t splitmix64_at(uint64_t seed, uint64_t idx) {   /* sda_amd/synth.py */
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Two order-sensitive sums over the i64 words (tests/golden/make_golden.py computes the same). */
static void checksum(const int64_t* v, uint64_t n, uint64_t* c1, uint64_t* c2) {
    uint64_t a = 0, b = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t k = splitmix64_at(0xC5C5, i) | 1u;
        a += (uint64_t)v[i] * k;
        b += (uint64_t)v[i] ^ k;
    }
    *c1 = a;
    *c2 = b;
}

static const sda_sharing_scheme CONFIG_PACKED = {SDA_SHARING_PACKED_SHAMIR, 26, 2147482801, 8, 7, 50280738,
                                                 1761728707};

static void* hbm(uint64_t bytes) {
    void* p = NULL;
    check(sda_hbm_alloc(0, bytes, &p), "sda_hbm_alloc");
    return p;
}

static void stats(uint64_t* live, uint64_t* pooled, uint64_t* retired) {
    check(sda_hbm_stats(0, live, pooled, retired), "sda_hbm_stats");
}

static int mode_seq(sda_engine* h) {
    const sda_sharing_scheme* s = &CONFIG_PACKED;
    const uint64_t p = (uint64_t)s->modulus, V = 8, Dm = 1000000, B = Dm / 8, n = 26, t = 7;
    const uint64_t a_bytes = 300ull << 23, sh_words = V * n * B;   /* 2.4 GB, as the torch test's buffer */
    uint64_t live, pooled, retired0, retired;
    setenv("SDA_HBM_POOL_MB", "0", 1);                              /* every free releases (and retires) */
    stats(&live, &pooled, &retired0);
    int64_t* h1 = malloc(sh_words * 8);
    int64_t* h2 = malloc(sh_words * 8);
    uint8_t* hb = malloc(a_bytes);
    if (!h1 || !h2 || !hb) return 2;
    for (int r = 0; r < 3; ++r) {
        int64_t* a = hbm(a_bytes);
        check(sda_synth_fill_dev(h, a, 300, 1u << 20, 40 + r, 1, 1ll << 40, NULL), "fill a");
        hcheck(hipDeviceSynchronize(), "sync");
        const uintptr_t a_lo = (uintptr_t)a, a_hi = a_lo + a_bytes;
        check(sda_hbm_free(a), "free a");
        check(sda_hbm_trim(0, 0), "trim");
        stats(&live, &pooled, &retired);
        if (pooled != 0) { printf("seq: pooled %" PRIu64 " after trim\n", pooled); return 1; }
        void* blk = NULL;                                           /* the foreign allocation (torch's role) */
        hcheck(hipMalloc(&blk, a_bytes), "hipMalloc");
        hcheck(hipMemset(blk, 0x5A, a_bytes), "hipMemset");
        int64_t* sec = hbm(V * Dm * 8);
        int64_t* drw = hbm(V * B * t * 8);
        int64_t* sh_h = hbm(sh_words * 8);
        const uintptr_t bufs[3][2] = {{(uintptr_t)sec, V * Dm * 8}, {(uintptr_t)drw, V * B * t * 8},
                                      {(uintptr_t)sh_h, sh_words * 8}};
        for (int i = 0; i < 3; ++i)
            if (!(bufs[i][0] + bufs[i][1] <= a_lo || bufs[i][0] >= a_hi)) {
                printf("seq: a new buffer lies in a retired range\n");
                return 1;
            }
        check(sda_synth_fill_dev(h, sec, V, Dm, 21 + r, 0, (int64_t)p, NULL), "fill sec");
        check(sda_synth_fill_dev(h, drw, V * B, t, 22 + r, 0, (int64_t)p - 1, NULL), "fill drw");
        int64_t* sh_t = NULL;
        hcheck(hipMalloc((void**)&sh_t, sh_words * 8), "hipMalloc shares");
        check(sda_packed_generate_mode_dev(h, s, sec, Dm, V, drw, sh_h, SDA_REVEAL_EXACT, NULL), "gen hbm");
        check(sda_packed_generate_mode_dev(h, s, sec, Dm, V, drw, sh_t, SDA_REVEAL_EXACT, NULL), "gen hipMalloc");
        hcheck(hipDeviceSynchronize(), "sync");
        for (int rep = 0; rep < 2; ++rep) {
            hcheck(hipMemcpy(h1, sh_h, sh_words * 8, hipMemcpyDeviceToHost), "d2h");
            hcheck(hipMemcpy(h2, sh_t, sh_words * 8, hipMemcpyDeviceToHost), "d2h");
            if (memcmp(h1, h2, sh_words * 8) != 0) { printf("seq: round %d read %d differs\n", r, rep); return 1; }
        }
        hcheck(hipMemcpy(hb, blk, a_bytes, hipMemcpyDeviceToHost), "d2h blk");
        for (uint64_t i = 0; i < a_bytes; ++i)
            if (hb[i] != 0x5A) { printf("seq: foreign block byte %" PRIu64 " changed\n", i); return 1; }
        check(sda_hbm_free(sec), "free");
        check(sda_hbm_free(drw), "free");
        check(sda_hbm_free(sh_h), "free");
        hcheck(hipFree(sh_t), "hipFree");
        hcheck(hipFree(blk), "hipFree");
    }
    check(sda_hbm_trim(0, 0), "trim");
    stats(&live, &pooled, &retired);
    printf("seq: ok rounds 3 pooled %" PRIu64 " retired_delta %" PRIu64 "\n", pooled, retired - retired0);
    free(h1);
    free(h2);
    free(hb);
    return 0;
}

static int mode_gen(sda_engine* h) {
    const sda_sharing_scheme* s = &CONFIG_PACKED;
    const uint64_t p = (uint64_t)s->modulus, D = 1000000, B = D / 8, n = 26, t = 7;
    int64_t *dsec = hbm(D * 8), *ddr = hbm(B * t * 8), *dsh = hbm(n * B * 8);
    check(sda_synth_fill_dev(h, dsec, 1, D, 0x5DA + 2, 0, (int64_t)p, NULL), "fill secrets");
    check(sda_synth_fill_dev(h, ddr, B, t, 0x5DA + 3, 0, (int64_t)p - 1, NULL), "fill draws");
    int64_t* sec = malloc(D * 8);
    int64_t* dr = malloc(B * t * 8);
    int64_t* sh = malloc(n * B * 8);
    if (!sec || !dr || !sh) return 2;
    hcheck(hipMemcpy(sec, dsec, D * 8, hipMemcpyDeviceToHost), "d2h");
    hcheck(hipMemcpy(dr, ddr, B * t * 8, hipMemcpyDeviceToHost), "d2h");
    uint64_t c1, c2;
    check(sda_share_generate(h, s, sec, D, dr, B * t, sh, n * B), "sda_share_generate");
    checksum(sh, n * B, &c1, &c2);
    printf("gen_host: %" PRIu64 " %" PRIu64 "\n", c1, c2);
    check(sda_packed_generate_dev(h, s, dsec, D, 1, ddr, dsh, NULL), "sda_packed_generate_dev");
    hcheck(hipDeviceSynchronize(), "sync");
    memset(sh, 0, n * B * 8);
    hcheck(hipMemcpy(sh, dsh, n * B * 8, hipMemcpyDeviceToHost), "d2h");
    checksum(sh, n * B, &c1, &c2);
    printf("gen_dev: %" PRIu64 " %" PRIu64 "\n", c1, c2);
    check(sda_hbm_free(dsec), "free");
    check(sda_hbm_free(ddr), "free");
    check(sda_hbm_free(dsh), "free");
    free(sec);
    free(dr);
    free(sh);
    return 0;
}

static int mode_cycle(long cycles) {
    setenv("SDA_HBM_CHUNK_MB", "2", 1);
    uint64_t live, pooled, retired0, retired, peak = 0;
    stats(&live, &pooled, &retired0);
    uint64_t rng = 0;
    for (long c = 0; c < cycles; ++c) {
        void* bufs[3];
        const int nb = 1 + (int)(splitmix64_at(7, rng++) % 3);
        for (int i = 0; i < nb; ++i) {
            const uint64_t mib = 2 + splitmix64_at(7, rng++) % 191;      /* 2 .. 192 MiB */
            const uint64_t bytes = (mib << 20) - splitmix64_at(7, rng++) % 4096;
            bufs[i] = hbm(bytes);
            hcheck(hipMemsetAsync(bufs[i], (int)(c & 0xFF), 4096, NULL), "memset");
            hcheck(hipMemsetAsync((char*)bufs[i] + bytes - 4096, (int)(c & 0xFF), 4096, NULL), "memset");
        }
        for (int i = 0; i < nb; ++i) check(sda_hbm_free(bufs[i]), "free");
        stats(&live, &pooled, &retired);
        if (pooled > peak) peak = pooled;
    }
    hcheck(hipDeviceSynchronize(), "sync");
    stats(&live, &pooled, &retired);
    printf("cycle: cycles %ld retired %" PRIu64 " pooled %" PRIu64 " live %" PRIu64 " peak_pooled %" PRIu64 "\n",
           cycles, retired - retired0, pooled, live, peak);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: hbm_cycle seq|gen|cycle [N]\n");
        return 2;
    }
    sda_engine* h = NULL;
    check(sda_engine_create(0, &h), "sda_engine_create");
    int rc = 2;
    if (!strcmp(argv[1], "seq")) rc = mode_seq(h);
    else if (!strcmp(argv[1], "gen")) rc = mode_gen(h);
    else if (!strcmp(argv[1], "cycle")) rc = mode_cycle(argc > 2 ? atol(argv[2]) : 10000);
    sda_engine_destroy(h);
    return rc;
}
