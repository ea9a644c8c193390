// chacha_reject_search.hip -- test-vector search (not product code): 128-bit ChaCha seeds whose rand-0.3
// gen_range(0, m) stream (chacha.hip's definition: ChaCha20, key = seed words zero-padded to 8, 64-bit
// block counter from 0, next_u64 = high word first) REJECTS a draw among its first `pairs` pairs.
// Such draws occur with probability (2^64 mod m + 1) / 2^64 per pair (< 2^-33 for the field prime), so
// the tests that exercise the engine's rejection fix-up need seeds found this way.
//   hipcc -O3 --offload-arch=gfx950 tools/chacha_reject_search.hip -o tools/chacha_reject_search
//   ./tools/chacha_reject_search <m> <pairs> <seeds_log2> <w1> <w2> <w3>
// prints "seed s w1 w2 w3 pair P" for every rejected pair of seeds (s, w1, w2, w3), s < 2^seeds_log2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define QR(a, b, c, d)                                          \
    a += b; d ^= a; d = (d << 16) | (d >> 16);                  \
    c += d; b ^= c; b = (b << 12) | (b >> 20);                  \
    a += b; d ^= a; d = (d << 8) | (d >> 24);                   \
    c += d; b ^= c; b = (b << 7) | (b >> 25);

__global__ void search(uint64_t zone, uint64_t blocks_per_seed, uint64_t pairs, uint32_t w1, uint32_t w2, uint32_t w3,
                       uint64_t total, unsigned long long* count, uint64_t* hits, uint32_t cap) {
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t s = (uint32_t)(g / blocks_per_seed);
    const uint64_t blk = g % blocks_per_seed;
    const uint32_t in[16] = {0x61707865u, 0x3320646Eu, 0x79622D32u, 0x6B206574u, s, w1, w2, w3, 0, 0, 0, 0,
                             (uint32_t)blk, (uint32_t)(blk >> 32), 0, 0};
    uint32_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = in[i];
    for (int r = 0; r < 10; ++r) {
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
    for (int q = 0; q < 8; ++q) {
        const uint64_t pair = blk * 8 + q;
        const uint64_t v = ((uint64_t)(x[2 * q] + in[2 * q]) << 32) | (uint64_t)(x[2 * q + 1] + in[2 * q + 1]);
        if (pair < pairs && v >= zone) {
            const unsigned long long i = atomicAdd(count, 1ull);
            if (i < cap) hits[i] = ((uint64_t)s << 40) | pair;
        }
    }
  }
}

int main(int argc, char** argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: %s m pairs seeds_log2 w1 w2 w3\n", argv[0]);
        return 2;
    }
    const uint64_t m = strtoull(argv[1], nullptr, 0), pairs = strtoull(argv[2], nullptr, 0);
    const int lg = atoi(argv[3]);
    const uint32_t w1 = (uint32_t)strtoul(argv[4], nullptr, 0), w2 = (uint32_t)strtoul(argv[5], nullptr, 0),
                   w3 = (uint32_t)strtoul(argv[6], nullptr, 0);
    if (m < 2 || pairs == 0 || pairs >= (1ull << 40) || lg < 0 || lg > 24) return 2;
    const uint64_t zone = UINT64_MAX - UINT64_MAX % m;
    const uint64_t bps = (pairs + 7) / 8, total = bps << lg;
    const uint32_t cap = 4096;
    unsigned long long* count;
    uint64_t* hits;
    if (hipMalloc(&count, 8) != hipSuccess || hipMalloc(&hits, cap * 8) != hipSuccess) return 1;
    (void)hipMemset(count, 0, 8);
    const uint64_t grid = (total + 255) / 256 < (1ull << 20) ? (total + 255) / 256 : (1ull << 20);   // grid-stride
    hipLaunchKernelGGL(search, dim3((unsigned)grid), dim3(256), 0, 0, zone, bps, pairs, w1, w2, w3, total, count, hits,
                       cap);
    unsigned long long n = 0;
    if (hipMemcpy(&n, count, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    uint64_t h[cap];
    const uint32_t k = n < cap ? (uint32_t)n : cap;
    if (k && hipMemcpy(h, hits, k * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("m %llu zone %llu rejected-per-pair %.3g pairs %llu seeds %llu hits %llu\n", (unsigned long long)m,
           (unsigned long long)zone, (double)(UINT64_MAX % m + 1) / 18446744073709551616.0,
           (unsigned long long)pairs, 1ull << lg, n);
    for (uint32_t i = 0; i < k; ++i)
        printf("seed %llu 0x%x 0x%x 0x%x pair %llu\n", (unsigned long long)(h[i] >> 40), w1, w2, w3,
               (unsigned long long)(h[i] & ((1ull << 40) - 1)));
    return 0;
}
