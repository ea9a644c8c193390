// hbm_diag.hip -- scripts/hbm_diag.py without torch: the same alloc / trim / realloc sequence on ROCm's own
// HIP runtime (/opt/rocm, linked directly), with hipMalloc blocks standing in for torch's allocations.
// Each round: VMM buffer A (64 MiB chunks) filled, unmapped + released, its range returned to the runtime
// (argv[1] = 1) or kept reserved (0); a hipMalloc block T filled with a pattern; a new VMM buffer X and a
// hipMalloc block REF filled by the same kernel; then mismatches X vs REF (three reads), zeros in X and
// words of T that lost the pattern are counted on the device.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/hbm_diag.hip -o tools/hbm_diag && ./tools/hbm_diag 1 6
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);   \
            exit(2);                                                                              \
        }                                                                                         \
    } while (0)

constexpr uint64_t kPattern = 0x5A5A5A5A5A5A5A5Aull;
constexpr size_t kChunk = 64ull << 20;

__device__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void fill(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = mix(seed ^ (i * 0x100000001B3ull)) | 1;           // never 0
}
__global__ void fill_const(uint64_t* p, uint64_t n, uint64_t v) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}
__global__ void count_ne(const uint64_t* a, const uint64_t* b, uint64_t n, unsigned long long* out) {
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        c += a[i] != b[i];
    if (c) atomicAdd(out, c);
}
__global__ void count_eq(const uint64_t* a, uint64_t n, uint64_t v, unsigned long long* out) {
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        c += a[i] == v;
    if (c) atomicAdd(out, c);
}

struct Vmm {
    void* ptr = nullptr;
    size_t bytes = 0;
    std::vector<hipMemGenericAllocationHandle_t> h;
};

Vmm vmm_alloc(size_t bytes) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    Vmm v;
    size_t n = (bytes + kChunk - 1) / kChunk;
    v.bytes = n * kChunk;
    CK(hipMemAddressReserve(&v.ptr, v.bytes, kChunk, nullptr, 0));
    for (size_t i = 0; i < n; ++i) {
        hipMemGenericAllocationHandle_t c;
        CK(hipMemCreate(&c, kChunk, &prop, 0));
        v.h.push_back(c);
        CK(hipMemMap(static_cast<char*>(v.ptr) + i * kChunk, kChunk, 0, c, 0));
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(v.ptr, v.bytes, &acc, 1));
    return v;
}

void vmm_free(Vmm& v, bool va_free) {
    CK(hipDeviceSynchronize());
    for (size_t i = 0; i < v.h.size(); ++i) CK(hipMemUnmap(static_cast<char*>(v.ptr) + i * kChunk, kChunk));
    for (auto c : v.h) CK(hipMemRelease(c));
    if (va_free) CK(hipMemAddressFree(v.ptr, v.bytes));
    v.h.clear();
}

unsigned long long* g_cnt;
unsigned long long ne(const uint64_t* a, const uint64_t* b, uint64_t n) {
    CK(hipMemset(g_cnt, 0, 8));
    count_ne<<<4096, 256>>>(a, b, n, g_cnt);
    unsigned long long c;
    CK(hipMemcpy(&c, g_cnt, 8, hipMemcpyDeviceToHost));
    return c;
}
unsigned long long eq(const uint64_t* a, uint64_t n, uint64_t v) {
    CK(hipMemset(g_cnt, 0, 8));
    count_eq<<<4096, 256>>>(a, n, v, g_cnt);
    unsigned long long c;
    CK(hipMemcpy(&c, g_cnt, 8, hipMemcpyDeviceToHost));
    return c;
}

int main(int argc, char** argv) {
    const bool va_free = argc > 1 && atoi(argv[1]) == 1;
    const int rounds = argc > 2 ? atoi(argv[2]) : 6;
    int rt = 0;
    CK(hipRuntimeGetVersion(&rt));
    printf("hbm_diag (ROCm runtime %d, no torch) va_free=%d\n", rt, (int)va_free);
    CK(hipMalloc(&g_cnt, 64));
    const uint64_t cols = 1ull << 20;
    std::vector<std::pair<uintptr_t, uintptr_t>> trimmed;
    int bad = 0;
    for (int r = 0; r < rounds; ++r) {
        const uint64_t rows_a = (r % 3 == 0) ? 300 : (r % 3 == 1) ? 130 : 40;
        Vmm a = vmm_alloc(rows_a * cols * 8);
        fill<<<4096, 256>>>(static_cast<uint64_t*>(a.ptr), rows_a * cols, 500 + r);
        CK(hipDeviceSynchronize());
        trimmed.push_back({(uintptr_t)a.ptr, (uintptr_t)a.ptr + a.bytes});
        vmm_free(a, va_free);
        uint64_t* t = nullptr;
        const uint64_t nt = 300 * cols;
        CK(hipMalloc(&t, nt * 8));
        fill_const<<<4096, 256>>>(t, nt, kPattern);
        const uint64_t nx = 130 * cols;
        Vmm x = vmm_alloc(nx * 8);
        bool reused = false;
        for (auto& p : trimmed)
            reused |= p.first < (uintptr_t)x.ptr + x.bytes && (uintptr_t)x.ptr < p.second;
        uint64_t* ref = nullptr;
        CK(hipMalloc(&ref, nx * 8));
        fill<<<4096, 256>>>(static_cast<uint64_t*>(x.ptr), nx, 600 + r);
        fill<<<4096, 256>>>(ref, nx, 600 + r);
        CK(hipDeviceSynchronize());
        unsigned long long d[3], z[2];
        for (auto& v : d) v = ne(static_cast<uint64_t*>(x.ptr), ref, nx);
        for (auto& v : z) v = eq(static_cast<uint64_t*>(x.ptr), nx, 0);
        const unsigned long long tchg = nt - eq(t, nt, kPattern);
        const bool ok = !d[0] && !d[1] && !d[2] && !z[0] && !z[1] && !tchg;
        bad += !ok;
        printf("round %d: A %llux%llu X at %p overlaps-trimmed=%d diffs=[%llu,%llu,%llu] zeros=[%llu,%llu] "
               "hipMalloc-block-changed=%llu%s\n",
               r, (unsigned long long)rows_a, (unsigned long long)cols, x.ptr, (int)reused, d[0], d[1], d[2], z[0],
               z[1], tchg, ok ? "" : "  MISMATCH");
        fflush(stdout);
        CK(hipFree(ref));
        CK(hipFree(t));
        vmm_free(x, va_free);
        trimmed.push_back({(uintptr_t)x.ptr, (uintptr_t)x.ptr + x.bytes});
    }
    printf("hbm_diag %s\n", bad ? "BAD ROUNDS" : "OK");
    return bad ? 1 : 0;
}
