// elementwise.hip -- one-pass kernels of the sharing/masking traits.
//
//   additive generate  client/src/crypto/sharing/additive.rs:32-51 (+ batched.rs:19-53 scatter)
//   full mask          client/src/crypto/masking/full.rs:22-35     (s + mask) % m
//   unmask             client/src/crypto/masking/{full.rs:55-66, chacha.rs:80-91} (ms - m) % q
//   positive           client/src/receive.rs:14-20
//   synth fill         benchmark input generator (splitmix64 stream)
// All are HBM-bound streams; each lane handles one element with the generic exact `%`.
#include "kernels.h"

namespace sda {

namespace {

__global__ __launch_bounds__(256) void additive_generate_kernel(const int64_t* __restrict__ secrets, uint64_t D,
                                                                const int64_t* __restrict__ draws, uint64_t n,
                                                                int64_t* __restrict__ out, Mod64 M) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= D) return;
    int64_t last = secrets[b];
    const int64_t* r = draws + b * (n - 1);
    for (uint64_t j = 0; j + 1 < n; ++j) {
        const int64_t x = r[j];
        out[j * D + b] = x;                                            // shares[j] = draw j
        last = trem64((int64_t)((uint64_t)last - (uint64_t)x), M);     // fold: (sum - x) % m
    }
    out[(n - 1) * D + b] = last;
}

__global__ __launch_bounds__(256) void addsub_trem_kernel(const int64_t* __restrict__ a,
                                                          const int64_t* __restrict__ b, int sign, uint64_t D,
                                                          int64_t* __restrict__ out, Mod64 M) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= D) return;
    const uint64_t x = sign > 0 ? (uint64_t)a[i] + (uint64_t)b[i] : (uint64_t)a[i] - (uint64_t)b[i];
    out[i] = trem64((int64_t)x, M);
}

__global__ __launch_bounds__(256) void positive_kernel(const int64_t* __restrict__ v, uint64_t D,
                                                       int64_t* __restrict__ out, int64_t m) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= D) return;
    const int64_t x = v[i];
    out[i] = x < 0 ? (int64_t)((uint64_t)x + (uint64_t)m) : x;
}

// recipient epilogue (receive.rs:149-157 + :14-20): out = positive((ms - mask) % q) in one pass;
// mask == nullptr (None masking, none.rs:28-32) skips the unmask, pos_m == 0 skips positive().
__global__ __launch_bounds__(256) void unmask_positive_kernel(const int64_t* __restrict__ ms,
                                                              const int64_t* __restrict__ mask, uint64_t D,
                                                              Mod64 Q, int64_t pos_m, int64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= D) return;
    int64_t x = ms[i];
    if (mask) x = trem64((int64_t)((uint64_t)x - (uint64_t)mask[i]), Q);
    if (pos_m && x < 0) x = (int64_t)((uint64_t)x + (uint64_t)pos_m);
    out[i] = x;
}

__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_fill_kernel(int64_t* __restrict__ dst, uint64_t total,
                                                         uint64_t seed, int64_t lo, Mod64 R) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const uint64_t z = splitmix64_at(seed, i);
        dst[i] = (int64_t)((uint64_t)lo + umod64(z, R));
    }
}

inline unsigned grid_for(uint64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

hipError_t launch_additive_generate(const int64_t* secrets, uint64_t D, const int64_t* draws,
                                    uint64_t n, int64_t* out, int64_t modulus, hipStream_t s) {
    if (D == 0) return hipSuccess;
    hipLaunchKernelGGL(additive_generate_kernel, dim3(grid_for(D)), dim3(256), 0, s, secrets, D, draws, n, out,
                       make_mod64(modulus));
    return hipGetLastError();
}

hipError_t launch_addsub_trem(const int64_t* a, const int64_t* b, int sign, uint64_t D, int64_t* out,
                              int64_t modulus, hipStream_t s) {
    if (D == 0) return hipSuccess;
    hipLaunchKernelGGL(addsub_trem_kernel, dim3(grid_for(D)), dim3(256), 0, s, a, b, sign, D, out,
                       make_mod64(modulus));
    return hipGetLastError();
}

hipError_t launch_positive(const int64_t* v, uint64_t D, int64_t* out, int64_t modulus, hipStream_t s) {
    if (D == 0) return hipSuccess;
    hipLaunchKernelGGL(positive_kernel, dim3(grid_for(D)), dim3(256), 0, s, v, D, out, modulus);
    return hipGetLastError();
}

hipError_t launch_unmask_positive(const int64_t* ms, const int64_t* mask, uint64_t D, int64_t q, int64_t pos_m,
                                  int64_t* out, hipStream_t s) {
    if (D == 0) return hipSuccess;
    hipLaunchKernelGGL(unmask_positive_kernel, dim3(grid_for(D)), dim3(256), 0, s, ms, mask, D,
                       make_mod64(q > 0 ? q : 1), pos_m, out);
    return hipGetLastError();
}

hipError_t launch_synth_fill(int64_t* dst, uint64_t rows, uint64_t cols, uint64_t seed, int64_t lo,
                             int64_t hi, hipStream_t s) {
    const uint64_t total = rows * cols;
    if (total == 0) return hipSuccess;
    const uint64_t range = (uint64_t)hi - (uint64_t)lo;
    Mod64 R;
    R.m = range;
    R.mu = range > 1 ? UINT64_MAX / range : 0;
    const uint64_t blocks = total / 256 + 1;
    hipLaunchKernelGGL(synth_fill_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s,
                       dst, total, seed, lo, R);
    return hipGetLastError();
}

}  // namespace sda
