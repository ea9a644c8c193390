// combine.hip -- north-star kernel (1): exact clerk share-combine on gfx950.
//
// Reference: client/src/crypto/sharing/combiner.rs:16-28
//     for share in shares { for (ix, value) in share { result[ix] += value; result[ix] %= m } }
// The recurrence is sequential along the participation axis and independent across columns,
// so one lane owns VEC adjacent columns and walks all n rows in reference order: the signed,
// order-dependent result of Rust's truncated `%` is reproduced bit for bit, and the matrix
// is still read exactly once with fully coalesced loads (a wave reads 64 * VEC * 8 contiguous
// bytes of one row per instruction).  UNROLL rows are loaded before the dependent chain so
// every lane keeps UNROLL * VEC * 8 bytes in flight; with ~30 waves per CU that covers HBM
// latency.  Non-temporal loads keep the once-read stream from thrashing L2/MALL.
//
// Roofline: HBM.  Algorithmic bytes per launch = 8 * n * dim (read) + 8 * dim (write)
// (4 * n * dim read for the int32 rows of the clerk's decode -> combine).
#include <stdlib.h>

#include "kernels.h"

namespace sda {

namespace {

template <typename T, int VEC> struct vec_t { typedef T type __attribute__((ext_vector_type(VEC))); };
template <typename T> struct vec_t<T, 1> { typedef T type; };

template <typename T, int VEC>
__device__ __forceinline__ int64_t lane_of(const typename vec_t<T, VEC>::type& v, int e) {
    if constexpr (VEC == 1) { return (int64_t)v; } else { return (int64_t)v[e]; }
}

// ACC: continue the recurrence from `out` (a previous combine result, |r| < m) instead of 0 --
// a clerk job streamed through HBM in row tiles is bit-identical to one pass over all rows.
// T: the row element type -- int64_t (the ABI's shares), or int32_t for decoded field shares
// (the clerk's decode -> combine, whose payload values fit: half the bytes to read).
template <typename T, int VEC, int UNROLL, bool SMALL_M, bool ACC>
__global__ __launch_bounds__(256) void combine_exact_kernel(const T* __restrict__ in,
                                                            uint64_t n, uint64_t n_lanes,
                                                            uint64_t stride,
                                                            int64_t* __restrict__ out, Mod64 M) {
    typedef typename vec_t<T, VEC>::type V;
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= n_lanes) return;
    const V* p = reinterpret_cast<const V*>(in + lane * VEC);
    const uint64_t vstride = stride / VEC;     // stride in units of V (host guarantees divisibility)
    int64_t r[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) r[e] = ACC ? out[lane * VEC + e] : 0;

    uint64_t i = 0;
    for (; i + UNROLL <= n; i += UNROLL) {
        V v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(p + (uint64_t)u * vstride);
        p += (uint64_t)UNROLL * vstride;
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int e = 0; e < VEC; ++e) r[e] = add_trem(r[e], lane_of<T, VEC>(v[u], e), M, SMALL_M);
    }
    for (; i < n; ++i) {
        V v = __builtin_nontemporal_load(p);
        p += vstride;
#pragma unroll
        for (int e = 0; e < VEC; ++e) r[e] = add_trem(r[e], lane_of<T, VEC>(v, e), M, SMALL_M);
    }
    typedef typename vec_t<int64_t, VEC>::type VO;
    VO o;
    if constexpr (VEC == 1) { o = r[0]; } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) o[e] = r[e];
    }
    reinterpret_cast<VO*>(out)[lane] = o;
}

template <typename T, int VEC, int UNROLL, bool ACC>
hipError_t launch_vec(const T* in, uint64_t n, uint64_t dim, uint64_t stride, int64_t* out,
                      const Mod64& M, bool small_m, hipStream_t s) {
    const uint64_t n_lanes = dim / VEC;
    const uint64_t blocks = (n_lanes + 255) / 256;
    if (small_m)
        hipLaunchKernelGGL((combine_exact_kernel<T, VEC, UNROLL, true, ACC>), dim3((unsigned)blocks), dim3(256), 0, s,
                           in, n, n_lanes, stride, out, M);
    else
        hipLaunchKernelGGL((combine_exact_kernel<T, VEC, UNROLL, false, ACC>), dim3((unsigned)blocks), dim3(256), 0, s,
                           in, n, n_lanes, stride, out, M);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void mod_canonical_kernel(const int64_t* __restrict__ sums, uint64_t dim,
                                                            int64_t* __restrict__ out, Mod64 M) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < dim) out[i] = (int64_t)umod64((uint64_t)sums[i], M);
}

}  // namespace

hipError_t launch_combine_exact(const int64_t* in, uint64_t n, uint64_t dim, uint64_t stride,
                                int64_t* out, int64_t modulus, hipStream_t s, bool accumulate) {
    if (dim == 0) return hipSuccess;
    const Mod64 M = make_mod64(modulus);
    const bool small_m = modulus <= ((int64_t)1 << 62);
    const uintptr_t a = (uintptr_t)in | (uintptr_t)out;
    // widest vector whose columns, row stride and base addresses all line up
    const bool v2 = dim % 2 == 0 && stride % 2 == 0 && (a % 16) == 0;
    if (accumulate)
        return v2 ? launch_vec<int64_t, 2, 8, true>(in, n, dim, stride, out, M, small_m, s)
                  : launch_vec<int64_t, 1, 8, true>(in, n, dim, stride, out, M, small_m, s);
    return v2 ? launch_vec<int64_t, 2, 8, false>(in, n, dim, stride, out, M, small_m, s)
              : launch_vec<int64_t, 1, 8, false>(in, n, dim, stride, out, M, small_m, s);
}

hipError_t launch_combine_exact32(const int32_t* in, uint64_t n, uint64_t dim, uint64_t stride,
                                  int64_t* out, int64_t modulus, hipStream_t s) {
    if (dim == 0) return hipSuccess;
    const Mod64 M = make_mod64(modulus);
    const bool small_m = modulus <= ((int64_t)1 << 62);
    // 2 columns per lane (8-byte loads: the i64 kernel's grid) or, with SDA_COMBINE32_VEC=4 (A/B knob),
    // 4 (16-byte loads, half the lanes)
    const char* env = getenv("SDA_COMBINE32_VEC");
    const bool want4 = env && atoi(env) == 4;
    const uintptr_t a = (uintptr_t)in, o = (uintptr_t)out;
    if (want4 && dim % 4 == 0 && stride % 4 == 0 && a % 16 == 0 && o % 32 == 0)
        return launch_vec<int32_t, 4, 8, false>(in, n, dim, stride, out, M, small_m, s);
    const bool v2 = dim % 2 == 0 && stride % 2 == 0 && a % 8 == 0 && o % 16 == 0;
    return v2 ? launch_vec<int32_t, 2, 8, false>(in, n, dim, stride, out, M, small_m, s)
              : launch_vec<int32_t, 1, 8, false>(in, n, dim, stride, out, M, small_m, s);
}

hipError_t launch_mod_canonical(const int64_t* sums, uint64_t dim, int64_t* out, int64_t modulus,
                                hipStream_t s) {
    if (dim == 0) return hipSuccess;
    const Mod64 M = make_mod64(modulus);
    hipLaunchKernelGGL(mod_canonical_kernel, dim3((unsigned)((dim + 255) / 256)), dim3(256), 0, s,
                       sums, dim, out, M);
    return hipGetLastError();
}

}  // namespace sda
