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
// latency.  The i64 kernels are software-pipelined (PIPE: the next 4 rows load while the current 4
// rows' chain runs), so a wave never sits computing with nothing in flight.  Non-temporal loads keep
// the once-read stream from thrashing L2/MALL.
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
// FLAG (pass 1 of the multi-GPU participation split): also raise flags[0] when an input
// is negative (the ranks' canonical sums then lose the sign the reference's order gives: the split
// runs its replay pass) and flags[1] when an input lies outside [-(2^63 - m), 2^63 - m] (the
// reference's `r + v` may wrap i64 there, which no split can reproduce).  One OR of the high word per
// element (plus a 64-bit range check); every writer stores the same 1, so plain stores suffice.
// PIPE (the i64 default since round 6; SDA_COMBINE_PIPE=0 turns it off): software-pipelined -- the next UNROLL
// rows are loaded before the current UNROLL rows' dependent chain runs, so a wave keeps loads in flight while it
// computes (two register buffers).
template <typename T, int VEC, int UNROLL, bool SMALL_M, bool ACC, bool FLAG = false, bool PIPE = false>
__global__ __launch_bounds__(256) void combine_exact_kernel(const T* __restrict__ in,
                                                            uint64_t n, uint64_t n_lanes,
                                                            uint64_t stride,
                                                            int64_t* __restrict__ out, Mod64 M,
                                                            int64_t* __restrict__ flags = nullptr,
                                                            uint32_t wlo = 0, uint32_t nwide = 0) {
    typedef typename vec_t<T, VEC>::type V;
    // (natural workgroup order: the XCD-chunked order of xcd.h measured neutral here, profiles/r04b)
    // wlo > 0: balanced grid (combine_grid) -- workgroup g owns wlo lanes (+ 8 for the first nwide workgroups),
    // starting at g wlo + 8 min(g, nwide): multiples of 8 lanes, so every wave segment stays 128-byte aligned
    uint64_t lane;
    if (wlo) {
        const uint64_t g = blockIdx.x;
        const uint32_t width = wlo + (g < nwide ? 8u : 0u);
        if (threadIdx.x >= width) return;
        lane = g * wlo + 8 * (g < nwide ? g : (uint64_t)nwide) + threadIdx.x;
    } else {
        lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    }
    if (lane >= n_lanes) return;
    const V* p = reinterpret_cast<const V*>(in + lane * VEC);
    const uint64_t vstride = stride / VEC;     // stride in units of V (host guarantees divisibility)
    int64_t r[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) r[e] = ACC ? out[lane * VEC + e] : 0;

    uint32_t neg = 0, risk = 0;
    const uint64_t lim = ((uint64_t)1 << 63) - M.m;        // no-wrap range [-lim, lim]
    auto step = [&](int e, int64_t x) {
        r[e] = add_trem(r[e], x, M, SMALL_M);
        if constexpr (FLAG) {
            neg |= hi32(x);
            risk |= (uint32_t)((uint64_t)x + lim > 2 * lim);
        }
    };
    uint64_t i = 0;
    if constexpr (PIPE) {
        // a buffer's loads are issued on every path that reaches its chain, and the last whole batch is peeled
        // off: a load on one side of a branch makes the compiler's counter merge wait for it before the other
        // buffer's use
        const uint64_t full = n - n % UNROLL;           // rows in whole batches (uniform)
        const V* p0 = p;
        V a[UNROLL], b[UNROLL];
        auto load = [&](V (&x)[UNROLL], uint64_t r0) {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) x[u] = __builtin_nontemporal_load(p0 + (r0 + u) * vstride);
        };
        auto chain = [&](const V (&x)[UNROLL]) {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
#pragma unroll
                for (int e = 0; e < VEC; ++e) step(e, lane_of<T, VEC>(x[u], e));
        };
        if (full) {
            load(a, 0);
            for (uint64_t j = 0;; j += 2 * UNROLL) {        // a holds rows j.., in flight
                if (j + UNROLL == full) { chain(a); break; }
                load(b, j + UNROLL);
                chain(a);
                if (j + 2 * UNROLL == full) { chain(b); break; }
                load(a, j + 2 * UNROLL);
                chain(b);
            }
        }
        i = full;
        p = p0 + full * vstride;
    } else {
        for (; i + UNROLL <= n; i += UNROLL) {
            V v[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(p + (uint64_t)u * vstride);
            p += (uint64_t)UNROLL * vstride;
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
#pragma unroll
                for (int e = 0; e < VEC; ++e) step(e, lane_of<T, VEC>(v[u], e));
        }
    }
    for (; i < n; ++i) {
        V v = __builtin_nontemporal_load(p);
        p += vstride;
#pragma unroll
        for (int e = 0; e < VEC; ++e) step(e, lane_of<T, VEC>(v, e));
    }
    if constexpr (FLAG) {
        if ((int32_t)neg < 0) flags[0] = 1;
        if (risk) flags[1] = 1;
    }
    typedef typename vec_t<int64_t, VEC>::type VO;
    VO o;
    if constexpr (VEC == 1) { o = r[0]; } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) o[e] = r[e];
    }
    reinterpret_cast<VO*>(out)[lane] = o;
}

// Balanced grid (the pipelined kernels' default; SDA_COMBINE_BALANCE=0 is the A/B knob): the grid is whole rounds
// of resident workgroups and every workgroup holds (nearly) the same number of lanes, so each CU has the same work
// to the end.  The plain grid of 256-lane workgroups left 1,954 workgroups for configs[1]'s 1M columns on 2,048
// slots: 162 CUs ran 8 of them, 94 ran 7 and idled for the last eighth.  In one process, interleaved
// (scripts/combine_pipe_inproc.py, profiles/r06w): 12.770 -> 12.563 ms per configs[1] launch, 13.050 -> 12.760 ms
// per configs[3] 1000 x 10M tile; bit-identical.
bool combine_balance() {
    const char* e = getenv("SDA_COMBINE_BALANCE");
    return !(e && e[0] == '0');
}

// The balanced grid of a kernel: G = whole rounds of (CUs x resident workgroups per CU) workgroups, the lanes
// split as G wlo + 8 nwide (wlo a multiple of 8, at most 248).  false when the job is too small to fill a round.
// (per_cu: the kernel's resident 256-lane workgroups per CU, queried once per instantiation by the caller; the
// smallest jobs -- below 64 lanes per slot of a 256-CU part -- skip the device queries altogether)
bool combine_grid(int per_cu, uint64_t n_lanes, uint64_t* G, uint32_t* wlo, uint32_t* nwide) {
    if (per_cu <= 0 || n_lanes < (uint64_t)per_cu * 256 * 64) return false;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return false;
    const uint64_t slots = (uint64_t)cus * (uint64_t)per_cu;
    if (n_lanes < slots * 64) return false;
    const uint64_t rounds = (n_lanes + slots * 256 - 1) / (slots * 256);
    const uint64_t g = slots * rounds;
    uint64_t lo = n_lanes / g / 8 * 8;
    if (lo > 248) lo = 248;
    const uint64_t wide = (n_lanes - g * lo + 7) / 8;
    if (lo == 0 || wide > g) return false;
    *G = g;
    *wlo = (uint32_t)lo;
    *nwide = (uint32_t)wide;
    return g <= 0x7FFFFFFFull;
}

template <typename T, int VEC, int UNROLL, bool ACC, bool FLAG = false, bool PIPE = false>
hipError_t launch_vec(const T* in, uint64_t n, uint64_t dim, uint64_t stride, int64_t* out,
                      const Mod64& M, bool small_m, hipStream_t s, int64_t* flags = nullptr) {
    const uint64_t n_lanes = dim / VEC;
    uint64_t blocks = (n_lanes + 255) / 256;
    uint32_t wlo = 0, nwide = 0;
    if (PIPE && combine_balance()) {
        // resident workgroups per CU of this instantiation (the same on every MI355X): queried once
        static const int per_cu_small = [] {
            int v = 0;
            return hipOccupancyMaxActiveBlocksPerMultiprocessor(
                       &v, reinterpret_cast<const void*>(combine_exact_kernel<T, VEC, UNROLL, true, ACC, FLAG, PIPE>),
                       256, 0) == hipSuccess ? v : 0;
        }();
        static const int per_cu_big = [] {
            int v = 0;
            return hipOccupancyMaxActiveBlocksPerMultiprocessor(
                       &v, reinterpret_cast<const void*>(combine_exact_kernel<T, VEC, UNROLL, false, ACC, FLAG, PIPE>),
                       256, 0) == hipSuccess ? v : 0;
        }();
        uint64_t g;
        if (combine_grid(small_m ? per_cu_small : per_cu_big, n_lanes, &g, &wlo, &nwide)) blocks = g;
        else wlo = nwide = 0;
    }
    if (small_m)
        hipLaunchKernelGGL((combine_exact_kernel<T, VEC, UNROLL, true, ACC, FLAG, PIPE>), dim3((unsigned)blocks),
                           dim3(256), 0, s, in, n, n_lanes, stride, out, M, flags, wlo, nwide);
    else
        hipLaunchKernelGGL((combine_exact_kernel<T, VEC, UNROLL, false, ACC, FLAG, PIPE>), dim3((unsigned)blocks),
                           dim3(256), 0, s, in, n, n_lanes, stride, out, M, flags, wlo, nwide);
    return hipGetLastError();
}

// The i64 kernels run software-pipelined, two buffers of 4 rows (PIPE): one process, one 80 GB buffer, the
// variants interleaved (scripts/combine_pipe_inproc.py, profiles/r06m): 12.298 ms unpipelined (8 rows per
// batch), 12.134 ms pipelined at 4 rows, 12.175 at 6, 12.192 at 2; bit-identical.  SDA_COMBINE_PIPE=0 (A/B
// knob) launches the unpipelined kernel.
bool combine_pipe() {
    const char* e = getenv("SDA_COMBINE_PIPE");
    return !(e && e[0] == '0');
}

// canonical residue in [0, m) of a signed i64 value
__device__ __forceinline__ int64_t canon64(int64_t v, const Mod64& M) {
    const int64_t r = trem64(v, M);
    return r < 0 ? r + (int64_t)M.m : r;
}

// Multi-GPU finalize: the all-reduced int64 sums of the ranks' results (|sum| <= G (m - 1) <= 2^63 - 1,
// checked on the host), signed when the ranks' results were -> their canonical residue.
__global__ __launch_bounds__(256) void mod_canonical_kernel(const int64_t* __restrict__ sums, uint64_t dim,
                                                            int64_t* __restrict__ out, Mod64 M) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < dim) out[i] = canon64(sums[i], M);
}

// ---- signed participation split, pass 2 (DESIGN.md §5 "signed inputs") ----
// Keep the reference's running value as r = c - m s: c its canonical residue, s = [r < 0] (s = 1 needs
// c != 0).  One step r' = (r + v) % m (no i64 wrap: pass 1 refused such v) gives c' = (c + v) mod m and
//   v >= 0:  s' = s AND [c + v < m]                  -> "reset" when c + v >= m, else no event
//   v <  0:  s' = (s OR [c + v < 0]) AND [c' != 0]   -> "reset" when c' = 0, "set" when c + v < 0,
//                                                       else no event
// so, given c at the chunk's start, every step maps s to s, to 0 or to 1, and a chunk of rows maps it
// through its LAST event.  The chunk's c trajectory needs only the incoming residue c_in (the other
// ranks' pass-1 sums), never s: this pass replays it and records the last event as a code that an
// all-reduce MAX over the ranks resolves in participation order -- 0 none, 2g+1 reset, 2g+2 set (g = the
// rank).  A step with c' = 0 always leaves s' = 0, so it may be called a reset whatever the sign of v.
template <int VEC, int UNROLL, bool SMALL_M>
__global__ __launch_bounds__(256) void combine_replay_kernel(const int64_t* __restrict__ in, uint64_t n,
                                                             uint64_t n_lanes, uint64_t stride,
                                                             int64_t* __restrict__ state, int32_t* __restrict__ code,
                                                             int32_t reset_code, Mod64 M) {
    typedef typename vec_t<int64_t, VEC>::type V;
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= n_lanes) return;
    const V* p = reinterpret_cast<const V*>(in + lane * VEC);
    const uint64_t vstride = stride / VEC;
    const int64_t m = (int64_t)M.m;
    int64_t c[VEC];
    int32_t cd[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
        c[e] = state[lane * VEC + e];
        cd[e] = code[lane * VEC + e];
    }
    auto step = [&](int e, int64_t v) {
        int64_t cn;
        bool hi, lo;
        if (SMALL_M && ((uint64_t)v + (uint64_t)(m - 1) < (uint64_t)(2 * m - 1))) {   // v in (-m, m)
            const int64_t t = c[e] + v;                  // (-m, 2m)
            hi = t >= m;
            lo = t < 0;
            cn = hi ? t - m : (lo ? t + m : t);
        } else {                                         // any v, any m: exact unsigned forms
            const uint64_t uc = (uint64_t)c[e];
            const uint64_t mag = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
            const uint64_t rr = umod64(mag, M);
            const uint64_t vr = (v < 0 && rr) ? M.m - rr : rr;              // v mod m, canonical
            const uint64_t sum = uc + vr;                                   // < 2m < 2^64
            cn = (int64_t)(sum >= M.m ? sum - M.m : sum);
            hi = v >= 0 && mag >= M.m - uc;              // c + v >= m
            lo = v < 0 && mag > uc;                      // c + v < 0
        }
        c[e] = cn;
        cd[e] = (cn == 0 || hi) ? reset_code : (lo ? reset_code + 1 : cd[e]);
    };
    uint64_t i = 0;
    for (; i + UNROLL <= n; i += UNROLL) {
        V v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(p + (uint64_t)u * vstride);
        p += (uint64_t)UNROLL * vstride;
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int e = 0; e < VEC; ++e) step(e, lane_of<int64_t, VEC>(v[u], e));
    }
    for (; i < n; ++i) {
        V v = __builtin_nontemporal_load(p);
        p += vstride;
#pragma unroll
        for (int e = 0; e < VEC; ++e) step(e, lane_of<int64_t, VEC>(v, e));
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
        state[lane * VEC + e] = c[e];
        code[lane * VEC + e] = cd[e];
    }
}

// gathered [world][dim] = every rank's pass-1 result: c_in = canonical(sum over ranks < rank),
// total = canonical(sum over all ranks); code = rank 0's own sign (its pass 1 started at the job's
// start, r = 0): 1 + [r_0 < 0], else 0 (no event yet).  |partial sums| <= world (m - 1) <= 2^63 - 1.
__global__ __launch_bounds__(256) void split_prefix_kernel(const int64_t* __restrict__ gathered, uint64_t world,
                                                           uint64_t rank, uint64_t dim, int64_t* __restrict__ c_in,
                                                           int64_t* __restrict__ total, int32_t* __restrict__ code,
                                                           Mod64 M) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= dim) return;
    int64_t before = 0, all = 0;
    for (uint64_t g = 0; g < world; ++g) {
        const int64_t v = gathered[g * dim + i];
        if (g < rank) before += v;
        all += v;
    }
    c_in[i] = canon64(before, M);
    total[i] = canon64(all, M);
    code[i] = rank == 0 ? 1 + (gathered[i] < 0) : 0;
}

// out = the reference's signed result: total - m when the last sign event (MAX-reduced code) set s.
__global__ __launch_bounds__(256) void split_resolve_kernel(const int64_t* __restrict__ total,
                                                            const int32_t* __restrict__ code, uint64_t dim,
                                                            int64_t* __restrict__ out, int64_t m) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= dim) return;
    const bool neg = ((code[i] - 1) & 1) != 0;
    out[i] = total[i] - (neg ? m : 0);
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
    const bool pipe = v2 && combine_pipe();
    if (accumulate) {
        if (pipe) return launch_vec<int64_t, 2, 4, true, false, true>(in, n, dim, stride, out, M, small_m, s);
        return v2 ? launch_vec<int64_t, 2, 8, true>(in, n, dim, stride, out, M, small_m, s)
                  : launch_vec<int64_t, 1, 8, true>(in, n, dim, stride, out, M, small_m, s);
    }
    if (pipe) return launch_vec<int64_t, 2, 4, false, false, true>(in, n, dim, stride, out, M, small_m, s);
    return v2 ? launch_vec<int64_t, 2, 8, false>(in, n, dim, stride, out, M, small_m, s)
              : launch_vec<int64_t, 1, 8, false>(in, n, dim, stride, out, M, small_m, s);
}

hipError_t launch_combine_split(const int64_t* in, uint64_t n, uint64_t dim, uint64_t stride, int64_t* inout,
                                int64_t modulus, int64_t* flags, hipStream_t s) {
    if (dim == 0 || n == 0) return hipSuccess;
    const Mod64 M = make_mod64(modulus);
    const bool small_m = modulus <= ((int64_t)1 << 62);
    const uintptr_t a = (uintptr_t)in | (uintptr_t)inout;
    const bool v2 = dim % 2 == 0 && stride % 2 == 0 && (a % 16) == 0;
    if (v2 && combine_pipe())
        return launch_vec<int64_t, 2, 4, true, true, true>(in, n, dim, stride, inout, M, small_m, s, flags);
    return v2 ? launch_vec<int64_t, 2, 8, true, true>(in, n, dim, stride, inout, M, small_m, s, flags)
              : launch_vec<int64_t, 1, 8, true, true>(in, n, dim, stride, inout, M, small_m, s, flags);
}

hipError_t launch_combine_replay(const int64_t* in, uint64_t n, uint64_t dim, uint64_t stride, int64_t* state,
                                 int32_t* code, int32_t reset_code, int64_t modulus, hipStream_t s) {
    if (dim == 0 || n == 0) return hipSuccess;
    const Mod64 M = make_mod64(modulus);
    const bool small_m = modulus <= ((int64_t)1 << 62);
    const uintptr_t a = (uintptr_t)in | (uintptr_t)state;
    const bool v2 = dim % 2 == 0 && stride % 2 == 0 && (a % 16) == 0 && (uintptr_t)code % 8 == 0;
    const int vec = v2 ? 2 : 1;
    const uint64_t n_lanes = dim / vec;
    const dim3 grid((unsigned)((n_lanes + 255) / 256));
    if (v2) {
        if (small_m) hipLaunchKernelGGL((combine_replay_kernel<2, 8, true>), grid, dim3(256), 0, s, in, n, n_lanes, stride, state, code, reset_code, M);
        else hipLaunchKernelGGL((combine_replay_kernel<2, 8, false>), grid, dim3(256), 0, s, in, n, n_lanes, stride, state, code, reset_code, M);
    } else {
        if (small_m) hipLaunchKernelGGL((combine_replay_kernel<1, 8, true>), grid, dim3(256), 0, s, in, n, n_lanes, stride, state, code, reset_code, M);
        else hipLaunchKernelGGL((combine_replay_kernel<1, 8, false>), grid, dim3(256), 0, s, in, n, n_lanes, stride, state, code, reset_code, M);
    }
    return hipGetLastError();
}

hipError_t launch_split_prefix(const int64_t* gathered, uint64_t world, uint64_t rank, uint64_t dim, int64_t* c_in,
                               int64_t* total, int32_t* code, int64_t modulus, hipStream_t s) {
    if (dim == 0) return hipSuccess;
    hipLaunchKernelGGL(split_prefix_kernel, dim3((unsigned)((dim + 255) / 256)), dim3(256), 0, s, gathered, world,
                       rank, dim, c_in, total, code, make_mod64(modulus));
    return hipGetLastError();
}

hipError_t launch_split_resolve(const int64_t* total, const int32_t* code, uint64_t dim, int64_t* out,
                                int64_t modulus, hipStream_t s) {
    if (dim == 0) return hipSuccess;
    hipLaunchKernelGGL(split_resolve_kernel, dim3((unsigned)((dim + 255) / 256)), dim3(256), 0, s, total, code, dim,
                       out, modulus);
    return hipGetLastError();
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
