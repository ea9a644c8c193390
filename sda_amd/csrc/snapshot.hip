// snapshot.hip -- snapshot transposition.
//
//   server/src/stores.rs:86-101  AggregationsStore::iter_snapshot_clerk_jobs_data
//     for participation in snapshot order: for (ix, share) in clerk_encryptions: shares[ix].push(share)
//   (server-store-mongodb/src/aggregations.rs:164-195 computes the same grouping with $unwind/$group.)
//
// The snapshot arrives as P participations, each with n clerk payloads back to back
// ([participation][clerk] ragged byte blobs); the clerking jobs want [clerk][participation].
// This is a ragged byte gather: HBM-bound, 2 bytes of traffic per payload byte.
//
// Blobs are cut into 32 KiB chunks; a workgroup moves a contiguous run of 4 of them.  Every lane owns
// 16-byte aligned DESTINATION quads so stores are dwordx4.  The source shift (src - dst) mod 16 is
// uniform per blob: shift 0 takes aligned dwordx4 loads; any other shift takes one unaligned dwordx4
// load per quad (gfx950 runs with unaligned access mode, so the hardware splits the line crossing).
// A/B (profiles/r01h/ab_snapshot.txt): unaligned 7.25 ms vs 7.57 ms for two aligned loads + a
// uniform switch over v_alignbyte (SDA_SNAP_UNALIGNED=0); with 4-chunk workgroups 6.5-6.8 ms for
// 16 GB, the same rate as a same-size device-to-device copy.
// All loads of a chunk are issued before its stores.  The <16-byte head and tail of a chunk, whose
// quad is shared with the neighbouring blob, are written with byte stores.
#include "kernels.h"

namespace sda {

namespace {

constexpr uint32_t kThreads = 256;
#ifndef SDA_SNAP_UNALIGNED
#define SDA_SNAP_UNALIGNED 1
#endif
#ifndef SDA_SNAP_NT_LOAD
#define SDA_SNAP_NT_LOAD 0
#endif
#ifndef SDA_SNAP_CHUNKS_PER_WG
#define SDA_SNAP_CHUNKS_PER_WG 4
#endif
#ifndef SDA_SNAP_QUADS
#define SDA_SNAP_QUADS 8
#endif
constexpr uint32_t kQuadsPerThread = SDA_SNAP_QUADS;
constexpr uint64_t kChunk = (uint64_t)kThreads * kQuadsPerThread * 16;   // 32 KiB per workgroup

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// out dword j of a 16-byte window starting at byte o of the 32-byte pair (a, b)
template <int Q, int R>
__device__ __forceinline__ u32x4 window(const u32x4& a, const u32x4& b) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    u32x4 r;
    if constexpr (R == 0) {
        r.x = w[Q]; r.y = w[Q + 1]; r.z = w[Q + 2]; r.w = w[Q + 3];
    } else {
        r.x = __builtin_amdgcn_alignbyte(w[Q + 1], w[Q], R);
        r.y = __builtin_amdgcn_alignbyte(w[Q + 2], w[Q + 1], R);
        r.z = __builtin_amdgcn_alignbyte(w[Q + 3], w[Q + 2], R);
        r.w = __builtin_amdgcn_alignbyte(w[Q + 4], w[Q + 3], R);
    }
    return r;
}

template <int O>
__device__ __forceinline__ void copy_body(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                          uint64_t d_lo, uint64_t d_hi, int64_t shift) {
    // dst quads [d_lo, d_hi) (16-aligned absolute dst offsets); source byte = dst byte + shift.
    // All loads of the chunk are issued before the first store (kQuadsPerThread x 32 B in flight per lane).
    u32x4 v[kQuadsPerThread];
#pragma unroll
    for (uint32_t it = 0; it < kQuadsPerThread; ++it) {
        const uint64_t d = d_lo + ((uint64_t)it * kThreads + threadIdx.x) * 16;
        if (d < d_hi) {
            const uint64_t s = (uint64_t)((int64_t)d + shift);
            const u32x4* p = reinterpret_cast<const u32x4*>(src + (s & ~(uint64_t)15));
            if constexpr (O == 0) {
                v[it] = p[0];
            } else if constexpr (SDA_SNAP_UNALIGNED && SDA_SNAP_NT_LOAD) {
                typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
                v[it] = __builtin_nontemporal_load(reinterpret_cast<const u32x4u*>(src + s));
            } else if constexpr (SDA_SNAP_UNALIGNED) {
                __builtin_memcpy(&v[it], src + s, 16);     // one unaligned dwordx4 (unaligned access mode)
            } else {
                v[it] = window<O / 4, O % 4>(p[0], p[1]);
            }
        }
    }
#pragma unroll
    for (uint32_t it = 0; it < kQuadsPerThread; ++it) {
        const uint64_t d = d_lo + ((uint64_t)it * kThreads + threadIdx.x) * 16;
        if (d < d_hi) __builtin_nontemporal_store(v[it], reinterpret_cast<u32x4*>(dst + d));
    }
}

__device__ __forceinline__ void copy_chunk(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                           const SnapshotCopy& c, uint64_t chunk) {
    const uint64_t c0 = chunk * kChunk;
    const uint64_t c1 = c0 + kChunk < c.len ? c0 + kChunk : c.len;
    const uint64_t a = c.dst + c0, e = c.dst + c1;            // absolute dst byte range of this chunk
    const int64_t shift = (int64_t)c.src - (int64_t)c.dst;
    uint64_t A = (a + 15) & ~(uint64_t)15, E = e & ~(uint64_t)15;
    if (A > E) A = E = e;                                      // chunk inside one quad: all bytes
    // head [a, A) and tail [E, e): < 16 bytes each, byte stores (quads shared with neighbouring blobs)
    const uint32_t t = threadIdx.x;
    if (t < 16 && a + t < A) dst[a + t] = src[(uint64_t)((int64_t)(a + t) + shift)];
    if (t >= 64 && t < 80 && E + (t - 64) < e) dst[E + (t - 64)] = src[(uint64_t)((int64_t)(E + (t - 64)) + shift)];
    if (A >= E) return;
    switch ((uint32_t)((uint64_t)shift & 15)) {               // uniform over the workgroup
#define SDA_CASE(O) case O: copy_body<O>(src, dst, A, E, shift); break;
        SDA_CASE(0) SDA_CASE(1) SDA_CASE(2) SDA_CASE(3) SDA_CASE(4) SDA_CASE(5) SDA_CASE(6) SDA_CASE(7)
        SDA_CASE(8) SDA_CASE(9) SDA_CASE(10) SDA_CASE(11) SDA_CASE(12) SDA_CASE(13) SDA_CASE(14) SDA_CASE(15)
#undef SDA_CASE
    }
}

// Workgroup w walks the contiguous chunk range [total*w/G, total*(w+1)/G) of the clerk-major blob
// list: one binary search over the chunk prefix for its first blob, then a forward walk, so the
// host plan is one entry per blob rather than one per chunk.
__global__ __launch_bounds__(kThreads) void snapshot_transpose_kernel(const uint8_t* __restrict__ src,
                                                                      uint8_t* __restrict__ dst,
                                                                      const SnapshotCopy* __restrict__ blobs,
                                                                      const uint64_t* __restrict__ chunk_start,
                                                                      uint64_t n_blobs, uint64_t total_chunks) {
    const uint64_t G = gridDim.x, w = blockIdx.x;
    const uint64_t lo = total_chunks * w / G, hi = total_chunks * (w + 1) / G;
    if (lo >= hi) return;
    uint64_t l = 0, r = n_blobs - 1;                           // last b with chunk_start[b] <= lo
    while (l < r) {
        const uint64_t mid = (l + r + 1) / 2;
        if (chunk_start[mid] <= lo) l = mid; else r = mid - 1;
    }
    uint64_t b = l, next = chunk_start[b + 1];
    SnapshotCopy c = blobs[b];
    for (uint64_t ch = lo; ch < hi; ++ch) {
        if (ch >= next) {                                      // every planned blob has >= 1 chunk
            ++b;
            next = chunk_start[b + 1];
            c = blobs[b];
        }
        copy_chunk(src, dst, c, ch - chunk_start[b]);
    }
}

}  // namespace

uint64_t snapshot_chunk_bytes() { return kChunk; }

hipError_t launch_snapshot_transpose(const uint8_t* src, uint8_t* dst, const SnapshotCopy* blobs,
                                     const uint64_t* chunk_start, uint64_t n_blobs, uint64_t total_chunks,
                                     hipStream_t s) {
    if (!n_blobs || !total_chunks) return hipSuccess;
    // short-lived workgroups of SDA_SNAP_CHUNKS_PER_WG chunks each: the dispatcher balances the
    // ragged tail better than long walks (A/B in profiles/r01h/ab_snapshot.txt)
    const uint64_t cpw = total_chunks / SDA_SNAP_CHUNKS_PER_WG < 0x7fffffffull
                             ? SDA_SNAP_CHUNKS_PER_WG : total_chunks / 0x7fffffffull + 1;
    const uint64_t g = (total_chunks + cpw - 1) / cpw;
    snapshot_transpose_kernel<<<dim3((uint32_t)g), dim3(kThreads), 0, s>>>(src, dst, blobs, chunk_start, n_blobs,
                                                                          total_chunks);
    return hipGetLastError();
}

}  // namespace sda
