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
// One workgroup moves one 16 KiB chunk of one blob.  Every lane owns 16-byte aligned DESTINATION
// quads so stores are dwordx4; the source shift (src - dst) mod 16 is the same for the whole blob,
// so the byte re-alignment is a wave-uniform switch over v_alignbyte on two dwordx4 loads (the
// second one is the neighbouring lane's first, served from the TCP).  The <16-byte head and tail
// of the chunk, where a quad is shared with the adjacent blob, are written with byte stores.
#include "kernels.h"

namespace sda {

namespace {

constexpr uint32_t kThreads = 256;
constexpr uint32_t kQuadsPerThread = 4;
constexpr uint64_t kChunk = (uint64_t)kThreads * kQuadsPerThread * 16;   // 16 KiB per workgroup

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
    // dst quads [d_lo, d_hi) (16-aligned absolute dst offsets); source byte = dst byte + shift
    for (uint32_t it = 0; it < kQuadsPerThread; ++it) {
        const uint64_t d = d_lo + ((uint64_t)it * kThreads + threadIdx.x) * 16;
        if (d >= d_hi) break;
        const uint64_t s = (uint64_t)((int64_t)d + shift);
        const u32x4* p = reinterpret_cast<const u32x4*>(src + (s & ~(uint64_t)15));
        const u32x4 a = p[0];
        u32x4 v;
        if constexpr (O == 0) {
            v = a;
        } else {
            const u32x4 b = p[1];
            v = window<O / 4, O % 4>(a, b);
        }
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + d));
    }
}

__global__ __launch_bounds__(kThreads) void snapshot_transpose_kernel(const uint8_t* __restrict__ src,
                                                                      uint8_t* __restrict__ dst,
                                                                      const SnapshotCopy* __restrict__ blobs,
                                                                      const uint32_t* __restrict__ block_blob,
                                                                      const uint32_t* __restrict__ block_chunk) {
    const SnapshotCopy c = blobs[block_blob[blockIdx.x]];
    const uint64_t c0 = (uint64_t)block_chunk[blockIdx.x] * kChunk;
    const uint64_t c1 = c0 + kChunk < c.len ? c0 + kChunk : c.len;
    const uint64_t a = c.dst + c0, e = c.dst + c1;            // absolute dst byte range of this chunk
    const int64_t shift = (int64_t)c.src - (int64_t)c.dst;
    uint64_t A = (a + 15) & ~(uint64_t)15, E = e & ~(uint64_t)15;
    if (A > E) A = E = e;                                      // chunk inside one quad: all bytes
    // head [a, A) and tail [E, e): < 16 bytes each, byte stores (quads shared with neighbouring blobs)
    const uint32_t t = threadIdx.x;
    if (t < 16 && a + t < A) dst[a + t] = src[(uint64_t)((int64_t)(a + t) + shift)];
    if (t >= 32 && t < 48 && E + (t - 32) < e && E + (t - 32) >= A)
        dst[E + (t - 32)] = src[(uint64_t)((int64_t)(E + (t - 32)) + shift)];
    if (A >= E) return;
    switch ((uint32_t)((uint64_t)shift & 15)) {               // uniform over the workgroup
#define SDA_CASE(O) case O: copy_body<O>(src, dst, A, E, shift); break;
        SDA_CASE(0) SDA_CASE(1) SDA_CASE(2) SDA_CASE(3) SDA_CASE(4) SDA_CASE(5) SDA_CASE(6) SDA_CASE(7)
        SDA_CASE(8) SDA_CASE(9) SDA_CASE(10) SDA_CASE(11) SDA_CASE(12) SDA_CASE(13) SDA_CASE(14) SDA_CASE(15)
#undef SDA_CASE
    }
}

}  // namespace

uint64_t snapshot_chunk_bytes() { return kChunk; }

hipError_t launch_snapshot_transpose(const uint8_t* src, uint8_t* dst, const SnapshotCopy* blobs,
                                     const uint32_t* block_blob, const uint32_t* block_chunk, uint64_t n_blocks,
                                     hipStream_t s) {
    // grid.x is limited to 2^31-1 workgroups; one launch per 2^30 chunks (16 PiB) is never split in practice
    const uint64_t per = (uint64_t)1 << 30;
    for (uint64_t b = 0; b < n_blocks; b += per) {
        const uint64_t g = n_blocks - b < per ? n_blocks - b : per;
        snapshot_transpose_kernel<<<dim3((uint32_t)g), dim3(kThreads), 0, s>>>(src, dst, blobs, block_blob + b,
                                                                              block_chunk + b);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace sda
