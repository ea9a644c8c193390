// xcd.h -- XCD-aware workgroup order for the streaming kernels (gfx950: 8 XCDs, each with its own L2).
//
// The command processor hands workgroups to the XCDs round-robin in linear dispatch order, so with
// the natural order eight consecutive tiles -- adjacent 2 KiB pieces of the same HBM rows -- land on
// eight different XCDs and reach the memory controllers interleaved from eight L2s.  xcd_chunk()
// renames the linear id so that the workgroups one XCD receives walk ONE contiguous eighth of the
// grid in order.  Measured on share-gen's memory pattern (tools/ubench_gen.hip, profiles/r04a): 41 GB
// of 37 % reads / 63 % writes in [n][B] clerk rows, 5.36 TB/s natural -> 6.32 TB/s chunked.
#pragma once
#include <stdint.h>

namespace sda {

constexpr uint32_t kXcds = 8;

// Bijective on [0, total): the blocks sharing an XCD (same L % 8) get consecutive ids.
__device__ __forceinline__ uint64_t xcd_chunk(uint64_t L, uint64_t total) {
    const uint64_t q = total / kXcds, r = total % kXcds, x = L % kXcds;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + L / kXcds;
}

// The 2-D grid (x fastest, as dispatched) as one linear id, renamed by xcd_chunk.
__device__ __forceinline__ uint64_t xcd_linear_block() {
    const uint64_t L = blockIdx.x + (uint64_t)blockIdx.y * gridDim.x;
    return xcd_chunk(L, (uint64_t)gridDim.x * gridDim.y);
}

}  // namespace sda
