// xcd.h -- XCD-aware workgroup order for the streaming kernels (gfx950: 8 XCDs, each with its own L2).
//
// The command processor hands workgroups to the XCDs round-robin in linear dispatch order, so with
// the natural order eight consecutive tiles -- adjacent 2 KiB pieces of the same HBM rows -- land on
// eight different XCDs and reach the memory controllers interleaved from eight L2s.  xcd_chunk32()
// renames the linear id so that the workgroups one XCD receives walk ONE contiguous eighth of the
// grid in order.  Measured on share-gen's memory pattern (tools/ubench_gen.hip, profiles/r04a): 41 GB
// of 37 % reads / 63 % writes in [n][B] clerk rows, 5.36 TB/s natural -> 6.32 TB/s chunked.
#pragma once
#include <stdint.h>

namespace sda {

constexpr uint32_t kXcds = 8;

// Bijective on [0, total): the blocks sharing an XCD (same L % 8) get consecutive ids.
__device__ __forceinline__ uint32_t xcd_chunk32(uint32_t L, uint32_t total) {
    const uint32_t q = total / kXcds, r = total % kXcds, x = L % kXcds;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + L / kXcds;
}

// The 2-D grid (x fastest, as dispatched) renamed by xcd_chunk: the block coordinates this workgroup
// takes.  32-bit arithmetic throughout (one 32-bit division by gridDim.x): the host launches the remapped
// kernels only when the grid holds fewer than 2^32 workgroups.
__device__ __forceinline__ void xcd_block_xy(uint32_t* bx, uint32_t* by) {
    const uint32_t L = xcd_chunk32(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
    *by = L / gridDim.x;
    *bx = L - *by * gridDim.x;
}

}  // namespace sda
