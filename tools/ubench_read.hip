// ubench_read.hip -- HBM read ceiling on gfx950 for the combine's access pattern: a [rows][cols]
// i64 matrix streamed once, each lane owning VEC columns and walking the rows (as combine.hip),
// versus a flat grid-stride read.  Prints TB/s per variant (algorithmic bytes / kernel time).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_read.hip -o tools/ubench_read && ./tools/ubench_read
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef int64_t v2 __attribute__((ext_vector_type(2)));

// column walk: lane owns 2 columns, reads UNROLL rows before consuming (XOR keeps the loads live)
template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void colwalk(const v2* __restrict__ p, uint64_t rows, uint64_t lanes,
                                               uint64_t* __restrict__ sink) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= lanes) return;
    const v2* q = p + lane;
    int64_t acc = 0;
    for (uint64_t r = 0; r + UNROLL <= rows; r += UNROLL) {
        v2 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(q + (r + u) * lanes) : q[(r + u) * lanes];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u][0] + v[u][1];
    }
    if (acc == 0x123456789) sink[0] = acc;
}

// flat grid-stride read of 16 B per lane per load
__global__ __launch_bounds__(256) void flat(const v2* __restrict__ p, uint64_t n, uint64_t* __restrict__ sink) {
    int64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n; i += 8 * stride) {
        v2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u][0] + v[u][1];
    }
    for (; i < n; i += stride) acc ^= p[i][0];
    if (acc == 0x123456789) sink[0] = acc;
}

// LDS-DMA stream (global_load_lds_dwordx4): each wave moves 1 KiB per instruction straight into its
// own LDS slots, DEPTH instructions in flight, then reads its 16 B per slot back (ds_read_b128).
// COLWALK: the combine's pattern (a wave's 64 lanes own 128 adjacent columns = 1 KiB of one row and
// walk the rows); else a flat grid-stride over 1 KiB pieces.  AUX: cache policy bits (2 = nt).
typedef __attribute__((address_space(3))) void lds_void;
template <int DEPTH, bool COLWALK, int AUX>
__global__ __launch_bounds__(256) void glds(const v2* __restrict__ p, uint64_t rows, uint64_t lanes, uint64_t n,
                                            uint64_t* __restrict__ sink) {
    __shared__ v2 buf[4][DEPTH][64];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    int64_t acc = 0;
    if (COLWALK) {
        const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u) >= lanes) return;
        const v2* q = p + (lane < lanes ? lane : lanes - 1);
        for (uint64_t r = 0; r + DEPTH <= rows; r += DEPTH) {
#pragma unroll
            for (int u = 0; u < DEPTH; ++u)
                __builtin_amdgcn_global_load_lds((const void*)(q + (r + u) * lanes), (lds_void*)&buf[w][u][0], 16, 0, AUX);
            __builtin_amdgcn_s_waitcnt(0x3f70);   // vmcnt(0)
#pragma unroll
            for (int u = 0; u < DEPTH; ++u) { const v2 v = buf[w][u][l]; acc ^= v[0] + v[1]; }
        }
    } else {
        const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
        const uint64_t pieces = n / 64;
        for (uint64_t c = wave; c + (DEPTH - 1) * nw < pieces; c += DEPTH * nw) {
#pragma unroll
            for (int u = 0; u < DEPTH; ++u)
                __builtin_amdgcn_global_load_lds((const void*)(p + (c + u * nw) * 64 + l), (lds_void*)&buf[w][u][0], 16, 0, AUX);
            __builtin_amdgcn_s_waitcnt(0x3f70);
#pragma unroll
            for (int u = 0; u < DEPTH; ++u) { const v2 v = buf[w][u][l]; acc ^= v[0] + v[1]; }
        }
    }
    if (acc == 0x123456789) sink[0] = acc;
}

template <typename F>
static void timeit(const char* name, double bytes, F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < 5; ++r) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-40s %7.3f ms  %6.3f TB/s\n", name, ms / 5, bytes / (ms / 5 * 1e-3) / 1e12);
}

int main() {
    const uint64_t rows = 10000, cols = 1000000;               // configs[1]: 80 GB
    const uint64_t n16 = rows * cols / 2;
    v2* p;
    if (hipMalloc(&p, n16 * 16) != hipSuccess) { printf("alloc failed\n"); return 1; }
    (void)hipMemset(p, 1, n16 * 16);
    uint64_t* sink;
    (void)hipMalloc(&sink, 64);
    const double bytes = (double)n16 * 16;
    const uint64_t lanes = cols / 2;
    const unsigned cblocks = (unsigned)((lanes + 255) / 256);
    timeit("colwalk unroll 8 nt (combine pattern)", bytes, [&] { hipLaunchKernelGGL((colwalk<8, true>), dim3(cblocks), dim3(256), 0, 0, p, rows, lanes, sink); });
    timeit("colwalk unroll 16 nt", bytes, [&] { hipLaunchKernelGGL((colwalk<16, true>), dim3(cblocks), dim3(256), 0, 0, p, rows, lanes, sink); });
    timeit("colwalk unroll 8 cached", bytes, [&] { hipLaunchKernelGGL((colwalk<8, false>), dim3(cblocks), dim3(256), 0, 0, p, rows, lanes, sink); });
    timeit("colwalk unroll 4 nt", bytes, [&] { hipLaunchKernelGGL((colwalk<4, true>), dim3(cblocks), dim3(256), 0, 0, p, rows, lanes, sink); });
    for (unsigned g : {2048u, 8192u, 32768u})
        timeit(g == 2048 ? "flat grid-stride 2048 blocks" : (g == 8192 ? "flat grid-stride 8192 blocks" : "flat grid-stride 32768 blocks"),
               bytes, [&] { hipLaunchKernelGGL(flat, dim3(g), dim3(256), 0, 0, p, n16, sink); });
    timeit("glds colwalk depth 8 nt", bytes, [&] { hipLaunchKernelGGL((glds<8, true, 2>), dim3(cblocks), dim3(256), 0, 0, p, rows, lanes, n16, sink); });
    timeit("glds colwalk depth 8 default", bytes, [&] { hipLaunchKernelGGL((glds<8, true, 0>), dim3(cblocks), dim3(256), 0, 0, p, rows, lanes, n16, sink); });
    timeit("glds colwalk depth 16 nt", bytes, [&] { hipLaunchKernelGGL((glds<16, true, 2>), dim3(cblocks), dim3(256), 0, 0, p, rows, lanes, n16, sink); });
    for (unsigned g : {2048u, 8192u})
        timeit(g == 2048 ? "glds flat depth 8 nt 2048 blocks" : "glds flat depth 8 nt 8192 blocks", bytes,
               [&] { hipLaunchKernelGGL((glds<8, false, 2>), dim3(g), dim3(256), 0, 0, p, rows, lanes, n16, sink); });
    timeit("glds flat depth 16 nt 2048 blocks", bytes, [&] { hipLaunchKernelGGL((glds<16, false, 2>), dim3(2048), dim3(256), 0, 0, p, rows, lanes, n16, sink); });
    (void)hipFree(p);
    return 0;
}
