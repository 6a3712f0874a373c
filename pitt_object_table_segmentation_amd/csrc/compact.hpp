// compact.hpp -- order-preserving stream compaction over per-point predicates (ExtractIndices,
// createNewIdxMap's running counter, getPointOnPlane's output, cluster member lists).
//
// Layout: 256-thread blocks own 2048-point tiles; thread t owns the 8 CONSECUTIVE points
// [8t, 8t+8) of its tile so a block-wide exclusive scan of per-thread counts yields output
// positions in ascending point order.  Three launches: count per tile, scan of tile counts,
// write.  All kernels are persistent grid-stride loops over tiles.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"

namespace pitt {

constexpr int kCTile = 2048;

__host__ __device__ inline int64_t ctiles(int64_t n) { return (n + kCTile - 1) / kCTile; }

// A host cloud uploaded as it lies (SF floats per point: PCL PointXYZ 4, packed xyz 3) -> SoA planes
// (the *_aos entry points: one H2D copy of the caller's bytes, no host-side deinterleave).
template <int SF>
__global__ __launch_bounds__(256) void k_aos_planes(const float* __restrict__ aos, int64_t n, float* __restrict__ x,
                                                    float* __restrict__ y, float* __restrict__ z) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        x[i] = aos[i * SF];
        y[i] = aos[i * SF + 1];
        z[i] = aos[i * SF + 2];
    }
}
// hx: a host AoS cloud of `stride_bytes` (12 or 16) per point -> planes x/y/z on the context's stream.
inline hipError_t upload_aos(hipStream_t s, void* scratch, const float* hx, int64_t n, int stride_bytes, float* x,
                             float* y, float* z) {
    if (n <= 0) return hipSuccess;
    hipError_t e = hipMemcpyAsync(scratch, hx, (size_t)n * stride_bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    if (stride_bytes == 16)
        hipLaunchKernelGGL(k_aos_planes<4>, dim3(g), dim3(256), 0, s, (const float*)scratch, n, x, y, z);
    else
        hipLaunchKernelGGL(k_aos_planes<3>, dim3(g), dim3(256), 0, s, (const float*)scratch, n, x, y, z);
    return hipGetLastError();
}

// Pred: __device__ bool operator()(int64_t i) const  (i < n guaranteed by the caller)
template <class Pred>
__global__ __launch_bounds__(kBlock) void k_pred_count(Pred pred, int64_t n, int32_t* __restrict__ tile_counts) {
    __shared__ int32_t lds4[kBlock / 64];
    const int64_t nt = ctiles(n);
    for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const int64_t b = t * kCTile + threadIdx.x * 8;
        int c = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) c += (b + k < n && pred(b + k)) ? 1 : 0;
        int total;
        (void)block_exscan(c, lds4, &total);
        if (threadIdx.x == 0) tile_counts[t] = total;
    }
}

// Single-block exclusive scan: offsets[t] for t < nt, offsets[nt] = total.
__global__ __launch_bounds__(kBlock) void k_scan_tiles(const int32_t* __restrict__ counts, int64_t nt,
                                                       int32_t* __restrict__ offsets);

// Action: __device__ void operator()(int64_t i, int64_t pos) const  -- point i is output #pos
template <class Pred, class Action>
__global__ __launch_bounds__(kBlock) void k_pred_apply(Pred pred, Action act, int64_t n,
                                                       const int32_t* __restrict__ offsets) {
    __shared__ int32_t lds4[kBlock / 64];
    const int64_t nt = ctiles(n);
    for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const int64_t b = t * kCTile + threadIdx.x * 8;
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) bits |= ((b + k < n && pred(b + k)) ? 1u : 0u) << k;
        int total;
        int pos = block_exscan(__builtin_popcount(bits), lds4, &total) + offsets[t];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if ((bits >> k) & 1u) act(b + k, (int64_t)pos++);
    }
}

// Several small clouds at once (pitt_classify_clusters' selections): one block per cloud walks its tiles in
// order with a running offset -- count, scan and write in one launch.  cnt: the cloud's output count.
template <class Pred, class Action>
struct SelectItem {
    Pred pred;
    Action act;
    int64_t n;
    int32_t* cnt;
};
template <class Pred, class Action>
__global__ __launch_bounds__(kBlock) void k_select_small(const SelectItem<Pred, Action>* __restrict__ items) {
    __shared__ int32_t lds4[kBlock / 64];
    const SelectItem<Pred, Action> it = items[blockIdx.x];
    const int64_t nt = ctiles(it.n);
    int64_t run = 0;
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t b = t * kCTile + threadIdx.x * 8;
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) bits |= ((b + k < it.n && it.pred(b + k)) ? 1u : 0u) << k;
        int total;
        int64_t pos = block_exscan(__builtin_popcount(bits), lds4, &total) + run;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if ((bits >> k) & 1u) it.act(b + k, pos++);
        run += total;
    }
    if (threadIdx.x == 0) *it.cnt = (int32_t)run;
}
constexpr int64_t kSelectSmallTiles = 8;  // clouds up to 16k points take k_select_small

inline int grid_for_tiles(int64_t nt) { return (int)(nt < 1 ? 1 : (nt > 2048 ? 2048 : nt)); }

}  // namespace pitt
