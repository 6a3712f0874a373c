// introsort.hip -- the permutation libstdc++'s std::sort gives a vector of (key, value) pairs compared
// by key only, reproduced on the device (VoxelGrid's index_vector, PCL 1.7 voxel_grid.hpp; DESIGN.md
// s3b, assumption A10: the libstdc++ >= 4.9 introsort, which this image's g++ ships).
//
// std::sort = __introsort_loop (partition segments longer than 16, depth limit 2 floor(log2 n), then
// heapsort) + __final_insertion_sort.  Every element of a final segment (<= 16) is <= every element of
// the next one, and insertion sort moves an element only past strictly greater keys, so the final
// pass equals a STABLE sort by key of the array the partitions leave.  The partitions are emulated
// level by level, all segments of a level at once:
//
//   pivot   __move_median_to_first(first, first + 1, mid, last - 1): the median key is swapped to
//           `first` (one thread per segment);
//   ranks   __unguarded_partition(first + 1, last, first) swaps the k-th left stop (key >= p) with the
//           k-th right stop (key <= p, counted from the end) while the first lies left of the second;
//           both ranks come from two device-wide exclusive scans of the stop flags;
//   cut     after K swaps the scan returns min(L[K], R[K - 1]) (R[K - 1] alone when L is exhausted);
//   split   [first, cut) and [cut, last) with depth - 1; segments of <= 16 are final;
//   heap    a segment whose depth runs out is heap-sorted exactly as std::__partial_sort(first, last,
//           last) (make_heap + sort_heap, one thread).
// The caller then runs a stable radix sort by key.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_scan.hpp>

#include <algorithm>
#include <vector>

#include "ctx.hpp"
#include "device_common.hpp"

namespace pitt {

struct ISeg {
    int32_t f, l, depth;
    uint32_t pivot;
    int32_t nL, nR, K, cut, childL, childR, active, pad;
};

constexpr int kIsThreshold = 16;  // _S_threshold

__device__ __forceinline__ void is_swap(uint32_t* key, uint32_t* val, int a, int b) {
    const uint32_t ka = key[a], va = val[a];
    key[a] = key[b];
    val[a] = val[b];
    key[b] = ka;
    val[b] = va;
}

// pivot: median of (first + 1, mid, last - 1) to first; a segment out of depth goes to the heap list
__global__ void k_is_pivot(ISeg* __restrict__ segs, int nseg, uint32_t* __restrict__ key, uint32_t* __restrict__ val,
                           int32_t* __restrict__ heap, int32_t* __restrict__ heap_cnt) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    ISeg g = segs[s];
    g.K = 0;
    g.active = 1;
    if (g.depth == 0) {
        g.active = 0;
        heap[atomicAdd(heap_cnt, 1)] = s;
        segs[s] = g;
        return;
    }
    const int f = g.f, a = f + 1, b = f + (g.l - f) / 2, c = g.l - 1;
    const uint32_t ka = key[a], kb = key[b], kc = key[c];
    int m;
    if (ka < kb) m = (kb < kc) ? b : (ka < kc) ? c : a;
    else m = (ka < kc) ? a : (kb < kc) ? c : b;
    is_swap(key, val, f, m);
    g.pivot = key[f];
    segs[s] = g;
}

__global__ void k_is_flags(const int32_t* __restrict__ segid, const ISeg* __restrict__ segs, const uint32_t* __restrict__ key,
                           int64_t n, int32_t* __restrict__ FL, int32_t* __restrict__ FR) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
        int fl = 0, fr = 0;
        if (i < n) {
            const int s = segid[i];
            if (s >= 0 && segs[s].active && i != segs[s].f) {
                const uint32_t p = segs[s].pivot, k = key[i];
                fl = !(k < p);
                fr = !(p < k);
            }
        }
        FL[i] = fl;
        FR[i] = fr;
    }
}

__global__ void k_is_counts(ISeg* __restrict__ segs, int nseg, const int32_t* __restrict__ SL,
                            const int32_t* __restrict__ SR) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg || !segs[s].active) return;
    const int b = segs[s].f + 1, l = segs[s].l;
    segs[s].nL = SL[l] - SL[b];
    segs[s].nR = SR[l] - SR[b];
}

// posL[first + 1 + k] = position of the k-th left stop; posR[first + 1 + k] = the k-th right stop
// from the end (both inside the segment's own range)
__global__ void k_is_rank(const int32_t* __restrict__ segid, const ISeg* __restrict__ segs,
                          const int32_t* __restrict__ FL, const int32_t* __restrict__ FR, const int32_t* __restrict__ SL,
                          const int32_t* __restrict__ SR, int64_t n, int32_t* __restrict__ posL,
                          int32_t* __restrict__ posR) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!FL[i] && !FR[i]) continue;
        const ISeg& g = segs[segid[i]];
        const int b = g.f + 1;
        if (FL[i]) posL[b + (SL[i] - SL[b])] = (int32_t)i;
        if (FR[i]) posR[b + (SR[g.l] - SR[i + 1])] = (int32_t)i;
    }
}

// K = the number of k < min(nL, nR) with posL[k] < posR[k]: the predicate holds on a prefix (posL
// rises, posR falls), so one thread per segment finds its end by bisection
__global__ void k_is_k(ISeg* __restrict__ segs, int nseg, const int32_t* __restrict__ posL,
                       const int32_t* __restrict__ posR) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg || !segs[s].active) return;
    const int b = segs[s].f + 1;
    int lo = 0, hi = min(segs[s].nL, segs[s].nR);  // first k where the predicate fails
    while (lo < hi) {
        const int mid = lo + ((hi - lo) >> 1);
        if (posL[b + mid] < posR[b + mid]) lo = mid + 1;
        else hi = mid;
    }
    segs[s].K = lo;
}

__global__ void k_is_swap(const int32_t* __restrict__ segid, const ISeg* __restrict__ segs,
                          const int32_t* __restrict__ posL, const int32_t* __restrict__ posR, int64_t n,
                          uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const int s = segid[j];
        if (s < 0 || !segs[s].active) continue;
        const int k = (int)j - (segs[s].f + 1);
        if (k >= 0 && k < segs[s].K) is_swap(key, val, posL[j], posR[j]);  // disjoint pairs
    }
}

__global__ void k_is_split(ISeg* __restrict__ segs, int nseg, const int32_t* __restrict__ posL,
                           const int32_t* __restrict__ posR, ISeg* __restrict__ next, int32_t* __restrict__ next_cnt) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    ISeg g = segs[s];
    g.childL = g.childR = -1;
    if (g.active) {
        const int b = g.f + 1, K = g.K;
        int cut;
        if (K < g.nL) cut = K > 0 ? min(posL[b + K], posR[b + K - 1]) : posL[b + K];
        else cut = posR[b + K - 1];
        g.cut = cut;
        const int d = g.depth - 1;
        if (cut - g.f > kIsThreshold) {
            const int id = atomicAdd(next_cnt, 1);
            ISeg c = {};
            c.f = g.f;
            c.l = cut;
            c.depth = d;
            next[id] = c;
            g.childL = id;
        }
        if (g.l - cut > kIsThreshold) {
            const int id = atomicAdd(next_cnt, 1);
            ISeg c = {};
            c.f = cut;
            c.l = g.l;
            c.depth = d;
            next[id] = c;
            g.childR = id;
        }
    }
    segs[s] = g;
}

__global__ void k_is_segid(int32_t* __restrict__ segid, const ISeg* __restrict__ segs, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int s = segid[i];
        if (s < 0) continue;
        const ISeg& g = segs[s];
        segid[i] = !g.active ? -1 : (i < g.cut ? g.childL : g.childR);
    }
}

// ---- std::__partial_sort(first, last, last): __make_heap + __sort_heap (libstdc++ stl_heap.h) -------
__device__ void is_push_heap(uint32_t* key, uint32_t* val, int hole, int top, uint32_t vk, uint32_t vv) {
    int parent = (hole - 1) / 2;
    while (hole > top && key[parent] < vk) {
        key[hole] = key[parent];
        val[hole] = val[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    key[hole] = vk;
    val[hole] = vv;
}

__device__ void is_adjust_heap(uint32_t* key, uint32_t* val, int hole, int len, uint32_t vk, uint32_t vv) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (key[second] < key[second - 1]) second--;
        key[hole] = key[second];
        val[hole] = val[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        key[hole] = key[second - 1];
        val[hole] = val[second - 1];
        hole = second - 1;
    }
    is_push_heap(key, val, hole, top, vk, vv);
}

__global__ void k_is_heap(const ISeg* __restrict__ segs, const int32_t* __restrict__ heap,
                          const int32_t* __restrict__ heap_cnt, uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= *heap_cnt) return;
    const ISeg g = segs[heap[h]];
    uint32_t* k = key + g.f;
    uint32_t* v = val + g.f;
    const int len = g.l - g.f;
    if (len >= 2) {  // __make_heap
        for (int parent = (len - 2) / 2;; --parent) {
            is_adjust_heap(k, v, parent, len, k[parent], v[parent]);
            if (parent == 0) break;
        }
    }
    for (int last = len; last > 1;) {  // __sort_heap: __pop_heap(first, last - 1, last - 1)
        --last;
        const uint32_t vk = k[last], vv = v[last];
        k[last] = k[0];
        v[last] = v[0];
        is_adjust_heap(k, v, 0, last, vk, vv);
    }
}

static inline int is_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096)); }

// Leaves key/val so that a stable sort by key gives std::sort's order.  depth_limit < 0: libstdc++'s
// 2 floor(log2 n); otherwise the given limit (tests reach the heapsort fallback with it).
int introsort_partitions(pitt_ctx* ctx, uint32_t* key, uint32_t* val, int64_t n, int depth_limit) {
    hipStream_t s = ctx->stream;
    if (n <= kIsThreshold) return PITT_OK;
    const int64_t cap = n / kIsThreshold + 16;  // active segments hold > 16 elements each
    ISeg* segA = (ISeg*)ctx->buf("is_segA", (size_t)cap * sizeof(ISeg));
    ISeg* segB = (ISeg*)ctx->buf("is_segB", (size_t)cap * sizeof(ISeg));
    int32_t* segid = (int32_t*)ctx->buf("is_segid", (size_t)n * 4);
    int32_t* FL = (int32_t*)ctx->buf("is_FL", (size_t)(n + 1) * 4);
    int32_t* FR = (int32_t*)ctx->buf("is_FR", (size_t)(n + 1) * 4);
    int32_t* SL = (int32_t*)ctx->buf("is_SL", (size_t)(n + 1) * 4);
    int32_t* SR = (int32_t*)ctx->buf("is_SR", (size_t)(n + 1) * 4);
    int32_t* posL = (int32_t*)ctx->buf("is_posL", (size_t)n * 4);
    int32_t* posR = (int32_t*)ctx->buf("is_posR", (size_t)n * 4);
    int32_t* cnt = (int32_t*)ctx->buf("is_cnt", 16);
    int32_t* heap = (int32_t*)ctx->buf("is_heap", (size_t)cap * 4);
    int32_t* hcnt = (int32_t*)ctx->pinned("is_hcnt", 16);
    if (!segA || !segB || !segid || !FL || !FR || !SL || !SR || !posL || !posR || !cnt || !heap || !hcnt)
        return ctx->fail(PITT_E_NOMEM, "introsort scratch");
    size_t scan_bytes = 0;
    PITT_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, FL, SL, (int)(n + 1), s));
    void* scan_tmp = ctx->buf("is_scan_tmp", std::max<size_t>(scan_bytes, 16));
    if (!scan_tmp) return ctx->fail(PITT_E_NOMEM, "introsort scan scratch");
    int lg = 0;
    while (((int64_t)2 << lg) <= n) ++lg;  // std::__lg(n)
    ISeg root = {};
    root.f = 0;
    root.l = (int32_t)n;
    root.depth = depth_limit >= 0 ? depth_limit : 2 * lg;
    PITT_HIP_TRY(hipStreamSynchronize(s));
    PITT_HIP_TRY(hipMemcpy(segA, &root, sizeof root, hipMemcpyHostToDevice));
    PITT_HIP_TRY(hipMemsetAsync(segid, 0, (size_t)n * 4, s));
    PITT_HIP_TRY(hipMemsetAsync(cnt, 0, 16, s));
    int nseg = 1;
    // heap segments are appended across levels into one list; their descriptors stay in a copy
    ISeg* heapsegs = (ISeg*)ctx->buf("is_heapsegs", (size_t)cap * sizeof(ISeg));
    int32_t* heapmap = (int32_t*)ctx->buf("is_heapmap", (size_t)cap * 4);
    if (!heapsegs || !heapmap) return ctx->fail(PITT_E_NOMEM, "introsort heap list");
    int nheap = 0;
    ISeg* cur = segA;
    ISeg* nxt = segB;
    const int g = is_grid(n);
    while (nseg > 0) {
        const int sb = (nseg + 255) / 256;
        PITT_HIP_TRY(hipMemsetAsync(cnt, 0, 16, s));
        hipLaunchKernelGGL(k_is_pivot, dim3(sb), dim3(256), 0, s, cur, nseg, key, val, heap, cnt + 1);
        hipLaunchKernelGGL(k_is_flags, dim3(g), dim3(256), 0, s, segid, cur, key, n, FL, FR);
        PITT_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, FL, SL, (int)(n + 1), s));
        PITT_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, FR, SR, (int)(n + 1), s));
        hipLaunchKernelGGL(k_is_counts, dim3(sb), dim3(256), 0, s, cur, nseg, SL, SR);
        hipLaunchKernelGGL(k_is_rank, dim3(g), dim3(256), 0, s, segid, cur, FL, FR, SL, SR, n, posL, posR);
        hipLaunchKernelGGL(k_is_k, dim3(sb), dim3(256), 0, s, cur, nseg, posL, posR);
        hipLaunchKernelGGL(k_is_swap, dim3(g), dim3(256), 0, s, segid, cur, posL, posR, n, key, val);
        hipLaunchKernelGGL(k_is_split, dim3(sb), dim3(256), 0, s, cur, nseg, posL, posR, nxt, cnt);
        hipLaunchKernelGGL(k_is_segid, dim3(g), dim3(256), 0, s, segid, cur, n);
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipMemcpyAsync(hcnt, cnt, 8, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        const int nh = hcnt[1];
        if (nh > 0) {  // this level's depth-exhausted segments: keep their descriptors for the heap pass
            std::vector<int32_t> hl((size_t)nh);
            PITT_HIP_TRY(hipMemcpy(hl.data(), heap, (size_t)nh * 4, hipMemcpyDeviceToHost));
            for (int i = 0; i < nh; ++i) {
                PITT_HIP_TRY(hipMemcpyAsync(heapsegs + nheap, cur + hl[(size_t)i], sizeof(ISeg),
                                            hipMemcpyDeviceToDevice, s));
                ++nheap;
            }
        }
        nseg = hcnt[0];
        std::swap(cur, nxt);
    }
    if (nheap > 0) {
        std::vector<int32_t> ids((size_t)nheap);
        for (int i = 0; i < nheap; ++i) ids[(size_t)i] = i;
        int32_t* hc = (int32_t*)ctx->buf("is_heapcnt", 16);
        if (!hc) return ctx->fail(PITT_E_NOMEM, "introsort heap count");
        PITT_HIP_TRY(hipStreamSynchronize(s));
        PITT_HIP_TRY(hipMemcpy(heapmap, ids.data(), (size_t)nheap * 4, hipMemcpyHostToDevice));
        PITT_HIP_TRY(hipMemcpy(hc, &nheap, 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_is_heap, dim3((nheap + 63) / 64), dim3(64), 0, s, heapsegs, heapmap, hc, key, val);
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipStreamSynchronize(s));
    }
    return PITT_OK;
}

}  // namespace pitt
