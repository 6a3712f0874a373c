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

struct ISmall {
    int32_t f, l, depth, pad;
};

constexpr int kIsThreshold = 16;  // _S_threshold
#ifndef PITT_IS_SMALL
#define PITT_IS_SMALL 2048
#endif
constexpr int kIsSmall = PITT_IS_SMALL;  // segments this short finish in one wave, in LDS
#ifndef PITT_IS_COOP_MAX
#define PITT_IS_COOP_MAX 64
#endif    // segments this short finish in one wave, in LDS

__device__ __forceinline__ void is_swap(uint32_t* key, uint32_t* val, int a, int b) {
    const uint32_t ka = key[a], va = val[a];
    key[a] = key[b];
    val[a] = val[b];
    key[b] = ka;
    val[b] = va;
}

// children of <= 16 are final; children of <= kIsSmall go to the one-wave list, larger ones to the next level
__device__ __forceinline__ int is_child(int f, int l, int d, ISeg* next, int32_t* next_cnt, ISmall* small,
                                        int32_t* small_cnt) {
    if (l - f <= kIsThreshold) return -1;
    if (l - f <= kIsSmall) {
        small[atomicAdd(small_cnt, 1)] = ISmall{f, l, d, 0};
        return -1;
    }
    const int id = atomicAdd(next_cnt, 1);
    ISeg c = {};
    c.f = f;
    c.l = l;
    c.depth = d;
    next[id] = c;
    return id;
}

__device__ __forceinline__ int is_load_count(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kIsLvT = 1024;  // threads per block of the level kernel
constexpr int kIsLvW = kIsLvT / 64;

// Exclusive scan of two flags over a kIsLvT-thread block; ta / tb = the block totals.
__device__ __forceinline__ void is_block_scan2(int a, int b, int& ea, int& eb, int& ta, int& tb, int* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int ia = a, ib = b;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int xa = __shfl_up(ia, off, 64), xb = __shfl_up(ib, off, 64);
        if (lane >= off) {
            ia += xa;
            ib += xb;
        }
    }
    if (lane == 63) {
        sh[w] = ia;
        sh[kIsLvW + w] = ib;
    }
    __syncthreads();
    int oa = 0, ob = 0;
    ta = tb = 0;
#pragma unroll
    for (int j = 0; j < kIsLvW; ++j) {
        const int sa = sh[j], sb = sh[kIsLvW + j];
        oa += j < w ? sa : 0;
        ob += j < w ? sb : 0;
        ta += sa;
        tb += sb;
    }
    __syncthreads();
    ea = oa + ia - a;
    eb = ob + ib - b;
}

// Grid barrier over a monotonically rising arrival counter (zeroed before the launch): barrier j
// waits for j * gridDim.x arrivals.  The grid is small enough that every block is resident.  Agent-
// scope release / acquire make the blocks' writes visible across the XCDs' L2s.
__device__ __forceinline__ void is_grid_sync(uint32_t* bar, uint32_t& target) {
    __syncthreads();
    target += gridDim.x;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
}

// All levels of segments longer than kIsSmall in one launch of a resident grid; a level is five grid-wide
// phases (grid barriers between them):
//   1 pivot   per segment: median of (first + 1, mid, last - 1) to first; depth 0 -> the heap list
//             (beside it, the previous level's step 7);
//   2 flags   per element: left stop (key >= p) / right stop (key <= p) of its segment, block-local
//             exclusive ranks over the block's contiguous chunk, block totals;
//   4 ranks   global rank = block-local rank + the prefix of the block totals (each block forms it);
//             per element: posL[first + 1 + k] = the k-th left stop, posR[first + 1 + k] = the k-th
//             right stop from the end; per segment nL / nR;
//   5 K       per segment: the swaps __unguarded_partition makes (posL[k] < posR[k] holds on a prefix);
//   6 swap    per element k < K: swap posL[k] <-> posR[k]; per segment: the cut, the children;
//   7 segid   per element: its child segment (or -1) -- run with the next level's step 1, after every
//             block has read the next level's segment count.
__global__ __launch_bounds__(kIsLvT) void k_is_levels(ISeg* __restrict__ segA, ISeg* __restrict__ segB,
                                                   ISeg* __restrict__ heap, ISmall* __restrict__ small,
                                                   int32_t* __restrict__ cnt, int32_t* __restrict__ segid,
                                                   uint8_t* __restrict__ F, int32_t* __restrict__ SL,
                                                   int32_t* __restrict__ SR, int32_t* __restrict__ posL,
                                                   int32_t* __restrict__ posR, int32_t* __restrict__ bsum,
                                                   uint32_t* __restrict__ key, uint32_t* __restrict__ val, int64_t n,
                                                   int64_t chunk, int levels, uint32_t* __restrict__ bar) {
    __shared__ int sh[2 * kIsLvW];
    __shared__ int preL[513], preR[513];  // G <= 512
    uint32_t target = 0;
    const int G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
    const int64_t gt = (int64_t)b * kIsLvT + tid, gstride = (int64_t)G * kIsLvT;
    const int64_t c0 = min(n, (int64_t)b * chunk), c1 = min(n, c0 + chunk);
    ISeg* cur = segA;
    ISeg* nxt = segB;
    for (int v = 0; v < levels; ++v) {
        const int nseg = is_load_count(cnt + 2 + v);  // the same value in every block (after a barrier)
        if (nseg == 0) break;
        if (v > 0) {  // 7 (of the previous level) next segment ids -- beside this level's pivots
            for (int64_t i = gt; i < n; i += gstride) {
                const int s = segid[i];
                if (s < 0) continue;
                const ISeg& g = nxt[s];
                segid[i] = !g.active ? -1 : (i < g.cut ? g.childL : g.childR);
            }
        }
        // 1 pivot
        for (int64_t s = gt; s < nseg; s += gstride) {
            ISeg g = cur[s];
            g.K = 0;
            g.active = 1;
            g.childL = g.childR = -1;
            if (g.depth == 0) {
                g.active = 0;
                heap[atomicAdd(cnt, 1)] = g;
            } else {
                const int f = g.f, a = f + 1, bb = f + (g.l - f) / 2, c = g.l - 1;
                const uint32_t ka = key[a], kb = key[bb], kc = key[c];
                int m;
                if (ka < kb) m = (kb < kc) ? bb : (ka < kc) ? c : a;
                else m = (ka < kc) ? a : (kb < kc) ? c : bb;
                is_swap(key, val, f, m);
                g.pivot = key[f];
            }
            cur[s] = g;
        }
        is_grid_sync(bar, target);
        // 2 flags and block-local ranks
        int carL = 0, carR = 0;
        for (int64_t base = c0; base < c1; base += kIsLvT) {
            const int64_t i = base + tid;
            int fl = 0, fr = 0;
            if (i < c1) {
                const int s = segid[i];
                if (s >= 0) {
                    const ISeg& g = cur[s];
                    if (g.active && i != g.f) {
                        const uint32_t p = g.pivot, k = key[i];
                        fl = !(k < p);
                        fr = !(p < k);
                    }
                }
            }
            int el, er, tl, tr;
            is_block_scan2(fl, fr, el, er, tl, tr, sh);
            if (i < c1) {
                SL[i] = carL + el;
                SR[i] = carR + er;
                F[i] = (uint8_t)(fl | (fr << 1));
            }
            carL += tl;
            carR += tr;
        }
        if (tid == 0) {
            bsum[b] = carL;
            bsum[G + b] = carR;
        }
        is_grid_sync(bar, target);
        // 4 stop positions; stop counts.  Global ranks = block-local rank + the prefix of the block
        // totals (every block forms the prefix itself: no separate pass)
        for (int j = tid; j <= G; j += kIsLvT) {
            int a = 0, r = 0;
            for (int q = 0; q < j; ++q) a += bsum[q], r += bsum[G + q];
            preL[j] = a;
            preR[j] = r;
        }
        __syncthreads();
        auto gl = [&](int64_t i) { return i >= n ? preL[G] : SL[i] + preL[i / chunk]; };
        auto gr = [&](int64_t i) { return i >= n ? preR[G] : SR[i] + preR[i / chunk]; };
        for (int64_t s = gt; s < nseg; s += gstride) {
            if (!cur[s].active) continue;
            const int bb = cur[s].f + 1, l = cur[s].l;
            cur[s].nL = gl(l) - gl(bb);
            cur[s].nR = gr(l) - gr(bb);
        }
        for (int64_t i = gt; i < n; i += gstride) {
            const int fb = F[i];
            if (!fb) continue;
            const ISeg& g = cur[segid[i]];
            const int bb = g.f + 1;
            if (fb & 1) posL[bb + (gl(i) - gl(bb))] = (int32_t)i;
            if (fb & 2) posR[bb + (gr(g.l) - gr(i + 1))] = (int32_t)i;
        }
        is_grid_sync(bar, target);
        // 5 K by bisection
        for (int64_t s = gt; s < nseg; s += gstride) {
            if (!cur[s].active) continue;
            const int bb = cur[s].f + 1;
            int lo = 0, hi = min(cur[s].nL, cur[s].nR);
            while (lo < hi) {
                const int mid = lo + ((hi - lo) >> 1);
                if (posL[bb + mid] < posR[bb + mid]) lo = mid + 1;
                else hi = mid;
            }
            cur[s].K = lo;
        }
        is_grid_sync(bar, target);
        // 6 swaps; cut and children
        for (int64_t j = gt; j < n; j += gstride) {
            const int s = segid[j];
            if (s < 0) continue;
            const ISeg& g = cur[s];
            if (!g.active) continue;
            const int k = (int)j - (g.f + 1);
            if (k >= 0 && k < g.K) is_swap(key, val, posL[j], posR[j]);  // disjoint pairs
        }
        for (int64_t s = gt; s < nseg; s += gstride) {
            ISeg g = cur[s];
            if (!g.active) continue;
            const int bb = g.f + 1, K = g.K;
            int cut;
            if (K < g.nL) cut = K > 0 ? min(posL[bb + K], posR[bb + K - 1]) : posL[bb + K];
            else cut = posR[bb + K - 1];
            cur[s].cut = cut;  // the swap loop above reads the other fields of cur[s]
            cur[s].childL = is_child(g.f, cut, g.depth - 1, nxt, cnt + 3 + v, small, cnt + 1);
            cur[s].childR = is_child(cut, g.l, g.depth - 1, nxt, cnt + 3 + v, small, cnt + 1);
        }
        is_grid_sync(bar, target);
        ISeg* t = cur;  // phase 7 runs at the top of the next level, over nxt (= this level's segments)
        cur = nxt;
        nxt = t;
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

__device__ void is_heap_sort(uint32_t* k, uint32_t* v, int len) {
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

// Heap segments (depth exhausted, all longer than kIsSmall) -- one 256-thread block each, the keys
// and 16-bit local indices resident in LDS (6 B per element):
//   make_heap  the parents of one heap depth sift down in parallel (their subtrees are disjoint, and
//              __make_heap takes every deeper parent first), deepest depth first;
//   sort_heap  one wave: each __adjust_heap descent reads the six-level subtree below the hole at
//              once (lane j: internal node j, its larger child by `right < left`), walks the path in
//              scalar registers and moves the path's children up with one store per lane; the
//              push-up of the displaced value runs on one lane.
// The values follow the local indices at the end (vtmp: the segment's original values).  A segment
// above kHeapLds elements falls back to the one-thread global-memory heapsort.
constexpr int kHeapLds = 26624;  // 6 B x 26624 = 156 KB of LDS

// Orders one wave's LDS accesses across lanes: LDS executes a wave's accesses in issue order, so a
// compiler barrier (no reordering of the accesses around it) is enough.
__device__ __forceinline__ void is_lds_fence() { asm volatile("" ::: "memory"); }

template <typename V>
__device__ void is_sift_lds(uint32_t* sk, V* si, int hole, int len, uint32_t vk, V vi) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (sk[second] < sk[second - 1]) second--;
        sk[hole] = sk[second];
        si[hole] = si[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        sk[hole] = sk[second - 1];
        si[hole] = si[second - 1];
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && sk[parent] < vk) {
        sk[hole] = sk[parent];
        si[hole] = si[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    sk[hole] = vk;
    si[hole] = vi;
}

// __make_heap over LDS by NT threads (t = this thread's rank): one heap depth at a time, deepest first
// (the parents of one depth have disjoint subtrees, and __make_heap takes every deeper parent first).
template <int NT, typename V>
__device__ void is_make_heap_lds(uint32_t* sk, V* si, int len, int t) {
    if (len < 2) return;
    const int last_parent = (len - 2) / 2;
    int D = 0;
    while ((2 << D) - 1 <= last_parent) ++D;  // depth of the last parent
    for (int d = D; d >= 0; --d) {
        const int lo = (1 << d) - 1, hi = min((2 << d) - 2, last_parent);
        for (int p = hi - t; p >= lo; p -= NT) is_sift_lds(sk, si, p, len, sk[p], si[p]);
        if constexpr (NT == 64) is_lds_fence();
        else __syncthreads();
    }
}

// __sort_heap over LDS by one wave: each __adjust_heap descent reads the six-level subtree below the
// hole at once (lane j: internal node j, its larger child by `right < left`), walks the path in
// scalar registers and moves the path's children up with one store per lane; the push-up of the
// displaced value runs on lane 0.
template <typename V>
__device__ void is_sort_heap_wave(uint32_t* sk, V* si, int len, int lane) {
    // lane j < 63: internal node j of a six-level subtree (breadth-first: depth dj, offset oj)
    const int dj = 31 - __clz(lane + 1), oj = lane + 1 - (1 << dj);
    for (int last = len - 1; last >= 1; --last) {
        const uint32_t vk = sk[last];
        const V vi = si[last];
        is_lds_fence();
        if (lane == 0) {
            sk[last] = sk[0];
            si[last] = si[0];
        }
        is_lds_fence();  // the stores above land before the reads below (LDS is in order per wave)
        const int n2 = (last - 1) / 2;  // nodes below n2 have two children inside [0, last)
        int hole = 0;
        while (hole < n2) {
            const int gn = ((hole + 1) << dj) - 1 + oj;
            const bool has2 = lane < 63 && gn < n2;
            uint32_t kl = 0, kr = 0;
            V il = 0, ir = 0;
            if (has2) {
                kl = sk[2 * gn + 1];
                kr = sk[2 * gn + 2];
                il = si[2 * gn + 1];
                ir = si[2 * gn + 2];
            }
            const bool left = has2 && kr < kl;  // libstdc++: second-- when right < left
            const uint64_t m2 = __ballot(has2), ml = __ballot(left);
            uint64_t path = 0;
            int j = 0;
            while (j < 63 && ((m2 >> j) & 1)) {
                path |= 1ull << j;
                j = 2 * j + (((ml >> j) & 1) ? 1 : 2);
            }
            if ((path >> lane) & 1) {  // the next round reads below the new hole only
                sk[gn] = left ? kl : kr;
                si[gn] = left ? il : ir;
            }
            const int dd = 31 - __clz(j + 1);
            hole = ((hole + 1) << dd) - 1 + (j + 1 - (1 << dd));
        }
        is_lds_fence();
        if (lane == 0) {  // the even-length tail and __push_heap of the displaced value
            if ((last & 1) == 0 && hole == (last - 2) / 2) {
                const int c = 2 * (hole + 1) - 1;
                sk[hole] = sk[c];
                si[hole] = si[c];
                hole = c;
            }
            int parent = (hole - 1) / 2;
            while (hole > 0 && sk[parent] < vk) {
                sk[hole] = sk[parent];
                si[hole] = si[parent];
                hole = parent;
                parent = (hole - 1) / 2;
            }
            sk[hole] = vk;
            si[hole] = vi;
        }
        is_lds_fence();
    }
}

__global__ __launch_bounds__(256) void k_is_heap(const ISeg* __restrict__ segs, const int32_t* __restrict__ heap_cnt,
                                                 uint32_t* __restrict__ key, uint32_t* __restrict__ val,
                                                 uint32_t* __restrict__ vtmp) {
    extern __shared__ uint32_t is_smem[];
    if ((int)blockIdx.x >= *heap_cnt) return;
    const ISeg g = segs[blockIdx.x];
    const int len = g.l - g.f, tid = threadIdx.x;
    if (len > kHeapLds) {
        if (tid == 0) is_heap_sort(key + g.f, val + g.f, len);
        return;
    }
    uint32_t* sk = is_smem;
    uint16_t* si = reinterpret_cast<uint16_t*>(is_smem + len);
    for (int i = tid; i < len; i += 256) {
        sk[i] = key[g.f + i];
        si[i] = (uint16_t)i;
        vtmp[g.f + i] = val[g.f + i];
    }
    __syncthreads();
    is_make_heap_lds<256>(sk, si, len, tid);
    if (tid < 64) is_sort_heap_wave(sk, si, len, tid);
    __syncthreads();
    for (int i = tid; i < len; i += 256) {
        key[g.f + i] = sk[i];
        val[g.f + i] = vtmp[g.f + si[i]];
    }
}

// One wave finishes a segment of <= kIsSmall elements in LDS: the same median / unguarded-partition /
// depth / heapsort steps as the level kernels, run one partition at a time with an explicit stack
// (right part pushed, left part continued, as __introsort_loop recurses).  Stops are ranked with
// ballots: left stops forward from first + 1, right stops backward from last - 1.
__global__ __launch_bounds__(64) void k_is_small(const ISmall* __restrict__ segs, const int32_t* __restrict__ small_cnt,
                                                 uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
    __shared__ uint32_t sk[kIsSmall], sv[kIsSmall];
    __shared__ int32_t pl[kIsSmall], pr[kIsSmall];
    __shared__ int32_t stk[3 * 72];
    if ((int)blockIdx.x >= *small_cnt) return;
    const ISmall g = segs[blockIdx.x];
    const int lane = threadIdx.x;
    const int len = g.l - g.f;
    for (int i = lane; i < len; i += 64) {
        sk[i] = key[g.f + i];
        sv[i] = val[g.f + i];
    }
    __syncthreads();
    int sp = 0, f = 0, l = len, depth = g.depth;
    for (;;) {
        while (l - f > kIsThreshold) {
            if (depth == 0) {
                __syncthreads();
                is_make_heap_lds<64>(sk + f, sv + f, l - f, lane);
                is_sort_heap_wave(sk + f, sv + f, l - f, lane);
                __syncthreads();
                break;
            }
            --depth;
            const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
            const uint32_t ka = sk[a], kb = sk[b], kc = sk[c];
            int m;
            if (ka < kb) m = (kb < kc) ? b : (ka < kc) ? c : a;
            else m = (ka < kc) ? a : (kb < kc) ? c : b;
            __syncthreads();
            if (lane == 0) {
                const uint32_t tk = sk[f], tv = sv[f];
                sk[f] = sk[m];
                sv[f] = sv[m];
                sk[m] = tk;
                sv[m] = tv;
            }
            __syncthreads();
            const uint32_t p = sk[f];
            int nL = 0, nR = 0;
            for (int base = f + 1; base < l; base += 64) {
                const int i = base + lane;
                const bool st = i < l && !(sk[i] < p);
                const uint64_t bal = __ballot(st);
                if (st) pl[nL + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = i;
                nL += __popcll(bal);
            }
            for (int base = l - 1; base > f; base -= 64) {
                const int i = base - lane;
                const bool st = i > f && !(p < sk[i]);
                const uint64_t bal = __ballot(st);
                if (st) pr[nR + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = i;
                nR += __popcll(bal);
            }
            __syncthreads();
            const int kmax = min(nL, nR);
            int K = kmax;  // the swaps run while the k-th left stop lies left of the k-th right stop
            for (int k0 = 0; k0 < kmax; k0 += 64) {
                const int k = k0 + lane;
                const uint64_t bal = __ballot(k < kmax && !(pl[k] < pr[k]));
                if (bal) {
                    K = k0 + __builtin_ctzll(bal);
                    break;
                }
            }
            for (int k = lane; k < K; k += 64) {
                const int x = pl[k], y = pr[k];
                const uint32_t tk = sk[x], tv = sv[x];
                sk[x] = sk[y];
                sv[x] = sv[y];
                sk[y] = tk;
                sv[y] = tv;
            }
            const int cut = K < nL ? (K > 0 ? min(pl[K], pr[K - 1]) : pl[K]) : pr[K - 1];
            __syncthreads();
            if (l - cut > kIsThreshold) {  // __introsort_loop(cut, last, depth)
                stk[3 * sp] = cut;
                stk[3 * sp + 1] = l;
                stk[3 * sp + 2] = depth;
                ++sp;
            }
            l = cut;
        }
        if (sp == 0) break;
        --sp;
        f = stk[3 * sp];
        l = stk[3 * sp + 1];
        depth = stk[3 * sp + 2];
    }
    __syncthreads();
    for (int i = lane; i < len; i += 64) {
        key[g.f + i] = sk[i];
        val[g.f + i] = sv[i];
    }
}

// Leaves key/val so that a stable sort by key gives std::sort's order.  depth_limit < 0: libstdc++'s
// 2 floor(log2 n); otherwise the given limit (tests reach the heapsort fallback with it).
int introsort_partitions(pitt_ctx* ctx, uint32_t* key, uint32_t* val, int64_t n, int depth_limit) {
    hipStream_t s = ctx->stream;
    if (n <= kIsThreshold) return PITT_OK;
    if (n > INT32_MAX - 1) return ctx->fail(PITT_E_INVALID, "introsort: n exceeds int32 positions");
    const int64_t cap = n / kIsSmall + 16;            // level segments hold > kIsSmall elements each
    const int64_t cap_small = n / kIsThreshold + 16;  // one-wave segments hold > 16 each
    const int kMaxLevels = 128;
    int lg = 0;
    while (((int64_t)2 << lg) <= n) ++lg;  // std::__lg(n)
    const int depth = depth_limit >= 0 ? depth_limit : 2 * lg;
    // every level lowers the depth of all its segments, so depth + 1 levels bound the loop
    if (depth > kMaxLevels - 4) return ctx->fail(PITT_E_INVALID, "introsort: depth limit above 124");
    // grid barriers need every block resident: at most PITT_IS_COOP_MAX blocks (64), well under one
    // block per CU, each within the occupancy limit (checked once).  A plain launch: the cooperative
    // launch API measured ~3.5 ms of host-side cost per call.
    static int coop_blocks = 0;
    if (coop_blocks == 0) {
        int dev = 0, per_cu = 0;
        hipDeviceProp_t prop;
        PITT_HIP_TRY(hipGetDevice(&dev));
        PITT_HIP_TRY(hipGetDeviceProperties(&prop, dev));
        PITT_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_is_levels, kIsLvT, 0));
        if (per_cu < 1) return ctx->fail(PITT_E_NODEVICE, "introsort: level kernel does not fit a CU");
        PITT_HIP_TRY(hipFuncSetAttribute((const void*)k_is_heap, hipFuncAttributeMaxDynamicSharedMemorySize, kHeapLds * 6));
        coop_blocks = std::max(1, std::min(prop.multiProcessorCount * std::min(per_cu, 1), PITT_IS_COOP_MAX));
    }
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(coop_blocks, (n + kIsLvT - 1) / kIsLvT));
    const int64_t chunk = (n + G - 1) / G;
    ISeg* segA = (ISeg*)ctx->buf("is_segA", (size_t)cap * sizeof(ISeg));
    ISeg* segB = (ISeg*)ctx->buf("is_segB", (size_t)cap * sizeof(ISeg));
    ISeg* heapsegs = (ISeg*)ctx->buf("is_heapsegs", (size_t)cap * sizeof(ISeg));
    ISmall* small = (ISmall*)ctx->buf("is_small", (size_t)cap_small * sizeof(ISmall));
    int32_t* segid = (int32_t*)ctx->buf("is_segid", (size_t)n * 4);
    uint8_t* F = (uint8_t*)ctx->buf("is_F", (size_t)n);
    int32_t* SL = (int32_t*)ctx->buf("is_SL", (size_t)(n + 1) * 4);
    int32_t* SR = (int32_t*)ctx->buf("is_SR", (size_t)(n + 1) * 4);
    int32_t* posL = (int32_t*)ctx->buf("is_posL", (size_t)n * 4);
    int32_t* posR = (int32_t*)ctx->buf("is_posR", (size_t)n * 4);
    int32_t* bsum = (int32_t*)ctx->buf("is_bsum", (size_t)2 * 512 * 4);
    // cnt[0] heap segments, cnt[1] one-wave segments, cnt[2 + v] level v's segment count
    // cnt[kMaxLevels + 2]: the grid barrier's arrival counter
    int32_t* cnt = (int32_t*)ctx->buf("is_cnt", (size_t)(kMaxLevels + 4) * 4);
    int32_t* hcnt = (int32_t*)ctx->pinned("is_hcnt", 16);
    uint32_t* vtmp = (uint32_t*)ctx->buf("is_vtmp", (size_t)n * 4);
    if (!vtmp || !segA || !segB || !heapsegs || !small || !segid || !F || !SL || !SR || !posL || !posR || !bsum || !cnt ||
        !hcnt)
        return ctx->fail(PITT_E_NOMEM, "introsort scratch");
    PITT_HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)(kMaxLevels + 4) * 4, s));
    uint32_t* bar = (uint32_t*)(cnt + kMaxLevels + 2);
    const int32_t one = 1;
    const ISmall sroot = {0, (int32_t)n, depth, 0};
    ISeg root = {};
    root.f = 0;
    root.l = (int32_t)n;
    root.depth = depth;
    if (n <= kIsSmall) {
        PITT_HIP_TRY(hipMemcpyAsync(small, &sroot, sizeof sroot, hipMemcpyHostToDevice, s));
        PITT_HIP_TRY(hipMemcpyAsync(cnt + 1, &one, 4, hipMemcpyHostToDevice, s));
    } else {
        PITT_HIP_TRY(hipMemcpyAsync(segA, &root, sizeof root, hipMemcpyHostToDevice, s));
        PITT_HIP_TRY(hipMemcpyAsync(cnt + 2, &one, 4, hipMemcpyHostToDevice, s));
        PITT_HIP_TRY(hipMemsetAsync(segid, 0, (size_t)n * 4, s));
        hipLaunchKernelGGL(k_is_levels, dim3(G), dim3(kIsLvT), 0, s, segA, segB, heapsegs, small, cnt, segid, F, SL, SR,
                           posL, posR, bsum, key, val, n, chunk, depth + 1, bar);
    }
    PITT_HIP_TRY(hipMemcpyAsync(hcnt, cnt, 8, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));  // the host memcpys above read stack values: complete them too
    if (hcnt[1] > 0) hipLaunchKernelGGL(k_is_small, dim3(hcnt[1]), dim3(64), 0, s, small, cnt + 1, key, val);
    if (hcnt[0] > 0)
        hipLaunchKernelGGL(k_is_heap, dim3(hcnt[0]), dim3(256), kHeapLds * 6, s, heapsegs, cnt, key, val, vtmp);
    PITT_HIP_TRY(hipGetLastError());
    return PITT_OK;
}

}  // namespace pitt
