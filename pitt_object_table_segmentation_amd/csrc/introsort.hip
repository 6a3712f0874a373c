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
#define PITT_IS_SMALL 8192
#endif
constexpr int kIsSmall = PITT_IS_SMALL;  // segments this short finish in one block, in LDS
static_assert(kIsSmall % 256 == 0 && kIsSmall <= 65536, "block segments: whole 256-element windows, 16-bit positions");
#ifndef PITT_IS_MEDIUM
#define PITT_IS_MEDIUM 65536
#endif
constexpr int kIsMedium = PITT_IS_MEDIUM;  // segments this short are partitioned by one block (global memory)
static_assert(kIsMedium >= kIsSmall, "medium segments are longer than the block-in-LDS ones");
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

// children of <= 16 are final; children of <= kIsSmall go to the one-block (LDS) list, of <= kIsMedium to
// the one-block (global memory) list, larger ones to the next level
__device__ __forceinline__ int is_child(int f, int l, int d, ISeg* next, int32_t* next_cnt, ISmall* small,
                                        int32_t* small_cnt, ISmall* med, int32_t* med_cnt) {
    if (l - f <= kIsThreshold) return -1;
    if (l - f <= kIsSmall) {
        small[atomicAdd(small_cnt, 1)] = ISmall{f, l, d, 0};
        return -1;
    }
    if (l - f <= kIsMedium) {
        med[atomicAdd(med_cnt, 1)] = ISmall{f, l, d, 0};
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
// cnt[0] heap segments, cnt[1] block (LDS) segments, cnt[2 + v] level v's segments, cnt[kIsMaxLevels + 2]
// the grid barrier's arrival counter, cnt[kIsMedCnt] block (global memory) segments
constexpr int kIsMaxLevels = 128;
constexpr int kIsMedCnt = kIsMaxLevels + 3;
#ifdef PITT_IS_WATCHDOG
__device__ long long g_is_lvdbg[64 * 11];
#endif
constexpr int kIsLvW = kIsLvT / 64;

// Exclusive scan of two 0/1 flags over a kIsLvT-thread block; ta / tb = the block totals.  Inside a wave
// the ranks are ballot bit counts (no shuffle chain).
__device__ __forceinline__ void is_block_scan2(int a, int b, int& ea, int& eb, int& ta, int& tb, int* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t ma = __ballot(a), mb = __ballot(b);
    const int ia = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
    const int ib = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
    if (lane == 0) {
        sh[w] = __popcll(ma);
        sh[kIsLvW + w] = __popcll(mb);
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
    ea = oa + ia;
    eb = ob + ib;
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
                                                   ISmall* __restrict__ med,
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
#ifdef PITT_IS_WATCHDOG
    long long tb[5], ta[5], t_lv = clock64();
    int nlv = 0;
#endif
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
#ifdef PITT_IS_WATCHDOG
        tb[0] = clock64();
#endif
        is_grid_sync(bar, target);
#ifdef PITT_IS_WATCHDOG
        ta[0] = clock64();
#endif
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
#ifdef PITT_IS_WATCHDOG
        tb[1] = clock64();
#endif
        is_grid_sync(bar, target);
#ifdef PITT_IS_WATCHDOG
        ta[1] = clock64();
#endif
        // 4 stop positions; stop counts.  Global ranks = block-local rank + the prefix of the block
        // totals (every block forms the prefix itself: no separate pass)
        for (int j = tid; j < G; j += kIsLvT) {  // the block totals into LDS, then each prefix from LDS
            preL[j + 1] = bsum[j];
            preR[j + 1] = bsum[G + j];
        }
        __syncthreads();
        int pa = 0, pr2 = 0;
        if (tid <= G) {
            for (int q = 1; q <= tid; ++q) pa += preL[q], pr2 += preR[q];
        }
        __syncthreads();
        if (tid <= G) {
            preL[tid] = pa;
            preR[tid] = pr2;
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
#ifdef PITT_IS_WATCHDOG
        tb[2] = clock64();
#endif
        is_grid_sync(bar, target);
#ifdef PITT_IS_WATCHDOG
        ta[2] = clock64();
#endif
        // 5 K: one wave per segment, a 64-way search (posL[k] < posR[k] holds on a prefix of k; every k
        // below lo holds it, and K <= hi)
        for (int64_t s = gt >> 6; s < nseg; s += gstride >> 6) {
            const ISeg g = cur[s];
            if (!g.active) continue;
            const int bb = g.f + 1;
            int lo = 0, hi = min(g.nL, g.nR);
            while (lo < hi) {
                const int step = (hi - lo + 63) >> 6;
                const int k = lo + step * (tid & 63);
                const bool fail = k < hi && !(posL[bb + k] < posR[bb + k]);
                const uint64_t fm = __ballot(fail);
                if (fm == 0) {  // every probe below hi held: so does every k up to the last one
                    const int np = (hi - lo + step - 1) / step;
                    lo = lo + (np - 1) * step + 1;
                } else {
                    const int f0 = __builtin_ctzll(fm);
                    hi = lo + step * f0;              // a failing k
                    if (f0 > 0) lo = lo + step * (f0 - 1) + 1;  // the probe before it held
                }
            }
            if ((tid & 63) == 0) cur[s].K = lo;
        }
#ifdef PITT_IS_WATCHDOG
        tb[3] = clock64();
#endif
        is_grid_sync(bar, target);
#ifdef PITT_IS_WATCHDOG
        ta[3] = clock64();
#endif
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
            cur[s].childL = is_child(g.f, cut, g.depth - 1, nxt, cnt + 3 + v, small, cnt + 1, med, cnt + kIsMedCnt);
            cur[s].childR = is_child(cut, g.l, g.depth - 1, nxt, cnt + 3 + v, small, cnt + 1, med, cnt + kIsMedCnt);
        }
#ifdef PITT_IS_WATCHDOG
        tb[4] = clock64();
#endif
        is_grid_sync(bar, target);
#ifdef PITT_IS_WATCHDOG
        ta[4] = clock64();
#endif
#ifdef PITT_IS_WATCHDOG
        if (b == 0 && tid == 0 && v < 64) {  // printed after the last level (a printf here would stall the grid)
            long long* d = g_is_lvdbg + v * 11;
            d[0] = nseg;
            d[1] = tb[0] - t_lv;
            for (int q = 1; q < 5; ++q) d[1 + q] = tb[q] - ta[q - 1];
            for (int q = 0; q < 5; ++q) d[6 + q] = ta[q] - tb[q];
            nlv = v + 1;
        }
        t_lv = ta[4];
#endif
        ISeg* t = cur;  // phase 7 runs at the top of the next level, over nxt (= this level's segments)
        cur = nxt;
        nxt = t;
    }
#ifdef PITT_IS_WATCHDOG
    if (b == 0 && tid == 0)
        for (int v = 0; v < nlv; ++v) {
            const long long* d = g_is_lvdbg + v * 11;
            printf("is_levels v %d nseg %lld phases %lld %lld %lld %lld %lld barriers %lld %lld %lld %lld %lld\n", v, d[0], d[1],
                   d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], d[10]);
        }
#endif
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
// compiler barrier (no reordering of the accesses around it) is enough; the wave barrier (convergent)
// keeps every lane of the wave at this point together, so no lane runs ahead into the next step.
__device__ __forceinline__ void is_lds_fence() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

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
    const int nh = *heap_cnt;  // the count on the device: no host round trip before the launch
    for (int hi = blockIdx.x; hi < nh; hi += gridDim.x) {
        const ISeg g = segs[hi];
        const int len = g.l - g.f, tid = threadIdx.x;
        if (len > kHeapLds) {
            if (tid == 0) is_heap_sort(key + g.f, val + g.f, len);
            __syncthreads();
            continue;
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
        __syncthreads();  // the next segment reuses the LDS
    }
}

// One block finishes a segment of <= kIsSmall elements in LDS, kIsSmallW waves working on disjoint
// sub-segments at once: the same median / unguarded-partition / depth / heapsort steps as the level
// kernels, one partition per wave at a time.  A wave takes a segment from the block's queue, partitions
// it, queues the right part and goes on with the left one, as __introsort_loop recurses; the segments
// in flight are disjoint, so each wave's stores touch only its own range (and its own range of pl /
// pr).  Queue: slot j of a circular list holds the j-th queued segment once ready[j % cap] == j + 1;
// `open` counts the segments queued and not yet finished (head, tail and open count in units of 64,
// see is_wave_inc), so a wave whose slot stays empty while open is 0 is done (a queued segment stays
// open until the wave that took its slot finishes it).
constexpr int kIsSmallW = 8;  // waves per block
// segments in flight are disjoint and longer than 16: fewer than kIsSmall / 17 + kIsSmallW at once
constexpr int kIsQCap = kIsSmall / (kIsThreshold + 1) + kIsSmallW < 256 ? 256 : kIsSmall / (kIsThreshold + 1) + kIsSmallW < 512 ? 512 : 1024;
static_assert(kIsSmall / (kIsThreshold + 1) + kIsSmallW < kIsQCap, "introsort queue too short");

struct IsQueue {
    int head, tail, open;
    int ready[kIsQCap];
    int f[kIsQCap], l[kIsQCap], depth[kIsQCap];
};

__device__ __forceinline__ int is_lds_add(int* p, int v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The queue counters count in units of 64: every lane of the wave adds 1 (wave-uniform control flow
// and a uniform operand, which the compiler folds into one ds_add of 64; a lane-0-only add either
// needs a lane-conditional branch, around which the compiler may let some lanes run ahead of the
// readfirstlane broadcasts, or a per-lane operand, which it serialises over the 64 lanes).  Returns
// the old count, broadcast, in queue entries.
__device__ __forceinline__ int is_wave_inc(int* p) {
    return __builtin_amdgcn_readfirstlane(is_lds_add(p, 1)) >> 6;
}

__device__ __forceinline__ int is_wave_load(int* p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}

// queues [f, l) at depth d (open first: the pushing wave's own segment keeps open above 0); every lane
// stores the same values
__device__ __forceinline__ void is_queue_push(IsQueue& Q, int f, int l, int d) {
    is_lds_add(&Q.open, 1);
    const int j = is_wave_inc(&Q.tail);
    const int s = j & (kIsQCap - 1);
    Q.f[s] = f;
    Q.l[s] = l;
    Q.depth[s] = d;
    __hip_atomic_store(&Q.ready[s], j + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Partition [f, l) (> 16 elements, depth left) in place by one wave; returns the cut.  One forward
// pass over 16-byte aligned 256-element windows (lane: four consecutive keys, one ds_read_b128) ranks
// both kinds of stops: left stops (key >= p) ascending into pl, right stops (key <= p) ascending into pr,
// so the k-th right stop from the end is pr[nR - 1 - k].  Positions are 16-bit (kIsSmall <= 65536).
__device__ __forceinline__ int is_partition_wave(uint32_t* sk, uint32_t* sv, uint16_t* pl, uint16_t* pr, int f, int l,
                                                 int lane) {
    const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const uint32_t ka = sk[a], kb = sk[b], kc = sk[c];
    int m;
    if (ka < kb) m = (kb < kc) ? b : (ka < kc) ? c : a;
    else m = (ka < kc) ? a : (kb < kc) ? c : b;
    {  // every lane swaps (the same values): no lane-conditional branch
        const uint32_t tk = sk[f], tv = sv[f], mk = sk[m], mv = sv[m];
        is_lds_fence();
        sk[f] = mk;
        sv[f] = mv;
        sk[m] = tk;
        sv[m] = tv;
    }
    is_lds_fence();
    const uint32_t p = sk[f];
    uint16_t* L = pl + f;
    uint16_t* Rs = pr + f;
    int nL = 0, nR = 0;
    for (int w = (f + 1) & ~3; w < l; w += 256) {
        const int g0 = w + 4 * lane;
        uint4 q = make_uint4(0u, 0u, 0u, 0u);
        if (g0 < l) q = *reinterpret_cast<const uint4*>(sk + g0);
        const uint32_t kk[4] = {q.x, q.y, q.z, q.w};
        bool fl[4], fr[4];
        uint64_t BL[4], BR[4];
        int below_l = 0, below_r = 0, tot_l = 0, tot_r = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = g0 + j;
            const bool in = i > f && i < l;
            fl[j] = in && !(kk[j] < p);
            fr[j] = in && !(p < kk[j]);
            BL[j] = __ballot(fl[j]);
            BR[j] = __ballot(fr[j]);
            below_l += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(BL[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)BL[j], 0u));
            below_r += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(BR[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)BR[j], 0u));
            tot_l += __popcll(BL[j]);
            tot_r += __popcll(BR[j]);
        }
        int rl = nL + below_l, rr = nR + below_r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (fl[j]) L[rl] = (uint16_t)(g0 + j);
            if (fr[j]) Rs[rr] = (uint16_t)(g0 + j);
            rl += fl[j];
            rr += fr[j];
        }
        nL += tot_l;
        nR += tot_r;
    }
    is_lds_fence();
    const int kmax = min(nL, nR);
    int K = kmax;  // the swaps run while the k-th left stop lies left of the k-th right stop (from the end)
    for (int k0 = 0; k0 < kmax; k0 += 64) {
        const int k = k0 + lane;
        const uint64_t bal = __ballot(k < kmax && !((int)L[k] < (int)Rs[nR - 1 - k]));
        if (bal) {
            K = k0 + __builtin_ctzll(bal);
            break;
        }
    }
    for (int k = lane; k < K; k += 64) {
        const int x = L[k], y = Rs[nR - 1 - k];
        const uint32_t tk = sk[x], tv = sv[x];
        sk[x] = sk[y];
        sv[x] = sv[y];
        sk[y] = tk;
        sv[y] = tv;
    }
    const int cut = K < nL ? (K > 0 ? min((int)L[K], (int)Rs[nR - K]) : (int)L[K]) : (int)Rs[nR - K];
    is_lds_fence();
    return __builtin_amdgcn_readfirstlane(cut);
}

__global__ __launch_bounds__(64 * kIsSmallW) void k_is_small(const ISmall* __restrict__ segs,
                                                              const int32_t* __restrict__ small_cnt,
                                                              uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
    __shared__ __attribute__((aligned(16))) uint32_t sk[kIsSmall];
    __shared__ uint32_t sv[kIsSmall];
    __shared__ uint16_t pl[kIsSmall], pr[kIsSmall];
    __shared__ IsQueue Q;
    const int ns = *small_cnt;  // the count on the device: no host round trip before the launch
    for (int si = blockIdx.x; si < ns; si += gridDim.x) {
        const ISmall g = segs[si];
        const int lane = threadIdx.x & 63;
        const int len = g.l - g.f;
        for (int i = threadIdx.x; i < len; i += 64 * kIsSmallW) {
            sk[i] = key[g.f + i];
            sv[i] = val[g.f + i];
        }
        for (int i = threadIdx.x; i < kIsQCap; i += 64 * kIsSmallW) Q.ready[i] = 0;
        if (threadIdx.x == 0) {
            Q.head = Q.tail = Q.open = 0;
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // the whole segment is the first queued one (counts in units of 64)
            Q.open = 64;
            Q.tail = 64;
            Q.f[0] = 0;
            Q.l[0] = len;
            Q.depth[0] = g.depth;
            Q.ready[0] = 1;
        }
        __syncthreads();
#ifdef PITT_IS_WATCHDOG
        __shared__ unsigned long long dbg_busy, dbg_max, dbg_parts, dbg_elems, dbg_spins, dbg_wait;
        if (threadIdx.x == 0) dbg_busy = dbg_max = dbg_parts = dbg_elems = dbg_spins = dbg_wait = 0;
        __syncthreads();
        const long long t_start = clock64();
        unsigned long long w_busy = 0, w_parts = 0, w_elems = 0, w_spins = 0, w_wait = 0;
#endif
        for (;;) {
#ifdef PITT_IS_WATCHDOG
            const long long tw = clock64();
#endif
            const int j = is_wave_inc(&Q.head);
            const int s = j & (kIsQCap - 1);
            bool got = false;
#ifdef PITT_IS_WATCHDOG
            unsigned spins = 0;
#endif
            for (;;) {
                if (is_wave_load(&Q.ready[s]) == j + 1) {
                    got = true;
                    break;
                }
                // open == 0: every queued segment is finished, and slot j was never filled (its segment would
                // stay open until this wave finished it)
                if (is_wave_load(&Q.open) == 0) break;
                // no s_sleep: a sleeping wave wakes far too late for the next queued segment (the tree's
                // partitions are short), and a polling wave issues one LDS read per round trip
#ifdef PITT_IS_WATCHDOG
                ++w_spins;
                if (++spins == (1u << 20)) {
                    if (lane == 0)
                        printf("is_small watchdog: block %d wave %d slot %d head %d tail %d open %d len %d\n",
                               (int)blockIdx.x, (int)(threadIdx.x >> 6), j, Q.head, Q.tail, Q.open, len);
                    break;
                }
#endif
            }
#ifdef PITT_IS_WATCHDOG
            w_wait += clock64() - tw;
#endif
            if (!got) break;
            int f = __builtin_amdgcn_readfirstlane(Q.f[s]);
            int l = __builtin_amdgcn_readfirstlane(Q.l[s]);
            int depth = __builtin_amdgcn_readfirstlane(Q.depth[s]);
#ifdef PITT_IS_WATCHDOG
            int iters = 0;
#endif
            while (l - f > kIsThreshold) {
#ifdef PITT_IS_WATCHDOG
                if (++iters > 4096) {
                    if (lane == 0) printf("is_small spine watchdog: block %d f %d l %d depth %d\n", (int)blockIdx.x, f, l, depth);
                    break;
                }
#endif
                if (depth == 0) {
                    is_make_heap_lds<64>(sk + f, sv + f, l - f, lane);
                    is_sort_heap_wave(sk + f, sv + f, l - f, lane);
                    break;
                }
                --depth;
#ifdef PITT_IS_WATCHDOG
                const long long t0 = clock64();
                const int cut = is_partition_wave(sk, sv, pl, pr, f, l, lane);
                w_busy += clock64() - t0;
                ++w_parts;
                w_elems += l - f;
#else
                const int cut = is_partition_wave(sk, sv, pl, pr, f, l, lane);
#endif
                if (l - cut > kIsThreshold) is_queue_push(Q, cut, l, depth);  // __introsort_loop(cut, last, depth)
                l = cut;
            }
            is_lds_fence();
            __hip_atomic_fetch_add(&Q.open, -1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);  // -64: finished
        }
#ifdef PITT_IS_WATCHDOG
        if (lane == 0) {
            atomicAdd(&dbg_busy, w_busy);
            atomicMax(&dbg_max, w_busy);
            atomicAdd(&dbg_parts, w_parts);
            atomicAdd(&dbg_elems, w_elems);
            atomicAdd(&dbg_spins, w_spins);
            atomicAdd(&dbg_wait, w_wait);
        }
        __syncthreads();
        if (threadIdx.x == 0 && blockIdx.x < 12)
            printf("is_small block %d len %d cycles %lld busy %llu maxwave %llu parts %llu elems %llu spins %llu wait %llu\n",
                   (int)blockIdx.x, len, clock64() - t_start, dbg_busy, dbg_max, dbg_parts, dbg_elems, dbg_spins, dbg_wait);
#endif
        __syncthreads();
        for (int i = threadIdx.x; i < len; i += 64 * kIsSmallW) {
            key[g.f + i] = sk[i];
            val[g.f + i] = sv[i];
        }
        __syncthreads();  // the next segment reuses the LDS
    }
}

// One 1024-thread block partitions a segment of <= kIsMedium elements in global memory (L2-resident, no
// grid barrier) with the level kernel's steps, one partition at a time: the left stops and the right stops
// are ranked in one pass (block scans of ballots, a running total), posL[f + 1 + k] = the k-th left stop
// and posR[f + 1 + k] = the k-th right stop ascending (the k-th from the end is posR[f + nR - k]); wave 0
// finds the swap count by a 64-way search; the block swaps.  The block goes on with the left part and
// stacks the right one while they are longer than kIsSmall; shorter ones go to the block (LDS) list, and
// a part whose depth runs out to the heap list.
constexpr int kIsMdT = 1024;
constexpr int kIsMdRows = 8;  // rows of kIsMdT elements per step of the medium kernel's stop ranking
__global__ __launch_bounds__(kIsMdT) void k_is_medium(const ISmall* __restrict__ segs, const int32_t* __restrict__ med_cnt,
                                                      ISmall* __restrict__ small, int32_t* __restrict__ small_cnt,
                                                      ISeg* __restrict__ heap, int32_t* __restrict__ heap_cnt,
                                                      uint32_t* __restrict__ key, uint32_t* __restrict__ val,
                                                      int32_t* __restrict__ posL, int32_t* __restrict__ posR) {
    __shared__ int mdL[kIsMdRows * kIsLvW], mdR[kIsMdRows * kIsLvW];
    __shared__ int stk[3 * 128];
    __shared__ int bc[2];
    const int tid = threadIdx.x;
    const int nm = *med_cnt;
    for (int mi = blockIdx.x; mi < nm; mi += gridDim.x) {
        const ISmall g0 = segs[mi];
        int sp = 0, f = g0.f, l = g0.l, depth = g0.depth;
        for (;;) {
            while (l - f > kIsSmall) {
                if (depth == 0) {  // std::__partial_sort of this part
                    if (tid == 0) {
                        ISeg h = {};
                        h.f = f;
                        h.l = l;
                        heap[atomicAdd(heap_cnt, 1)] = h;
                    }
                    l = f;  // nothing left of it here
                    break;
                }
                --depth;
                if (tid == 0) {  // median of (first + 1, mid, last - 1) to first
                    const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
                    const uint32_t ka = key[a], kb = key[b], kc = key[c];
                    int m;
                    if (ka < kb) m = (kb < kc) ? b : (ka < kc) ? c : a;
                    else m = (ka < kc) ? a : (kb < kc) ? c : b;
                    is_swap(key, val, f, m);
                    bc[0] = (int)key[f];
                }
                __syncthreads();
                const uint32_t p = (uint32_t)bc[0];
                int nL = 0, nR = 0;  // block-uniform running totals
                const int lane = tid & 63, w = tid >> 6;
                for (int base = f + 1; base < l; base += kIsMdT * kIsMdRows) {
                    // kIsMdRows rows of 1024 elements: every key load issued first, then per row and wave the
                    // ballot ranks, one exchange of the (row, wave) totals through LDS
                    uint32_t kk[kIsMdRows];
#pragma unroll
                    for (int u = 0; u < kIsMdRows; ++u) {
                        const int i = base + u * kIsMdT + tid;
                        kk[u] = i < l ? key[i] : 0u;
                    }
                    uint64_t bl[kIsMdRows], br[kIsMdRows];
#pragma unroll
                    for (int u = 0; u < kIsMdRows; ++u) {
                        const bool in = base + u * kIsMdT + tid < l;
                        bl[u] = __ballot(in && !(kk[u] < p));
                        br[u] = __ballot(in && !(p < kk[u]));
                        if (lane == 0) {
                            mdL[u * kIsLvW + w] = __popcll(bl[u]);
                            mdR[u * kIsLvW + w] = __popcll(br[u]);
                        }
                    }
                    __syncthreads();
                    int offL = nL, offR = nR;  // exclusive prefix in (row, wave) order, then the totals
                    int totL = 0, totR = 0;
#pragma unroll
                    for (int u = 0; u < kIsMdRows; ++u) {
                        int rl = 0, rr = 0, sl = 0, sr = 0;
#pragma unroll
                        for (int q = 0; q < kIsLvW; ++q) {
                            const int a = mdL[u * kIsLvW + q], b2 = mdR[u * kIsLvW + q];
                            rl += q < w ? a : 0;
                            rr += q < w ? b2 : 0;
                            sl += a;
                            sr += b2;
                        }
                        const int i = base + u * kIsMdT + tid;
                        const uint32_t lo32 = (uint32_t)bl[u], hi32 = (uint32_t)(bl[u] >> 32);
                        const uint32_t rlo = (uint32_t)br[u], rhi = (uint32_t)(br[u] >> 32);
                        if ((bl[u] >> lane) & 1ull)
                            posL[f + 1 + offL + totL + rl + (int)__builtin_amdgcn_mbcnt_hi(hi32, __builtin_amdgcn_mbcnt_lo(lo32, 0u))] = i;
                        if ((br[u] >> lane) & 1ull)
                            posR[f + 1 + offR + totR + rr + (int)__builtin_amdgcn_mbcnt_hi(rhi, __builtin_amdgcn_mbcnt_lo(rlo, 0u))] = i;
                        totL += sl;
                        totR += sr;
                    }
                    nL += totL;
                    nR += totR;
                    __syncthreads();  // mdL / mdR are read before the next rows overwrite them
                }
                const int32_t* L = posL + f + 1;
                const int32_t* R = posR + f + nR;  // R[-k]: the k-th right stop from the end
                if (tid < 64) {  // the swap count: posL[k] < the k-th right stop from the end holds on a prefix
                    int lo = 0, hi = min(nL, nR);
                    while (lo < hi) {
                        const int step = (hi - lo + 63) >> 6;
                        const int k = lo + step * tid;
                        const uint64_t fm = __ballot(k < hi && !(L[k] < R[-k]));
                        if (fm == 0) {
                            lo = lo + ((hi - lo + step - 1) / step - 1) * step + 1;
                        } else {
                            const int f0 = __builtin_ctzll(fm);
                            hi = lo + step * f0;
                            if (f0 > 0) lo = lo + step * (f0 - 1) + 1;
                        }
                    }
                    if (tid == 0) bc[1] = lo;
                }
                __syncthreads();
                const int K = bc[1];
                for (int k0 = tid; k0 < K; k0 += kIsMdT * 4) {  // disjoint pairs; 4 per thread, loads first
                    int x[4], y[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int k = k0 + u * kIsMdT;
                        x[u] = k < K ? L[k] : 0;
                        y[u] = k < K ? R[-k] : 0;
                    }
                    uint32_t kx[4], vx[4], ky[4], vy[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (k0 + u * kIsMdT < K) {
                            kx[u] = key[x[u]];
                            vx[u] = val[x[u]];
                            ky[u] = key[y[u]];
                            vy[u] = val[y[u]];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (k0 + u * kIsMdT < K) {
                            key[x[u]] = ky[u];
                            val[x[u]] = vy[u];
                            key[y[u]] = kx[u];
                            val[y[u]] = vx[u];
                        }
                    }
                }
                const int cut = K < nL ? (K > 0 ? min(L[K], R[-(K - 1)]) : L[K]) : R[-(K - 1)];
                __syncthreads();  // the swaps are done (and bc is free again)
                if (l - cut > kIsSmall) {  // __introsort_loop(cut, last, depth): stacked
                    if (tid == 0) {
                        stk[3 * sp] = cut;
                        stk[3 * sp + 1] = l;
                        stk[3 * sp + 2] = depth;
                    }
                    ++sp;
                } else if (l - cut > kIsThreshold && tid == 0) {
                    small[atomicAdd(small_cnt, 1)] = ISmall{cut, l, depth, 0};
                }
                l = cut;
            }
            if (l - f > kIsThreshold && tid == 0) small[atomicAdd(small_cnt, 1)] = ISmall{f, l, depth, 0};
            __syncthreads();  // the stack entry written by thread 0
            if (sp == 0) break;
            --sp;
            f = stk[3 * sp];
            l = stk[3 * sp + 1];
            depth = stk[3 * sp + 2];
            __syncthreads();
        }
    }
}

// The first segment (the whole array) and its count, written on the device.
__global__ void k_is_root(ISeg* __restrict__ seg, ISmall* __restrict__ small, ISmall* __restrict__ med,
                          int32_t* __restrict__ cnt, int32_t n, int32_t depth) {
    if (n <= kIsSmall) {
        small[0] = ISmall{0, n, depth, 0};
        cnt[1] = 1;
    } else if (n <= kIsMedium) {
        med[0] = ISmall{0, n, depth, 0};
        cnt[kIsMedCnt] = 1;
    } else {
        ISeg r = {};
        r.f = 0;
        r.l = n;
        r.depth = depth;
        seg[0] = r;
        cnt[2] = 1;
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
    const int kMaxLevels = kIsMaxLevels;
    const int64_t cap_med = n / kIsSmall + 16;  // block (global memory) segments hold > kIsSmall each
    int lg = 0;
    while (((int64_t)2 << lg) <= n) ++lg;  // std::__lg(n)
    const int depth = depth_limit >= 0 ? depth_limit : 2 * lg;
    // every level lowers the depth of all its segments, so depth + 1 levels bound the loop
    if (depth > kMaxLevels - 4) return ctx->fail(PITT_E_INVALID, "introsort: depth limit above 124");
    // grid barriers need every block resident: at most PITT_IS_COOP_MAX blocks (64), well under one
    // block per CU, each within the occupancy limit (checked once).  A plain launch: the cooperative
    // launch API measured ~3.5 ms of host-side cost per call.
    static int coop_blocks = 0, cu_count = 0;
    if (coop_blocks == 0) {
        int dev = 0, per_cu = 0;
        hipDeviceProp_t prop;
        PITT_HIP_TRY(hipGetDevice(&dev));
        PITT_HIP_TRY(hipGetDeviceProperties(&prop, dev));
        PITT_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_is_levels, kIsLvT, 0));
        if (per_cu < 1) return ctx->fail(PITT_E_NODEVICE, "introsort: level kernel does not fit a CU");
        PITT_HIP_TRY(hipFuncSetAttribute((const void*)k_is_heap, hipFuncAttributeMaxDynamicSharedMemorySize, kHeapLds * 6));
        coop_blocks = std::max(1, std::min(prop.multiProcessorCount * std::min(per_cu, 1), PITT_IS_COOP_MAX));
        cu_count = prop.multiProcessorCount;
    }
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(coop_blocks, (n + kIsLvT - 1) / kIsLvT));
    const int64_t chunk = (n + G - 1) / G;
    ISeg* segA = (ISeg*)ctx->buf("is_segA", (size_t)cap * sizeof(ISeg));
    ISeg* segB = (ISeg*)ctx->buf("is_segB", (size_t)cap * sizeof(ISeg));
    ISeg* heapsegs = (ISeg*)ctx->buf("is_heapsegs", (size_t)cap * sizeof(ISeg));
    ISmall* small = (ISmall*)ctx->buf("is_small", (size_t)cap_small * sizeof(ISmall));
    ISmall* med = (ISmall*)ctx->buf("is_med", (size_t)cap_med * sizeof(ISmall));
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
    uint32_t* vtmp = (uint32_t*)ctx->buf("is_vtmp", (size_t)n * 4);
    if (!vtmp || !segA || !segB || !heapsegs || !small || !med || !segid || !F || !SL || !SR || !posL || !posR || !bsum ||
        !cnt)
        return ctx->fail(PITT_E_NOMEM, "introsort scratch");
    PITT_HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)(kMaxLevels + 4) * 4, s));
    uint32_t* bar = (uint32_t*)(cnt + kMaxLevels + 2);
    hipLaunchKernelGGL(k_is_root, dim3(1), dim3(1), 0, s, segA, small, med, cnt, (int32_t)n, depth);
    if (n > kIsMedium) {
        PITT_HIP_TRY(hipMemsetAsync(segid, 0, (size_t)n * 4, s));
        hipLaunchKernelGGL(k_is_levels, dim3(G), dim3(kIsLvT), 0, s, segA, segB, heapsegs, small, med, cnt, segid, F, SL,
                           SR, posL, posR, bsum, key, val, n, chunk, depth + 1, bar);
    }
    if (n > kIsSmall) {
        const int med_grid = (int)std::max<int64_t>(1, std::min<int64_t>(cap_med, cu_count));
        hipLaunchKernelGGL(k_is_medium, dim3(med_grid), dim3(kIsMdT), 0, s, med, cnt + kIsMedCnt, small, cnt + 1, heapsegs,
                           cnt, key, val, posL, posR);
    }
    // the block and heap segments: grids sized for their bounds, every block looping over the counts the
    // level kernel left on the device (no host round trip)
    const int small_grid = (int)std::max<int64_t>(1, std::min<int64_t>(cap_small, cu_count));
    const int heap_grid = (int)std::max<int64_t>(1, std::min<int64_t>(cap, 32));
    hipLaunchKernelGGL(k_is_small, dim3(small_grid), dim3(64 * kIsSmallW), 0, s, small, cnt + 1, key, val);
    if (n > kIsSmall)
        hipLaunchKernelGGL(k_is_heap, dim3(heap_grid), dim3(256), kHeapLds * 6, s, heapsegs, cnt, key, val, vtmp);
    PITT_HIP_TRY(hipGetLastError());
    return PITT_OK;
}

// __final_insertion_sort after the partitions: every segment the partitions leave unsorted holds at most
// kIsThreshold (16) elements, and every element of a segment is <= every element of the next one, so a pair
// of positions more than 15 apart is already in (stable) order, and the stable order of the whole array
// puts element i at i + #{j in (i, i + 15] : key_j < key_i} - #{j in [i - 15, i) : key_j > key_i}.  One
// thread per element counts its window in LDS and scatters (key, value) to that position.
constexpr int kIsFinT = 256, kIsFinH = kIsThreshold - 1;
__global__ __launch_bounds__(kIsFinT) void k_is_final(const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                      int64_t n, uint32_t* __restrict__ ko, uint32_t* __restrict__ vo) {
    __shared__ uint32_t sk[kIsFinT + 2 * kIsFinH];
    const int64_t b0 = (int64_t)blockIdx.x * kIsFinT;
    for (int t = threadIdx.x; t < kIsFinT + 2 * kIsFinH; t += kIsFinT) {
        const int64_t j = b0 - kIsFinH + t;
        sk[t] = (j >= 0 && j < n) ? key[j] : 0u;
    }
    __syncthreads();
    const int64_t i = b0 + threadIdx.x;
    if (i >= n) return;
    const int c = threadIdx.x + kIsFinH;
    const uint32_t k = sk[c];
    int64_t pos = i;
#pragma unroll
    for (int d = 1; d <= kIsFinH; ++d) {
        pos += (i + d < n && sk[c + d] < k) ? 1 : 0;
        pos -= (i - d >= 0 && sk[c - d] > k) ? 1 : 0;
    }
    ko[pos] = k;
    vo[pos] = val[i];
}

// After introsort_partitions: std::sort's final order of (key, val) into (ko, vo).
int introsort_final(pitt_ctx* ctx, const uint32_t* key, const uint32_t* val, int64_t n, uint32_t* ko, uint32_t* vo) {
    if (n <= 0) return PITT_OK;
    const int64_t grid = (n + kIsFinT - 1) / kIsFinT;
    hipLaunchKernelGGL(k_is_final, dim3((unsigned)grid), dim3(kIsFinT), 0, ctx->stream, key, val, n, ko, vo);
    PITT_HIP_TRY(hipGetLastError());
    return PITT_OK;
}

}  // namespace pitt
