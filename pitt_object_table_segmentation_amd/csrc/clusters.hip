// clusters.hip -- EuclideanClusterExtraction (extractEuclideanClusters + sorted search::KdTree) on
// gfx950.  Replaces src/segmentation_services/cluster_segmentation_srv.cpp:57-69 (reference path).
//
// PCL grows a cluster by BFS over radius neighbours (FLANN L2_Simple: ((dx^2 + dy^2) + dz^2) < r^2
// in float, r^2 = (float)((double)tol_f * tol_f)), seeding clusters in ascending index order.
// Without duplicate points the clusters are exactly the connected components of that
// radius graph, and the seed of each is its smallest index.  Here:
//   k_cells ... k_scatter   hashed grid of cells of side tol / sqrt(3) (each cell a clique of the
//               radius graph), points grouped by cell
//   k_cell_union  union-find over CELLS: a cell pair within the 5x5x5 neighbourhood joins at its
//               first point pair closer than the radius (early exit), not per point pair
//   k_cell_roots / k_point_labels   component size and seed (smallest index), per-point labels;
//               kept-root compaction (ascending seeds = PCL discovery order)
//   host        std::sort(rbegin, rend, size <) -- the reference's own ordering call, so ties
//               and > 16 clusters order exactly as libstdc++ does it there
//   k_keys + bitonic sort of (slot << 32 | index): members ascending inside each cluster
//   k_sums      float sums in index order (the handler divides by n + 1, Q7)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#include "compact.hpp"
#include "ctx.hpp"
#include "xsum.hpp"

#pragma clang fp contract(off)

namespace pitt {

constexpr uint64_t kEmpty = ~0ull;

__device__ __forceinline__ uint64_t cell_key(int64_t cx, int64_t cy, int64_t cz) {
    return (uint64_t)(cx & 0x1FFFFF) | ((uint64_t)(cy & 0x1FFFFF) << 21) | ((uint64_t)(cz & 0x1FFFFF) << 42);
}
__device__ __forceinline__ uint32_t hash64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return (uint32_t)k;
}

__device__ __forceinline__ bool finite3(float x, float y, float z) {
    return isfinite(x) && isfinite(y) && isfinite(z);
}

// Grid origin: per-axis minimum over the FINITE points only (the oracle's and KdTreeFLANN's view:
// a point with an infinite or NaN coordinate is never indexed, so it must not move the origin --
// one -inf would otherwise overflow every cell index).  Grid-stride partial minima per block, then
// one block combines them (k_minxyz_final).
constexpr int kMinBlocks = 512;

// The finite points' bounds: part[6 b + k] = min (k < 3) / max (k >= 3) of coordinate k % 3.
__global__ __launch_bounds__(kBlock) void k_minxyz(const float* __restrict__ x, const float* __restrict__ y,
                                                   const float* __restrict__ z, int64_t n, float* __restrict__ part) {
    __shared__ float s[6][kBlock / 64];
    float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const float px = x[i], py = y[i], pz = z[i];
        if (finite3(px, py, pz)) {
            v[0] = fminf(v[0], px);
            v[1] = fminf(v[1], py);
            v[2] = fminf(v[2], pz);
            v[3] = fmaxf(v[3], px);
            v[4] = fmaxf(v[4], py);
            v[5] = fmaxf(v[5], pz);
        }
    }
    for (int d = 32; d >= 1; d >>= 1)
        for (int k = 0; k < 6; ++k) v[k] = k < 3 ? fminf(v[k], __shfl_xor(v[k], d, 64)) : fmaxf(v[k], __shfl_xor(v[k], d, 64));
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 6; ++k) s[k][w] = v[k];
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        float m = s[k][0];
        for (int i = 1; i < kBlock / 64; ++i) m = k < 3 ? fminf(m, s[k][i]) : fmaxf(m, s[k][i]);
        part[6 * blockIdx.x + k] = m;
    }
}

__global__ __launch_bounds__(64) void k_minxyz_final(const float* __restrict__ part, int nb, float* __restrict__ mn) {
    float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int i = threadIdx.x; i < nb; i += 64)
        for (int k = 0; k < 6; ++k) v[k] = k < 3 ? fminf(v[k], part[6 * i + k]) : fmaxf(v[k], part[6 * i + k]);
    for (int d = 32; d >= 1; d >>= 1)
        for (int k = 0; k < 6; ++k) v[k] = k < 3 ? fminf(v[k], __shfl_xor(v[k], d, 64)) : fmaxf(v[k], __shfl_xor(v[k], d, 64));
    if (threadIdx.x == 0)
        for (int k = 0; k < 6; ++k) mn[k] = v[k];
}

// ---- cell grid ---------------------------------------------------------------------------------
// Cells of side tol_f / sqrt(3) shrunk by 1e-4: two finite points in one cell are closer than
// tol (1 - 1e-4) -- far enough inside the radius that PCL's float test ((dx^2 + dy^2) + dz^2 < r^2)
// holds too -- so every cell is a clique of the radius graph.  A radius neighbour of a point lies
// at most two cells away on each axis (tol / cell < 1.7323), so the components of the point graph
// are the components of the cell graph whose edges are the cell pairs within that 5x5x5
// neighbourhood holding at least one point pair closer than the radius.
constexpr double kCellShrink = 1.0 - 1e-4;
constexpr int kCellBits = 21;
constexpr int64_t kCellSpan = ((int64_t)1 << kCellBits) - 8;  // grid coordinates (+2 neighbours) per axis

struct Grid {
    const float *x, *y, *z;
    const float* mn;
    double inv_cell;
    uint64_t* keys;   // [hsize] occupied cells' keys
    int32_t* hcid;    // [hsize] dense id of the cell in a slot
    uint32_t hmask;
};

__device__ __forceinline__ void cell_of(const Grid& g, int64_t i, int64_t& cx, int64_t& cy, int64_t& cz) {
    cx = (int64_t)floor(((double)g.x[i] - (double)g.mn[0]) * g.inv_cell);
    cy = (int64_t)floor(((double)g.y[i] - (double)g.mn[1]) * g.inv_cell);
    cz = (int64_t)floor(((double)g.z[i] - (double)g.mn[2]) * g.inv_cell);
}

__device__ __forceinline__ int32_t hash_find(const Grid& g, uint64_t key) {
    uint32_t h = hash64(key) & g.hmask;
    while (true) {
        const uint64_t k = g.keys[h];
        if (k == key) return (int32_t)h;
        if (k == kEmpty) return -1;
        h = (h + 1) & g.hmask;
    }
}

// Occupied cells into the hash; the inserting thread numbers the cell (dense id, any order) and
// records its key.  pslot[i] = the point's slot, -1 for a non-finite point (never indexed by
// KdTreeFLANN: a singleton).
__global__ void k_cells(Grid g, int64_t n, int32_t* __restrict__ pslot, int32_t* __restrict__ ncells,
                        uint64_t* __restrict__ ckey) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!finite3(g.x[i], g.y[i], g.z[i])) { pslot[i] = -1; continue; }
        int64_t cx, cy, cz;
        cell_of(g, i, cx, cy, cz);
        const uint64_t key = cell_key(cx, cy, cz);
        uint32_t h = hash64(key) & g.hmask;
        while (true) {
            const uint64_t prev = atomicCAS((unsigned long long*)&g.keys[h], (unsigned long long)kEmpty,
                                            (unsigned long long)key);
            if (prev == kEmpty) {
                const int32_t c = atomicAdd(ncells, 1);
                g.hcid[h] = c;
                ckey[c] = key;
                break;
            }
            if (prev == key) break;
            h = (h + 1) & g.hmask;
        }
        pslot[i] = (int32_t)h;
    }
}

// Per point: its cell id; per cell: point count and smallest point index.
__global__ void k_cell_count(const int32_t* __restrict__ pslot, int64_t n, const int32_t* __restrict__ hcid,
                             int32_t* __restrict__ pcid, int32_t* __restrict__ ccnt, int32_t* __restrict__ cmin) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t h = pslot[i];
        const int32_t c = h < 0 ? -1 : hcid[h];
        pcid[i] = c;
        if (c >= 0) {
            atomicAdd(&ccnt[c], 1);
            atomicMin(&cmin[c], (int32_t)i);
        }
    }
}

// Exclusive scan of the cells' counts (one 1024-thread block; the cell count is read on the device).
__global__ __launch_bounds__(1024) void k_cell_scan(const int32_t* __restrict__ ccnt, const int32_t* __restrict__ ncells,
                                                    int32_t* __restrict__ cstart) {
    __shared__ int32_t part[16];
    const int nc = *ncells;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int carry = 0;
    for (int base = 0; base < nc; base += 1024) {
        const int t = base + (int)threadIdx.x;
        const int v = t < nc ? ccnt[t] : 0;
        int inc = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(inc, d, 64);
            if (lane >= d) inc += o;
        }
        if (lane == 63) part[w] = inc;
        __syncthreads();
        int pre = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            pre += k < w ? part[k] : 0;
            tot += part[k];
        }
        if (t < nc) cstart[t] = carry + pre + inc - v;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) cstart[nc] = carry;
}

__global__ void k_scatter(const int32_t* __restrict__ pcid, int64_t n, const int32_t* __restrict__ cstart,
                          int32_t* __restrict__ cursor, int32_t* __restrict__ cpts) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t c = pcid[i];
        if (c < 0) continue;
        cpts[cstart[c] + atomicAdd(&cursor[c], 1)] = (int32_t)i;
    }
}

__device__ __forceinline__ int32_t uf_find(int32_t* parent, int32_t i) {
    int32_t p = __atomic_load_n(&parent[i], __ATOMIC_RELAXED);
    while (p != i) {
        const int32_t gp = __atomic_load_n(&parent[p], __ATOMIC_RELAXED);
        if (gp != p) __atomic_store_n(&parent[i], gp, __ATOMIC_RELAXED);  // path halving
        i = p;
        p = gp;
    }
    return i;
}

__device__ __forceinline__ void uf_union(int32_t* parent, int32_t a, int32_t b) {
    while (true) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a > b) { const int32_t t = a; a = b; b = t; }
        if (atomicCAS(&parent[b], b, a) == b) return;  // the larger root hooks under the smaller
    }
}

__global__ void k_cell_iota(int32_t* __restrict__ parent, const int32_t* __restrict__ ncells) {
    const int nc = *ncells;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += gridDim.x * blockDim.x) parent[c] = c;
}

// One wave per cell: against each of the 62 cells after it in the 5x5x5 neighbourhood (the other 62
// see it from their side), unless the two are already joined, look for one point pair closer than
// the radius (PCL's float order) and join the cells at the first such pair.  The 62 neighbours are
// looked up at once (lane o probes offset o); per neighbour its points are loaded 64 at a time (lane q
// holds point q) and walked by v_readlane against the cell's points (one per lane, loaded once per
// cell), eight at a time between ballots: no load waits inside the pair loop.
__global__ __launch_bounds__(256) void k_cell_union(Grid g, const int32_t* __restrict__ ncells,
                                                    const uint64_t* __restrict__ ckey, const int32_t* __restrict__ cstart,
                                                    const int32_t* __restrict__ cpts, float r2,
                                                    int32_t* __restrict__ parent) {
    const int nc = *ncells;
    const int lane = threadIdx.x & 63;
    const int nw = gridDim.x * 4;
    const float qnan = __builtin_nanf("");
    for (int c = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6))); c < nc; c += nw) {
        const uint64_t key = ckey[c];
        const int64_t cx = (int64_t)(key & 0x1FFFFF), cy = (int64_t)((key >> 21) & 0x1FFFFF), cz = (int64_t)(key >> 42);
        const int b0 = cstart[c], e0 = cstart[c + 1];
        // the neighbours: lane o < 62 probes offset 63 + o (the offsets after (0, 0, 0))
        int32_t d = -1;
        if (lane < 62) {
            const int o = 63 + lane;
            const int dx = o / 25 - 2, dy = (o / 5) % 5 - 2, dz = o % 5 - 2;
            if (cx + dx >= 0 && cy + dy >= 0 && cz + dz >= 0) {
                const int32_t h = hash_find(g, cell_key(cx + dx, cy + dy, cz + dz));
                if (h >= 0) d = g.hcid[h];
            }
        }
        uint64_t cand = __builtin_amdgcn_ballot_w64(d >= 0);
        if (!cand) continue;
        // the cell's first 64 points, one per lane (NaN past its end: never closer than the radius)
        float cx0 = qnan, cy0 = qnan, cz0 = qnan;
        if (b0 + lane < e0) {
            const int32_t i = cpts[b0 + lane];
            cx0 = g.x[i];
            cy0 = g.y[i];
            cz0 = g.z[i];
        }
        while (cand) {
            const int t = (int)__builtin_ctzll(cand);
            cand &= cand - 1;
            const int32_t dn = __builtin_amdgcn_readlane(d, t);
            if (uf_find(parent, c) == uf_find(parent, dn)) continue;
            const int b1 = cstart[dn], e1 = cstart[dn + 1];
            bool hit = false;
            for (int q0 = b1; q0 < e1 && !hit; q0 += 64) {
                float qx = qnan, qy = qnan, qz = qnan;
                if (q0 + lane < e1) {
                    const int32_t j = cpts[q0 + lane];
                    qx = g.x[j];
                    qy = g.y[j];
                    qz = g.z[j];
                }
                const int nq = __builtin_amdgcn_readfirstlane(e1 - q0 < 64 ? e1 - q0 : 64);
                for (int p0 = b0; p0 < e0 && !hit; p0 += 64) {
                    float px = cx0, py = cy0, pz = cz0;
                    if (p0 != b0) {  // cells of more than 64 points: the next 64
                        px = py = pz = qnan;
                        if (p0 + lane < e0) {
                            const int32_t i = cpts[p0 + lane];
                            px = g.x[i];
                            py = g.y[i];
                            pz = g.z[i];
                        }
                    }
                    for (int u0 = 0; u0 < nq && !hit; u0 += 8) {
                        bool any = false;
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            const int tt = u0 + u < nq ? u0 + u : nq - 1;  // a repeated pair changes nothing
                            const float bx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qx), tt));
                            const float by = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qy), tt));
                            const float bz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qz), tt));
                            const float ex = px - bx, ey = py - by, ez = pz - bz;
                            const float dd = ex * ex + ey * ey + ez * ez;  // FLANN L2_Simple order
                            any = any || dd < r2;
                        }
                        hit = __builtin_amdgcn_ballot_w64(any) != 0;
                    }
                }
            }
            if (hit && lane == 0) uf_union(parent, c, dn);
        }
    }
}

// Per cell: its points added to its root's size, its smallest index folded into the root's seed.  Cells
// of one wave that share a root (a large component: most of them) are reduced in the wave first, so a
// root takes one atomic per wave instead of one per cell.
__global__ void k_cell_roots(int32_t* __restrict__ parent, const int32_t* __restrict__ ncells,
                             const int32_t* __restrict__ ccnt, const int32_t* __restrict__ cmin,
                             int32_t* __restrict__ csize, int32_t* __restrict__ cseed) {
    const int nc = *ncells;
    const int lane = threadIdx.x & 63;
    for (int base = blockIdx.x * blockDim.x; base < nc; base += gridDim.x * blockDim.x) {  // uniform per wave
        const int c = base + (int)threadIdx.x;
        int32_t r = -1, cnt = 0, mn = INT_MAX;
        if (c < nc) {
            r = uf_find(parent, c);
            cnt = ccnt[c];
            mn = cmin[c];
        }
        uint64_t pend = __builtin_amdgcn_ballot_w64(c < nc);
        while (pend) {
            const int32_t r0 = __builtin_amdgcn_readlane(r, (int)__builtin_ctzll(pend));
            const bool mine = ((pend >> lane) & 1u) && r == r0;
            int sv = mine ? cnt : 0, mv = mine ? mn : INT_MAX;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                sv += __shfl_xor(sv, off, 64);
                const int o = __shfl_xor(mv, off, 64);
                mv = o < mv ? o : mv;
            }
            if (lane == 0) {
                atomicAdd(&csize[r0], sv);
                atomicMin(&cseed[r0], mv);
            }
            pend &= ~__builtin_amdgcn_ballot_w64(mine);
        }
    }
}

// Per point: label = its component's seed (a non-finite point is its own singleton); at a seed the
// component size.
__global__ void k_point_labels(const int32_t* __restrict__ pcid, int64_t n, int32_t* __restrict__ parent,
                               const int32_t* __restrict__ csize, const int32_t* __restrict__ cseed,
                               int32_t* __restrict__ label, int32_t* __restrict__ size) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t c = pcid[i];
        if (c < 0) {
            label[i] = (int32_t)i;
            size[i] = 1;
            continue;
        }
        const int32_t r = uf_find(parent, c);
        const int32_t sd = cseed[r];
        label[i] = sd;
        if (sd == (int32_t)i) size[i] = csize[r];
    }
}

struct KeptRoot {
    const int32_t* label;
    const int32_t* size;
    uint64_t mn, mx;
    __device__ bool operator()(int64_t i) const {
        if (label[i] != (int32_t)i) return false;
        const uint64_t s = (uint64_t)size[i];
        return s >= mn && s <= mx;
    }
};
struct WriteRoot {
    const int32_t* size;
    int32_t* roots;
    int32_t* sizes;
    __device__ void operator()(int64_t i, int64_t p) const {
        roots[p] = (int32_t)i;
        sizes[p] = size[i];
    }
};

__global__ void k_set_slots(const int32_t* __restrict__ roots, const int32_t* __restrict__ slots, int32_t k,
                            int32_t* __restrict__ rootslot) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < k; t += (int64_t)gridDim.x * blockDim.x)
        rootslot[roots[t]] = slots[t];
}

struct KeptPoint {
    const int32_t* label;
    const int32_t* rootslot;
    __device__ bool operator()(int64_t i) const { return rootslot[label[i]] >= 0; }
};
struct WriteKey {
    const int32_t* label;
    const int32_t* rootslot;
    uint64_t* keys;
    __device__ void operator()(int64_t i, int64_t p) const {
        keys[p] = ((uint64_t)(uint32_t)rootslot[label[i]] << 32) | (uint64_t)(uint32_t)i;
    }
};

// Bitonic sort of a power-of-two array of keys: LDS stages for j < 2048, global for larger j.
constexpr int kSortTile = 2048;
__global__ __launch_bounds__(1024) void k_bitonic_local(uint64_t* __restrict__ a, int64_t m, int kmax_local,
                                                        int64_t k_outer) {
    __shared__ uint64_t s[kSortTile];
    const int64_t base = (int64_t)blockIdx.x * kSortTile;
    for (int t = threadIdx.x; t < kSortTile; t += 1024) s[t] = a[base + t];
    __syncthreads();
    // k_outer == 0: full local sort (k = 2 .. kSortTile); else: merge steps j < kSortTile of stage k_outer
    for (int64_t k = (k_outer ? k_outer : 2); k <= (k_outer ? k_outer : (int64_t)kmax_local); k <<= 1) {
        for (int64_t j = (k_outer ? kSortTile / 2 : k / 2); j >= 1; j >>= 1) {
            for (int t = threadIdx.x; t < kSortTile; t += 1024) {
                const int64_t i = base + t;
                const int64_t l = i ^ j;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const uint64_t x = s[t], y = s[l - base];
                    if ((x > y) == up) { s[t] = y; s[l - base] = x; }
                }
            }
            __syncthreads();
        }
        if (k_outer) break;
    }
    for (int t = threadIdx.x; t < kSortTile; t += 1024) a[base + t] = s[t];
    (void)m;
}

__global__ void k_bitonic_global(uint64_t* __restrict__ a, int64_t m, int64_t k, int64_t j) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t l = i ^ j;
        if (l > i) {
            const bool up = (i & k) == 0;
            const uint64_t x = a[i], y = a[l];
            if ((x > y) == up) { a[i] = y; a[l] = x; }
        }
    }
}

__global__ void k_members(const uint64_t* __restrict__ keys, int64_t m, const float* __restrict__ x,
                          const float* __restrict__ y, const float* __restrict__ z, int32_t* __restrict__ idx,
                          float* __restrict__ cx, float* __restrict__ cy, float* __restrict__ cz) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < m; p += (int64_t)gridDim.x * blockDim.x) {
        const int32_t i = (int32_t)(keys[p] & 0xffffffffull);
        idx[p] = i;
        cx[p] = x[i];
        cy[p] = y[i];
        cz[p] = z[i];
    }
}

// Float sums in index order (cluster_segmentation_srv.cpp:88-90): one block per cluster.  Waves
// 1-3 stage 2048-element slices of x, y, z into a double-buffered LDS ring while lanes 0..2 of
// wave 0 run the three serial chains over the previous slice, 16 elements per unrolled step read
// as four float4 (the adds stay in index order: no reassociation).
constexpr int kSumChunk = 2048;

__global__ __launch_bounds__(256) void k_sums(const int64_t* __restrict__ coff, int32_t k, const float* __restrict__ cx,
                                              const float* __restrict__ cy, const float* __restrict__ cz,
                                              float* __restrict__ sums) {
    __shared__ float4 buf[2][3][kSumChunk / 4];
    const int c = blockIdx.x;
    if (c >= k) return;
    const int64_t b = coff[c], e = coff[c + 1];
    const int64_t nch = (e - b + kSumChunk - 1) / kSumChunk;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float s = 0.0f;
    for (int64_t i = 0; i <= nch; ++i) {
        if (w > 0 && i < nch) {  // stage slice i
            float* f = reinterpret_cast<float*>(buf[i & 1]);
            const int64_t i0 = b + i * kSumChunk;
            for (int t = (int)threadIdx.x - 64; t < kSumChunk; t += 192) {
                const int64_t j = i0 + t;
                const bool in = j < e;
                f[t] = in ? cx[j] : 0.0f;
                f[kSumChunk + t] = in ? cy[j] : 0.0f;
                f[2 * kSumChunk + t] = in ? cz[j] : 0.0f;
            }
        }
        if (w == 0 && lane < 3 && i > 0) {  // sum slice i - 1
            const float4* q = buf[(i - 1) & 1][lane];
            const int cnt = (int)min((int64_t)kSumChunk, e - (b + (i - 1) * kSumChunk));
            int t = 0;
            for (; t + 16 <= cnt; t += 16) {
                const float4 a0 = q[t / 4], a1 = q[t / 4 + 1], a2 = q[t / 4 + 2], a3 = q[t / 4 + 3];
                s = s + a0.x; s = s + a0.y; s = s + a0.z; s = s + a0.w;
                s = s + a1.x; s = s + a1.y; s = s + a1.z; s = s + a1.w;
                s = s + a2.x; s = s + a2.y; s = s + a2.z; s = s + a2.w;
                s = s + a3.x; s = s + a3.y; s = s + a3.z; s = s + a3.w;
            }
            const float* r = reinterpret_cast<const float*>(q);
            for (; t < cnt; ++t) s = s + r[t];
        }
        __syncthreads();
    }
    if (w == 0 && lane < 3) sums[3 * c + lane] = s;
}

static inline int ew(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096)); }

// Large member sets: the same float sums by the block-parallel exact walk (xsum.hpp).  The members'
// x, y, z are laid out as three streams with one 256-aligned segment per cluster (zeros past a
// cluster's end, which the walk never adds).
__global__ __launch_bounds__(256) void k_pad_members(const float* __restrict__ mxyz, int64_t M,
                                                     const int64_t* __restrict__ coff, const XsSeg* __restrict__ seg,
                                                     const int32_t* __restrict__ bseg, float* __restrict__ V, int64_t T) {
    const int64_t b = blockIdx.x;
    const int k = bseg[b];
    const XsSeg g = seg[k];
    const int64_t i = (b - g.blk0) * kXsBlk + threadIdx.x;
    const bool in = i < g.len;
#pragma unroll
    for (int s = 0; s < 3; ++s) V[s * T + b * kXsBlk + threadIdx.x] = in ? mxyz[s * M + coff[k] + i] : 0.0f;
}
constexpr int64_t kXsMinMembers = 16384;  // below: k_sums' three chains are short enough

template <class Pred, class Act>
static int compact(pitt_ctx* ctx, int64_t n, Pred pred, Act act, int64_t* total) {
    const int64_t nt = ctiles(n);
    int32_t* counts = (int32_t*)ctx->buf("cl_ccounts", (size_t)std::max<int64_t>(nt, 1) * 4);
    int32_t* offs = (int32_t*)ctx->buf("cl_coffs", (size_t)(nt + 1) * 4);
    if (!counts || !offs) return ctx->fail(PITT_E_NOMEM, "compaction scratch");
    hipStream_t s = ctx->stream;
    if (n > 0) hipLaunchKernelGGL((k_pred_count<Pred>), dim3(grid_for_tiles(nt)), dim3(kBlock), 0, s, pred, n, counts);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, counts, nt, offs);
    if (n > 0)
        hipLaunchKernelGGL((k_pred_apply<Pred, Act>), dim3(grid_for_tiles(nt)), dim3(kBlock), 0, s, pred, act, n, offs);
    PITT_HIP_TRY(hipGetLastError());
    int32_t* h = (int32_t*)ctx->pinned("cl_total", 16);
    PITT_HIP_TRY(hipMemcpyAsync(h, offs + nt, 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    *total = h[0];
    return PITT_OK;
}

// EuclideanClusterExtraction::extract (cluster_segmentation_srv.cpp:57-69).  x/y/z: host SoA, or
// device SoA when dev_in.  Results: host member lists into `out`, or the context's device buffer
// into `dout` (members at dout->indices[offset, offset + size)); the float sums come back to the host
// either way.
int euclidean_clusters_impl(pitt_ctx* ctx, const float* hx, const float* hy, const float* hz, int64_t n,
                            double tolerance, int32_t min_size, int32_t max_size, pitt_cluster_list* out,
                            pitt_cluster_list_dev* dout, bool dev_in, int aos_stride) {
    hipStream_t s = ctx->stream;
    ctx->keep_clusters.clear();
    ctx->keep_clusters_dev.clear();
    if (out) {
        out->n_clusters = 0;
        out->clusters = nullptr;
    }
    if (dout) {
        dout->n_clusters = 0;
        dout->clusters = nullptr;
        dout->indices = nullptr;
    }
    if (n == 0) return PITT_OK;  // extract(): empty input => no clusters
    const bool timing = ctx->host_timing && !dev_in;  // $PITT_HOST_TIMING=1: host phases on stderr
    const double tm0 = timing ? wall_ms() : 0.0;
    double tm_in = 0.0, tm_roots = 0.0;
    // KdTreeFLANN::radiusSearch: r^2 = (float)(radius * radius) with radius = (double)(float)tol
    const float tol_f = (float)tolerance;
    const float r2 = (float)((double)tol_f * (double)tol_f);
    const double cell = (double)tol_f * (1.0 / std::sqrt(3.0)) * kCellShrink;
    if (!(cell > 0.0) || !std::isfinite(cell)) return ctx->fail(PITT_E_INVALID, "tolerance must be > 0");
    uint32_t hsize = 1024;
    while ((int64_t)hsize < 2 * n) hsize <<= 1;
    const size_t N = (size_t)n;
    float* X = (float*)ctx->buf("cl_xyz", N * 3 * 4);
    float* MN = (float*)ctx->buf("cl_min", 64);
    uint64_t* KEYS = (uint64_t*)ctx->buf("cl_hkeys", (size_t)hsize * 8);
    int32_t* HCID = (int32_t*)ctx->buf("cl_hcid", (size_t)hsize * 4);
    uint64_t* CKEY = (uint64_t*)ctx->buf("cl_ckey", N * 8);
    int32_t* PSLOT = (int32_t*)ctx->buf("cl_pslot", N * 4);
    int32_t* PCID = (int32_t*)ctx->buf("cl_pcid", N * 4);
    // per-cell arrays (cells <= points): count, min index, start (+1), cursor, parent, size, seed
    int32_t* CELLS = (int32_t*)ctx->buf("cl_cells", (N * 7 + 16) * 4);
    int32_t* CPTS = (int32_t*)ctx->buf("cl_cpts", N * 4);
    int32_t* LABEL = (int32_t*)ctx->buf("cl_label", N * 4);
    int32_t* SIZE = (int32_t*)ctx->buf("cl_size", N * 4);
    int32_t* ROOTS = (int32_t*)ctx->buf("cl_roots", N * 4);
    int32_t* RSIZES = (int32_t*)ctx->buf("cl_rsizes", N * 4);
    int32_t* RSLOT = (int32_t*)ctx->buf("cl_rootslot", N * 4);
    if (!X || !MN || !KEYS || !HCID || !CKEY || !PSLOT || !PCID || !CELLS || !CPTS || !LABEL || !SIZE || !ROOTS ||
        !RSIZES || !RSLOT)
        return ctx->fail(PITT_E_NOMEM, "cluster scratch");
    int32_t* NCELLS = CELLS;                 // [1] (+ padding)
    int32_t* CCNT = CELLS + 16;              // [N]
    int32_t* CMIN = CCNT + N;                // [N]
    int32_t* CCUR = CMIN + N;                // [N]
    int32_t* CSIZE = CCUR + N;               // [N]
    int32_t* CSEED = CSIZE + N;              // [N]
    int32_t* CPAR = CSEED + N;               // [N]
    int32_t* CSTART = (int32_t*)ctx->buf("cl_cstart", (N + 1) * 4);
    if (!CSTART) return ctx->fail(PITT_E_NOMEM, "cluster scratch");
    float *Y = X + N, *Z = X + 2 * N;
    if (aos_stride) {  // the caller's host AoS cloud as it lies: one upload, deinterleaved on the device
        void* scr = ctx->buf("cl_aos", N * aos_stride);
        if (!scr) return ctx->fail(PITT_E_NOMEM, "cluster scratch");
        PITT_HIP_TRY(upload_aos(s, scr, hx, n, aos_stride, X, Y, Z));
    } else {
        const hipMemcpyKind kin = dev_in ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
        PITT_HIP_TRY(hipMemcpyAsync(X, hx, N * 4, kin, s));
        PITT_HIP_TRY(hipMemcpyAsync(Y, hy, N * 4, kin, s));
        PITT_HIP_TRY(hipMemcpyAsync(Z, hz, N * 4, kin, s));
    }
    if (timing) tm_in = wall_ms();
    PITT_HIP_TRY(hipMemsetAsync(KEYS, 0xFF, (size_t)hsize * 8, s));
    PITT_HIP_TRY(hipMemsetAsync(CELLS, 0, (N * 7 + 16) * 4, s));
    PITT_HIP_TRY(hipMemsetAsync(CMIN, 0x7F, N * 4, s));   // INT_MAX-ish: atomicMin seeds
    PITT_HIP_TRY(hipMemsetAsync(CSEED, 0x7F, N * 4, s));
    {
        const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, kMinBlocks));
        float* PART = (float*)ctx->buf("cl_minpart", (size_t)kMinBlocks * 6 * sizeof(float));
        if (!PART) return ctx->fail(PITT_E_NOMEM, "cluster scratch");
        hipLaunchKernelGGL(k_minxyz, dim3(nb), dim3(kBlock), 0, s, X, Y, Z, n, PART);
        hipLaunchKernelGGL(k_minxyz_final, dim3(1), dim3(64), 0, s, PART, nb, MN);
    }
    // the grid's extent must fit the 21-bit cell coordinates (else distinct cells would alias); the
    // bounds come from the device (k_minxyz), read back once
    {
        float* mm = (float*)ctx->pinned("cl_minmax_h", 64);
        PITT_HIP_TRY(hipMemcpyAsync(mm, MN, 24, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        for (int k = 0; k < 3; ++k)
            if (std::isfinite(mm[k]) && ((double)mm[3 + k] - (double)mm[k]) / cell >= (double)kCellSpan)
                return ctx->fail(PITT_E_INVALID, "cloud extent exceeds 2^21 cells of tolerance / sqrt(3)");
    }
    Grid g{X, Y, Z, MN, 1.0 / cell, KEYS, HCID, hsize - 1};
    hipLaunchKernelGGL(k_cells, dim3(ew(n)), dim3(256), 0, s, g, n, PSLOT, NCELLS, CKEY);
    hipLaunchKernelGGL(k_cell_count, dim3(ew(n)), dim3(256), 0, s, PSLOT, n, HCID, PCID, CCNT, CMIN);
    hipLaunchKernelGGL(k_cell_scan, dim3(1), dim3(1024), 0, s, CCNT, NCELLS, CSTART);
    hipLaunchKernelGGL(k_scatter, dim3(ew(n)), dim3(256), 0, s, PCID, n, CSTART, CCUR, CPTS);
    hipLaunchKernelGGL(k_cell_iota, dim3(ew(n)), dim3(256), 0, s, CPAR, NCELLS);
    hipLaunchKernelGGL(k_cell_union, dim3(ew(n)), dim3(256), 0, s, g, NCELLS, CKEY, CSTART, CPTS, r2, CPAR);
    hipLaunchKernelGGL(k_cell_roots, dim3(ew(n)), dim3(256), 0, s, CPAR, NCELLS, CCNT, CMIN, CSIZE, CSEED);
    hipLaunchKernelGGL(k_point_labels, dim3(ew(n)), dim3(256), 0, s, PCID, n, CPAR, CSIZE, CSEED, LABEL, SIZE);
    int64_t K = 0;
    int rc = compact(ctx, n, KeptRoot{LABEL, SIZE, (uint64_t)(int64_t)min_size, (uint64_t)(int64_t)max_size},
                     WriteRoot{SIZE, ROOTS, RSIZES}, &K);
    if (rc) return rc;
    if (K == 0) return PITT_OK;
    // PCL order: clusters discovered by ascending seed, then std::sort(rbegin, rend, size <).
    std::vector<int32_t> roots((size_t)K), sizes((size_t)K);
    {
        int32_t* h = (int32_t*)ctx->pinned("cl_roots_h", (size_t)K * 8);
        PITT_HIP_TRY(hipMemcpyAsync(h, ROOTS, (size_t)K * 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipMemcpyAsync(h + K, RSIZES, (size_t)K * 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        std::memcpy(roots.data(), h, (size_t)K * 4);
        std::memcpy(sizes.data(), h + K, (size_t)K * 4);
    }
    if (timing) tm_roots = wall_ms();
    struct RS {
        int32_t root, size;
    };
    std::vector<RS> order((size_t)K);
    for (int64_t i = 0; i < K; ++i) order[(size_t)i] = {roots[(size_t)i], sizes[(size_t)i]};
    std::sort(order.rbegin(), order.rend(), [](const RS& a, const RS& b) { return a.size < b.size; });
    std::vector<int32_t> slot_of((size_t)K);
    std::vector<int64_t> coff((size_t)K + 1, 0);
    for (int64_t t = 0; t < K; ++t) {
        roots[(size_t)t] = order[(size_t)t].root;
        slot_of[(size_t)t] = (int32_t)t;
        coff[(size_t)t + 1] = coff[(size_t)t] + order[(size_t)t].size;
    }
    const int64_t M = coff[(size_t)K];
    int64_t Mp = kSortTile;
    while (Mp < M) Mp <<= 1;
    uint64_t* SK = (uint64_t*)ctx->buf("cl_sortkeys", (size_t)Mp * 8);
    int32_t* SROOT = (int32_t*)ctx->buf("cl_sroot", (size_t)K * 8);
    int64_t* COFF = (int64_t*)ctx->buf("cl_coff", ((size_t)K + 1) * 8);
    int32_t* MIDX = (int32_t*)ctx->buf("cl_midx", (size_t)M * 4);
    float* MXYZ = (float*)ctx->buf("cl_mxyz", (size_t)M * 12);
    float* SUMS = (float*)ctx->buf("cl_sums", (size_t)K * 12);
    if (!SK || !SROOT || !COFF || !MIDX || !MXYZ || !SUMS) return ctx->fail(PITT_E_NOMEM, "cluster scratch");
    PITT_HIP_TRY(hipMemcpyAsync(SROOT, roots.data(), (size_t)K * 4, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemcpyAsync(SROOT + K, slot_of.data(), (size_t)K * 4, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemcpyAsync(COFF, coff.data(), ((size_t)K + 1) * 8, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemsetAsync(RSLOT, 0xFF, N * 4, s));
    PITT_HIP_TRY(hipMemsetAsync(SK, 0xFF, (size_t)Mp * 8, s));
    hipLaunchKernelGGL(k_set_slots, dim3(ew(K)), dim3(256), 0, s, SROOT, SROOT + K, (int32_t)K, RSLOT);
    int64_t M2 = 0;
    rc = compact(ctx, n, KeptPoint{LABEL, RSLOT}, WriteKey{LABEL, RSLOT, SK}, &M2);
    if (rc) return rc;
    if (M2 != M) return ctx->fail(PITT_E_INVALID, "cluster member count mismatch");
    // bitonic sort of Mp keys
    hipLaunchKernelGGL(k_bitonic_local, dim3((unsigned)(Mp / kSortTile)), dim3(1024), 0, s, SK, Mp, kSortTile, (int64_t)0);
    for (int64_t k = 2 * kSortTile; k <= Mp; k <<= 1) {
        for (int64_t j = k / 2; j >= kSortTile; j >>= 1)
            hipLaunchKernelGGL(k_bitonic_global, dim3(ew(Mp)), dim3(256), 0, s, SK, Mp, k, j);
        hipLaunchKernelGGL(k_bitonic_local, dim3((unsigned)(Mp / kSortTile)), dim3(1024), 0, s, SK, Mp, kSortTile, k);
    }
    hipLaunchKernelGGL(k_members, dim3(ew(M)), dim3(256), 0, s, SK, M, X, Y, Z, MIDX, MXYZ, MXYZ + M, MXYZ + 2 * M);
    if (M >= kXsMinMembers && K > 0) {  // the exact walk over the chip
        std::vector<XsSeg> hseg((size_t)K);
        int64_t nb = 0;
        for (int64_t t = 0; t < K; ++t) {
            hseg[(size_t)t] = XsSeg{nb, coff[(size_t)t + 1] - coff[(size_t)t]};
            nb += (hseg[(size_t)t].len + kXsBlk - 1) / kXsBlk;
        }
        const int64_t T = std::max<int64_t>(nb, 1) * kXsBlk;
        float* XV = (float*)ctx->buf("cl_xs_v", (size_t)3 * T * 4);
        XsSeg* XSEG = (XsSeg*)ctx->buf("cl_xs_seg", (size_t)K * sizeof(XsSeg));
        int32_t* XB = (int32_t*)ctx->buf("cl_xs_bseg", (size_t)std::max<int64_t>(nb, 1) * 4);
        char* hp = (char*)ctx->pinned("cl_xs_h", (size_t)K * sizeof(XsSeg) + (size_t)nb * 4);
        XsScratch scr;
        if (!XV || !XSEG || !XB || !hp) return ctx->fail(PITT_E_NOMEM, "cluster sums scratch");
        if (int e = xs_scratch(ctx, T / kXsBlk, 3, "cl", &scr)) return e;
        std::memcpy(hp, hseg.data(), (size_t)K * sizeof(XsSeg));
        int32_t* hb = (int32_t*)(hp + (size_t)K * sizeof(XsSeg));
        for (int64_t t = 0; t < K; ++t)
            for (int64_t j = 0; j < (hseg[(size_t)t].len + kXsBlk - 1) / kXsBlk; ++j) hb[hseg[(size_t)t].blk0 + j] = (int32_t)t;
        PITT_HIP_TRY(hipMemcpyAsync(XSEG, hp, (size_t)K * sizeof(XsSeg), hipMemcpyHostToDevice, s));
        if (nb) PITT_HIP_TRY(hipMemcpyAsync(XB, hb, (size_t)nb * 4, hipMemcpyHostToDevice, s));
        if (nb) hipLaunchKernelGGL(k_pad_members, dim3((unsigned)nb), dim3(kXsBlk), 0, s, MXYZ, M, COFF, XSEG, XB, XV, T);
        xs_enqueue(s, XV, T, 3, (int)K, XSEG, XB, SUMS, scr);
    } else {
        hipLaunchKernelGGL(k_sums, dim3((unsigned)K), dim3(256), 0, s, COFF, (int32_t)K, MXYZ, MXYZ + M, MXYZ + 2 * M, SUMS);
    }
    PITT_HIP_TRY(hipGetLastError());
    float* sums = (float*)ctx->pinned("cl_sums_h", (size_t)K * 12);
    PITT_HIP_TRY(hipMemcpyAsync(sums, SUMS, (size_t)K * 12, hipMemcpyDeviceToHost, s));
    if (dout) {  // members stay on the device
        PITT_HIP_TRY(hipStreamSynchronize(s));
        for (int64_t t = 0; t < K; ++t) {
            pitt_cluster_dev c;
            c.size = coff[(size_t)t + 1] - coff[(size_t)t];
            c.offset = coff[(size_t)t];
            c.sum_xyz[0] = sums[(size_t)t * 3];
            c.sum_xyz[1] = sums[(size_t)t * 3 + 1];
            c.sum_xyz[2] = sums[(size_t)t * 3 + 2];
            c.pad = 0.0f;
            ctx->keep_clusters_dev.push_back(c);
        }
        dout->n_clusters = (int32_t)K;
        dout->clusters = ctx->keep_clusters_dev.data();
        dout->indices = MIDX;
        return PITT_OK;
    }
    // members into the context's pinned output block (reused across calls; valid until the next call)
    int32_t* base = (int32_t*)ctx->pinned("cl_out_h", (size_t)std::max<int64_t>(M, 1) * 4);
    if (!base) return ctx->fail(PITT_E_NOMEM, "cluster members (pinned)");
    PITT_HIP_TRY(hipMemcpyAsync(base, MIDX, (size_t)M * 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    if (timing)
        std::fprintf(stderr, "pitt_euclidean_clusters n=%lld: input %.3f ms, components + roots %.3f ms, members + sums + "
                     "D2H %.3f ms (%lld clusters, %lld members)\n", (long long)n, tm_in - tm0, tm_roots - tm_in,
                     wall_ms() - tm_roots, (long long)K, (long long)M);
    for (int64_t t = 0; t < K; ++t) {
        pitt_cluster c;
        c.size = coff[(size_t)t + 1] - coff[(size_t)t];
        c.indices = base + coff[(size_t)t];
        c.sum_xyz[0] = sums[(size_t)t * 3];
        c.sum_xyz[1] = sums[(size_t)t * 3 + 1];
        c.sum_xyz[2] = sums[(size_t)t * 3 + 2];
        ctx->keep_clusters.push_back(c);
    }
    out->n_clusters = (int32_t)K;
    out->clusters = ctx->keep_clusters.data();
    return PITT_OK;
}

}  // namespace pitt

extern "C" int pitt_euclidean_clusters(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                       double tolerance, int32_t min_size, int32_t max_size, pitt_cluster_list* out) {
    if (!ctx) return PITT_E_INVALID;
    if (!out || n < 0 || (n > 0 && (!x || !y || !z))) return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::euclidean_clusters_impl(ctx, x, y, z, n, tolerance, min_size, max_size, out, nullptr, false, 0);
}

extern "C" int pitt_euclidean_clusters_aos(pitt_ctx* ctx, const float* xyz, int64_t n, int32_t stride_bytes,
                                           double tolerance, int32_t min_size, int32_t max_size, pitt_cluster_list* out) {
    if (!ctx) return PITT_E_INVALID;
    if (!out || n < 0 || (n > 0 && !xyz)) return ctx->fail(PITT_E_INVALID, "null argument");
    if (stride_bytes != 12 && stride_bytes != 16) return ctx->fail(PITT_E_INVALID, "stride must be 12 or 16");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::euclidean_clusters_impl(ctx, xyz, nullptr, nullptr, n, tolerance, min_size, max_size, out, nullptr,
                                         false, stride_bytes);
}

extern "C" int pitt_euclidean_clusters_dev(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                           double tolerance, int32_t min_size, int32_t max_size,
                                           pitt_cluster_list_dev* out) {
    if (!ctx) return PITT_E_INVALID;
    if (!out || n < 0 || (n > 0 && (!x || !y || !z))) return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::euclidean_clusters_impl(ctx, x, y, z, n, tolerance, min_size, max_size, nullptr, out, true, 0);
}

namespace pitt {
int find_supports_impl(pitt_ctx* ctx, const float* hx, const float* hy, const float* hz, int64_t N,
                       const pitt_support_params* sp, pitt_support_list* out, pitt_support_list_dev* dout,
                       bool dev_in, int aos_stride);

__global__ void k_offset_indices(const int32_t* __restrict__ src, int64_t m, int32_t* __restrict__ dst) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        dst[k] = src[k];
}
}  // namespace pitt

extern "C" void pitt_cluster_params_default(pitt_cluster_params* p) {
    if (!p) return;
    p->tolerance = 0.03;     // cluster_segmentation_srv.cpp:32
    p->min_rate = 0.01;      // :33
    p->max_rate = 0.99;      // :34
    p->min_input_size = 30;  // :35 (Q6)
    p->pad = 0;
}

// obj_segmentation.cpp:261-312: for each support (discovery order) clusterize its on-support cloud
// (cluster_segmentation_srv.cpp:54: skipped below min_input_size; :60-61 the size limits rounded from
// the rates), everything device-resident.  The supports' outputs live in the context arena under
// their own names, so the cluster calls do not disturb them; each support's members are copied into
// one scene buffer.
extern "C" int pitt_segment_objects_dev(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                        const pitt_support_params* sp, const pitt_cluster_params* cp,
                                        pitt_scene* out) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (!sp || !cp || !out || n < 0 || (n > 0 && (!x || !y || !z))) return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    out->n_objects = 0;
    out->objects = nullptr;
    out->indices = nullptr;
    int rc = find_supports_impl(ctx, x, y, z, n, sp, nullptr, &out->supports, true, 0);
    if (rc) return rc;
    const std::vector<pitt_support_dev> sups = ctx->keep_supports_dev;  // cluster calls clear the keep lists
    std::vector<pitt_object> objs;
    int64_t total = 0;
    for (const pitt_support_dev& su : sups) total += su.n_on_support;
    int32_t* IDX = (int32_t*)ctx->buf("scene_idx", (size_t)std::max<int64_t>(total, 1) * 4);
    if (!IDX) return ctx->fail(PITT_E_NOMEM, "scene indices");
    int64_t used = 0;
    for (size_t k = 0; k < sups.size(); ++k) {
        const pitt_support_dev& su = sups[k];
        const int64_t m = su.n_on_support;
        if (m < (int64_t)cp->min_input_size) continue;  // cluster_segmentation_srv.cpp:54
        const int32_t mn = (int32_t)std::round((double)m * cp->min_rate);
        const int32_t mx = (int32_t)std::round((double)m * cp->max_rate);
        pitt_cluster_list_dev L;
        rc = euclidean_clusters_impl(ctx, su.on_support_xyz, su.on_support_xyz + su.stride,
                                     su.on_support_xyz + 2 * su.stride, m, cp->tolerance, mn, mx, nullptr, &L, true, 0);
        if (rc) return rc;
        int64_t members = 0;
        for (int c = 0; c < L.n_clusters; ++c) {
            pitt_object o;
            o.support = (int32_t)k;
            o.pad = 0;
            o.size = L.clusters[c].size;
            o.offset = used + L.clusters[c].offset;
            for (int j = 0; j < 3; ++j) o.sum_xyz[j] = L.clusters[c].sum_xyz[j];
            o.pad2 = 0.0f;
            objs.push_back(o);
            members += o.size;
        }
        if (members > 0)
            PITT_HIP_TRY(hipMemcpyAsync(IDX + used, L.indices, (size_t)members * 4, hipMemcpyDeviceToDevice, ctx->stream));
        used += members;
    }
    PITT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->keep_supports_dev = sups;
    ctx->keep_objects = objs;
    out->supports.supports = ctx->keep_supports_dev.data();
    out->n_objects = (int32_t)ctx->keep_objects.size();
    out->objects = ctx->keep_objects.data();
    out->indices = IDX;
    return PITT_OK;
}
