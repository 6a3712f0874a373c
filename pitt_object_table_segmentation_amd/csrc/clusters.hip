// clusters.hip -- EuclideanClusterExtraction (extractEuclideanClusters + sorted search::KdTree) on
// gfx950.  Replaces src/segmentation_services/cluster_segmentation_srv.cpp:57-69 (reference path).
//
// PCL grows a cluster by BFS over radius neighbours (FLANN L2_Simple: ((dx^2 + dy^2) + dz^2) < r^2
// in float, r^2 = (float)((double)tol_f * tol_f)), seeding clusters in ascending index order.
// Without duplicate points the clusters are exactly the connected components of that
// radius graph, and the seed of each is its smallest index.  Here:
//   k_cells     hashed uniform grid, cell = 1.01 * tolerance (a neighbour is at most one cell away)
//   k_union     union-find over the 27-cell neighbourhood, smaller root wins (root = min index)
//   k_flatten / k_sizes / kept-root compaction (ascending seeds = PCL discovery order)
//   host        std::sort(rbegin, rend, size <) -- the reference's own ordering call, so ties
//               and > 16 clusters order exactly as libstdc++ does it there
//   k_keys + bitonic sort of (slot << 32 | index): members ascending inside each cluster
//   k_sums      float sums in index order (the handler divides by n + 1, Q7)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "compact.hpp"
#include "ctx.hpp"

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

__global__ __launch_bounds__(kBlock) void k_minxyz(const float* __restrict__ x, const float* __restrict__ y,
                                                   const float* __restrict__ z, int64_t n, float* __restrict__ part) {
    __shared__ float s[3][kBlock / 64];
    float a = INFINITY, b = INFINITY, c = INFINITY;
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const float px = x[i], py = y[i], pz = z[i];
        if (finite3(px, py, pz)) {
            a = fminf(a, px);
            b = fminf(b, py);
            c = fminf(c, pz);
        }
    }
    for (int d = 32; d >= 1; d >>= 1) {
        a = fminf(a, __shfl_xor(a, d, 64));
        b = fminf(b, __shfl_xor(b, d, 64));
        c = fminf(c, __shfl_xor(c, d, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s[0][w] = a; s[1][w] = b; s[2][w] = c; }
    __syncthreads();
    if (threadIdx.x < 3) {
        float m = s[threadIdx.x][0];
        for (int i = 1; i < kBlock / 64; ++i) m = fminf(m, s[threadIdx.x][i]);
        part[3 * blockIdx.x + threadIdx.x] = m;
    }
}

__global__ __launch_bounds__(64) void k_minxyz_final(const float* __restrict__ part, int nb, float* __restrict__ mn) {
    float a = INFINITY, b = INFINITY, c = INFINITY;
    for (int i = threadIdx.x; i < nb; i += 64) {
        a = fminf(a, part[3 * i]);
        b = fminf(b, part[3 * i + 1]);
        c = fminf(c, part[3 * i + 2]);
    }
    for (int d = 32; d >= 1; d >>= 1) {
        a = fminf(a, __shfl_xor(a, d, 64));
        b = fminf(b, __shfl_xor(b, d, 64));
        c = fminf(c, __shfl_xor(c, d, 64));
    }
    if (threadIdx.x == 0) { mn[0] = a; mn[1] = b; mn[2] = c; }
}

__global__ void k_iota_cl(int32_t* __restrict__ v, int64_t n) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        v[k] = (int32_t)k;
}

struct Grid {
    const float *x, *y, *z;
    const float* mn;
    double inv_cell;
    uint64_t* keys;   // [hsize]
    int32_t* slot;    // [n]
    int32_t* ccount;  // [hsize]
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

__global__ void k_cells(Grid g, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        // a non-finite point has no radius neighbours (FLANN distances are NaN): a singleton
        if (!finite3(g.x[i], g.y[i], g.z[i])) { g.slot[i] = -1; continue; }
        int64_t cx, cy, cz;
        cell_of(g, i, cx, cy, cz);
        const uint64_t key = cell_key(cx, cy, cz);
        uint32_t h = hash64(key) & g.hmask;
        while (true) {
            const uint64_t prev = atomicCAS((unsigned long long*)&g.keys[h], (unsigned long long)kEmpty,
                                            (unsigned long long)key);
            if (prev == kEmpty || prev == key) break;
            h = (h + 1) & g.hmask;
        }
        g.slot[i] = (int32_t)h;
        atomicAdd(&g.ccount[h], 1);
    }
}

__global__ void k_scatter(const int32_t* __restrict__ slot, int64_t n, const int32_t* __restrict__ cstart,
                          int32_t* __restrict__ cursor, int32_t* __restrict__ cpts) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t s = slot[i];
        if (s < 0) continue;
        cpts[cstart[s] + atomicAdd(&cursor[s], 1)] = (int32_t)i;
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
        // hook the larger root under the smaller one: roots end up as component minima
        if (atomicCAS(&parent[b], b, a) == b) return;
    }
}

__global__ void k_union(Grid g, int64_t n, const int32_t* __restrict__ cstart, const int32_t* __restrict__ cpts,
                        float r2, int32_t* __restrict__ parent) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float qx = g.x[i], qy = g.y[i], qz = g.z[i];
        if (!finite3(qx, qy, qz)) continue;
        int64_t cx, cy, cz;
        cell_of(g, i, cx, cy, cz);
        for (int dx = -1; dx <= 1; ++dx)
            for (int dy = -1; dy <= 1; ++dy)
                for (int dz = -1; dz <= 1; ++dz) {
                    const int32_t h = hash_find(g, cell_key(cx + dx, cy + dy, cz + dz));
                    if (h < 0) continue;
                    for (int32_t k = cstart[h]; k < cstart[h + 1]; ++k) {
                        const int32_t j = cpts[k];
                        if (j <= i) continue;
                        const float ex = qx - g.x[j], ey = qy - g.y[j], ez = qz - g.z[j];
                        const float d = ex * ex + ey * ey + ez * ez;  // FLANN L2_Simple order
                        if (d < r2) uf_union(parent, (int32_t)i, j);
                    }
                }
    }
}

__global__ void k_flatten_sizes(int32_t* __restrict__ parent, int64_t n, int32_t* __restrict__ size) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = uf_find(parent, (int32_t)i);
        atomicAdd(&size[r], 1);
    }
}

__global__ void k_labels(int32_t* __restrict__ parent, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        parent[i] = uf_find(parent, (int32_t)i);
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

// Float sums in index order (cluster_segmentation_srv.cpp:88-90): one block per cluster stages
// coordinates through LDS; lanes 0..2 run the three serial chains.
__global__ __launch_bounds__(256) void k_sums(const int64_t* __restrict__ coff, int32_t k, const float* __restrict__ cx,
                                              const float* __restrict__ cy, const float* __restrict__ cz,
                                              float* __restrict__ sums) {
    __shared__ float buf[3][1024];
    const int c = blockIdx.x;
    if (c >= k) return;
    const int64_t b = coff[c], e = coff[c + 1];
    float s = 0.0f;
    const int lane = threadIdx.x;
    for (int64_t i0 = b; i0 < e; i0 += 1024) {
        for (int t = lane; t < 1024; t += 256) {
            const int64_t i = i0 + t;
            buf[0][t] = i < e ? cx[i] : 0.0f;
            buf[1][t] = i < e ? cy[i] : 0.0f;
            buf[2][t] = i < e ? cz[i] : 0.0f;
        }
        __syncthreads();
        if (lane < 3) {
            const int64_t cnt = min((int64_t)1024, e - i0);
            for (int t = 0; t < cnt; ++t) s += buf[lane][t];
        }
        __syncthreads();
    }
    if (lane < 3) sums[3 * c + lane] = s;
}

static inline int ew(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096)); }

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

int euclidean_clusters_impl(pitt_ctx* ctx, const float* hx, const float* hy, const float* hz, int64_t n,
                            double tolerance, int32_t min_size, int32_t max_size, pitt_cluster_list* out) {
    hipStream_t s = ctx->stream;
    ctx->keep_clusters.clear();
    ctx->keep_i32.clear();
    out->n_clusters = 0;
    out->clusters = nullptr;
    if (n == 0) return PITT_OK;  // extract(): empty input => no clusters
    // KdTreeFLANN::radiusSearch: r^2 = (float)(radius * radius) with radius = (double)(float)tol
    const float tol_f = (float)tolerance;
    const float r2 = (float)((double)tol_f * (double)tol_f);
    const double cell = (double)tol_f * 1.01;
    if (!(cell > 0.0) || !std::isfinite(cell)) return ctx->fail(PITT_E_INVALID, "tolerance must be > 0");
    uint32_t hsize = 1024;
    while ((int64_t)hsize < 2 * n) hsize <<= 1;
    const size_t N = (size_t)n;
    float* X = (float*)ctx->buf("cl_xyz", N * 3 * 4);
    float* MN = (float*)ctx->buf("cl_min", 64);
    uint64_t* KEYS = (uint64_t*)ctx->buf("cl_hkeys", (size_t)hsize * 8);
    int32_t* SLOT = (int32_t*)ctx->buf("cl_slot", N * 4);
    int32_t* CCNT = (int32_t*)ctx->buf("cl_ccnt", ((size_t)hsize + 1) * 4);
    int32_t* CSTART = (int32_t*)ctx->buf("cl_cstart", ((size_t)hsize + 1) * 4);
    int32_t* CUR = (int32_t*)ctx->buf("cl_cursor", (size_t)hsize * 4);
    int32_t* CPTS = (int32_t*)ctx->buf("cl_cpts", N * 4);
    int32_t* PAR = (int32_t*)ctx->buf("cl_parent", N * 4);
    int32_t* SIZE = (int32_t*)ctx->buf("cl_size", N * 4);
    int32_t* ROOTS = (int32_t*)ctx->buf("cl_roots", N * 4);
    int32_t* RSIZES = (int32_t*)ctx->buf("cl_rsizes", N * 4);
    int32_t* RSLOT = (int32_t*)ctx->buf("cl_rootslot", N * 4);
    if (!X || !MN || !KEYS || !SLOT || !CCNT || !CSTART || !CUR || !CPTS || !PAR || !SIZE || !ROOTS || !RSIZES || !RSLOT)
        return ctx->fail(PITT_E_NOMEM, "cluster scratch");
    float *Y = X + N, *Z = X + 2 * N;
    PITT_HIP_TRY(hipMemcpyAsync(X, hx, N * 4, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemcpyAsync(Y, hy, N * 4, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemcpyAsync(Z, hz, N * 4, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemsetAsync(KEYS, 0xFF, (size_t)hsize * 8, s));
    PITT_HIP_TRY(hipMemsetAsync(CCNT, 0, ((size_t)hsize + 1) * 4, s));
    PITT_HIP_TRY(hipMemsetAsync(CUR, 0, (size_t)hsize * 4, s));
    PITT_HIP_TRY(hipMemsetAsync(SIZE, 0, N * 4, s));
    {
        const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, kMinBlocks));
        float* PART = (float*)ctx->buf("cl_minpart", (size_t)kMinBlocks * 3 * sizeof(float));
        if (!PART) return ctx->fail(PITT_E_NOMEM, "cluster scratch");
        hipLaunchKernelGGL(k_minxyz, dim3(nb), dim3(kBlock), 0, s, X, Y, Z, n, PART);
        hipLaunchKernelGGL(k_minxyz_final, dim3(1), dim3(64), 0, s, PART, nb, MN);
    }
    hipLaunchKernelGGL(k_iota_cl, dim3(ew(n)), dim3(256), 0, s, PAR, n);
    Grid g{X, Y, Z, MN, 1.0 / cell, KEYS, SLOT, CCNT, hsize - 1};
    hipLaunchKernelGGL(k_cells, dim3(ew(n)), dim3(256), 0, s, g, n);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, CCNT, (int64_t)hsize, CSTART);
    hipLaunchKernelGGL(k_scatter, dim3(ew(n)), dim3(256), 0, s, SLOT, n, CSTART, CUR, CPTS);
    hipLaunchKernelGGL(k_union, dim3(ew(n)), dim3(256), 0, s, g, n, CSTART, CPTS, r2, PAR);
    hipLaunchKernelGGL(k_flatten_sizes, dim3(ew(n)), dim3(256), 0, s, PAR, n, SIZE);
    hipLaunchKernelGGL(k_labels, dim3(ew(n)), dim3(256), 0, s, PAR, n);
    int64_t K = 0;
    int rc = compact(ctx, n, KeptRoot{PAR, SIZE, (uint64_t)(int64_t)min_size, (uint64_t)(int64_t)max_size},
                     WriteRoot{SIZE, ROOTS, RSIZES}, &K);
    if (rc) return rc;
    if (K == 0) return PITT_OK;
    // PCL order: clusters discovered by ascending seed, then std::sort(rbegin, rend, size <).
    std::vector<int32_t> roots((size_t)K), sizes((size_t)K);
    PITT_HIP_TRY(hipMemcpy(roots.data(), ROOTS, (size_t)K * 4, hipMemcpyDeviceToHost));
    PITT_HIP_TRY(hipMemcpy(sizes.data(), RSIZES, (size_t)K * 4, hipMemcpyDeviceToHost));
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
    rc = compact(ctx, n, KeptPoint{PAR, RSLOT}, WriteKey{PAR, RSLOT, SK}, &M2);
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
    hipLaunchKernelGGL(k_sums, dim3((unsigned)K), dim3(256), 0, s, COFF, (int32_t)K, MXYZ, MXYZ + M, MXYZ + 2 * M, SUMS);
    PITT_HIP_TRY(hipGetLastError());
    ctx->keep_i32.emplace_back((size_t)M);
    std::vector<float> sums((size_t)K * 3);
    PITT_HIP_TRY(hipMemcpyAsync(ctx->keep_i32.back().data(), MIDX, (size_t)M * 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipMemcpyAsync(sums.data(), SUMS, (size_t)K * 12, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    const int32_t* base = ctx->keep_i32.back().data();
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
    return pitt::euclidean_clusters_impl(ctx, x, y, z, n, tolerance, min_size, max_size, out);
}
