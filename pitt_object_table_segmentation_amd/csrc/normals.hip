// normals.hip -- pcl::NormalEstimation<PointXYZ, Normal> with a search::KdTree and setKSearch(k), as
// PCManager::estimateNormal (src/point_cloud_library/pc_manager.cpp:68-78, k = 50 from :18), called on
// the world cloud at src/obj_segmentation.cpp:253 and src/ransac_segmentation.cpp:233 (SURVEY.md s8f
// row 3).  Restated in oracle/pitt_oracle.cpp (orc_normal_estimation).
//
// Per query point (PCL 1.7 features/impl/normal_3d.hpp, feature.h):
//   * the k nearest finite points (KdTreeFLANN: exact, k clamped to the indexed point count), ordered
//     by FLANN's float distance (dx*dx + dy*dy) + dz*dz, equal distances by point index (A11);
//   * computeMeanAndCovarianceMatrix over them in that order (nine float accumulators, x (1/n), A6/A9);
//   * eigen33 -> normal; curvature = |l_min / trace|; flipNormalTowardsViewpoint; < 3 neighbours or a
//     non-finite query -> NaN.
//
// Device pipeline:
//   k_vox_minmax (voxel.hip)  finite bounding box and count
//   grid                      linear cell index per finite point (ordered compaction), stable radix
//                             sort, per-cell [begin, end) in a dense table
//   k_knn                     one wave per query: the cells of ring r around the query's cell are
//                             streamed into an LDS candidate buffer (distance bits, point index); the
//                             k best are selected by bisection on the distance bits (then on the index
//                             for ties) and compacted; r grows until the k-th distance is certainly
//                             below r*h (no point outside the ring can be closer); a 64-lane bitonic
//                             sort gives PCL's order
//   k_normals                 one thread per point: the nine accumulators over the ordered neighbours,
//                             eigen33, curvature, viewpoint flip
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "compact.hpp"
#include "ctx.hpp"
#include "device_common.hpp"

#pragma clang fp contract(off)

namespace pitt {

// voxel.hip
__global__ void k_vox_minmax(const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
                             int64_t n, float* __restrict__ part, int64_t* __restrict__ part_n);

constexpr int kNnMaxK = 64;     // neighbours per query (one per lane in the final sort)
constexpr int kNnCap = 1024;    // candidate buffer per wave (LDS)
constexpr int kNnWaves = 4;     // queries per block

struct NGrid {
    float mn[3];
    float inv_h;     // cells: (int)((p - mn) * inv_h), clamped to [0, dim - 1]
    float h;
    float margin;    // absolute slack on r * h for the ring test (cell-assignment rounding)
    int32_t dim[3];
};

__device__ __forceinline__ bool fin3(float x, float y, float z) {
    return __builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z);
}

__device__ __forceinline__ int cell_of(const NGrid& g, float v, int a) {
    const int c = (int)((v - g.mn[a]) * g.inv_h);
    return min(max(c, 0), g.dim[a] - 1);
}

struct FinitePt {
    const float *x, *y, *z;
    __device__ bool operator()(int64_t i) const { return fin3(x[i], y[i], z[i]); }
};

struct WriteCellKey {
    const float *x, *y, *z;
    NGrid g;
    uint32_t* key;
    uint32_t* val;
    __device__ void operator()(int64_t i, int64_t pos) const {
        const int cx = cell_of(g, x[i], 0), cy = cell_of(g, y[i], 1), cz = cell_of(g, z[i], 2);
        key[pos] = (uint32_t)cx + (uint32_t)g.dim[0] * ((uint32_t)cy + (uint32_t)g.dim[1] * (uint32_t)cz);
        val[pos] = (uint32_t)i;
    }
};

__global__ void k_fill_i32(int32_t* __restrict__ p, int64_t n, int32_t v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// begin[c] / end[c] of every occupied cell from the sorted keys
__global__ void k_cell_ranges(const uint32_t* __restrict__ key, int64_t m, int32_t* __restrict__ cbeg,
                              int32_t* __restrict__ cend) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t k = key[i];
        if (i == 0 || key[i - 1] != k) cbeg[k] = (int32_t)i;
        if (i == m - 1 || key[i + 1] != k) cend[k] = (int32_t)(i + 1);
    }
}

// occupied cells of a pilot grid (run heads of sorted keys), for choosing the final cell size
__global__ void k_count_runs(const uint32_t* __restrict__ key, int64_t m, unsigned long long* __restrict__ runs) {
    unsigned long long c = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        c += (i == 0 || key[i - 1] != key[i]) ? 1ull : 0ull;
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(runs, c);
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Keep the kk best (distance bits, index) of the fill candidates in slots [0, kk) (any order).
// The candidates of lane l are slots l + 64 i.  Bisection on the distance bits finds D, the kk-th
// smallest distance; ties at D are cut by the smallest indices (bisection on the index).
__device__ int nn_select(uint32_t* __restrict__ bd, int32_t* __restrict__ bi, int fill, int kk, int lane) {
    if (fill <= kk) return fill;
    constexpr int R = kNnCap / 64;
    uint32_t d[R];
    int32_t ix[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int s = lane + 64 * i;
        d[i] = s < fill ? bd[s] : 0xFFFFFFFFu;
        ix[i] = s < fill ? bi[s] : 0x7FFFFFFF;
    }
    uint32_t lo = 0, hi = 0x7F800000u;  // finite non-negative floats: bits order = value order
    while (lo < hi) {                     // smallest D with #(d <= D) >= kk
        const uint32_t mid = lo + ((hi - lo) >> 1);
        int c = 0;
#pragma unroll
        for (int i = 0; i < R; ++i) c += d[i] <= mid ? 1 : 0;
        if (wave_sum_i(c) >= kk) hi = mid;
        else lo = mid + 1;
    }
    const uint32_t D = lo;
    int lt = 0, eq = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        lt += d[i] < D ? 1 : 0;
        eq += d[i] == D ? 1 : 0;
    }
    lt = wave_sum_i(lt);
    eq = wave_sum_i(eq);
    int32_t I = 0x7FFFFFFF;  // indices at D kept: idx <= I
    const int need = kk - lt;
    if (eq > need) {
        int32_t a = 0, b = 0x7FFFFFFF;
        while (a < b) {
            const int32_t mid = a + ((b - a) >> 1);
            int c = 0;
#pragma unroll
            for (int i = 0; i < R; ++i) c += (d[i] == D && ix[i] <= mid) ? 1 : 0;
            if (wave_sum_i(c) >= need) b = mid;
            else a = mid + 1;
        }
        I = a;
    }
    // ordered compaction of the kept slots into [0, kk)
    int base = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const bool keep = d[i] < D || (d[i] == D && ix[i] <= I);
        const uint64_t b = __builtin_amdgcn_ballot_w64(keep);
        const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        if (keep) {
            bd[base + pre] = d[i];
            bi[base + pre] = ix[i];
        }
        base += __builtin_popcountll(b);
    }
    return kk;
}

template <int KMAX>
__global__ __launch_bounds__(64 * kNnWaves) void k_knn(const float* __restrict__ X, const float* __restrict__ Y,
                                                       const float* __restrict__ Z, const uint32_t* __restrict__ fin_idx,
                                                       int64_t nf, NGrid g, const int32_t* __restrict__ cbeg,
                                                       const int32_t* __restrict__ cend,
                                                       const uint32_t* __restrict__ sorted_idx, int k, int kk,
                                                       int32_t* __restrict__ nn, int32_t* __restrict__ nn_cnt) {
    __shared__ uint32_t s_d[kNnWaves][kNnCap];
    __shared__ int32_t s_i[kNnWaves][kNnCap];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    uint32_t* bd = s_d[w];
    int32_t* bi = s_i[w];
    const int rmax = max(g.dim[0], max(g.dim[1], g.dim[2]));
    for (int64_t qi = (int64_t)blockIdx.x * kNnWaves + w; qi < nf; qi += (int64_t)gridDim.x * kNnWaves) {
        const int q = (int)fin_idx[qi];
        const float qx = X[q], qy = Y[q], qz = Z[q];
        const int cx = cell_of(g, qx, 0), cy = cell_of(g, qy, 1), cz = cell_of(g, qz, 2);
        int fill = 0;
        // rings 1, 2, 4, ...: an isolated point (few neighbours near it) reaches its k-th neighbour
        // in O(log) ring scans instead of one per cell of distance
        for (int r = 1;; r = min(2 * r, rmax)) {
            fill = 0;
            const int ax0 = max(cx - r, 0), ax1 = min(cx + r, g.dim[0] - 1);
            const int ay0 = max(cy - r, 0), ay1 = min(cy + r, g.dim[1] - 1);
            const int az0 = max(cz - r, 0), az1 = min(cz + r, g.dim[2] - 1);
            for (int c = az0; c <= az1; ++c)
                for (int b = ay0; b <= ay1; ++b) {
                    const int64_t row = (int64_t)g.dim[0] * ((int64_t)b + (int64_t)g.dim[1] * c);
                    for (int a = ax0; a <= ax1; ++a) {
                        const int32_t beg = __builtin_amdgcn_readfirstlane(cbeg[row + a]);
                        if (beg < 0) continue;
                        const int32_t cnt = __builtin_amdgcn_readfirstlane(cend[row + a]) - beg;
                        for (int t0 = 0; t0 < cnt; t0 += 64) {
                            if (fill + 64 > kNnCap) fill = nn_select(bd, bi, fill, kk, lane);
                            const int t = t0 + lane;
                            if (t < cnt) {
                                const int j = (int)sorted_idx[beg + t];
                                const float dx = qx - X[j], dy = qy - Y[j], dz = qz - Z[j];
                                const float d2 = (dx * dx + dy * dy) + dz * dz;  // FLANN L2_Simple
                                bd[fill + lane] = __float_as_uint(d2);
                                bi[fill + lane] = j;
                            }
                            fill += min(64, cnt - t0);
                        }
                    }
                }
            const bool all = r >= rmax;
            if (fill < kk && !all) continue;
            fill = nn_select(bd, bi, fill, kk, lane);
            // the k-th distance (max of the kept) against the nearest possible outside point
            float dk = 0.0f;
            for (int s = lane; s < fill; s += 64) dk = fmaxf(dk, __uint_as_float(bd[s]));
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) dk = fmaxf(dk, __shfl_xor(dk, d, 64));
            const float lim = (float)r * g.h - g.margin;
            if (all || (lim > 0.0f && dk <= lim * lim * (1.0f - 1e-5f))) break;
        }
        // PCL order: ascending (distance, index); kk <= 64 keys, one per lane
        uint64_t key = lane < fill ? ((uint64_t)bd[lane] << 32) | (uint32_t)bi[lane] : ~0ull;
#pragma unroll
        for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                const uint32_t plo = __shfl_xor((uint32_t)key, stride, 64);
                const uint32_t phi = __shfl_xor((uint32_t)(key >> 32), stride, 64);
                const uint64_t p = ((uint64_t)phi << 32) | plo;
                const bool up = (lane & size) == 0 || size == 64;
                const bool lower = (lane & stride) == 0;
                key = (lower == up) ? (key < p ? key : p) : (key > p ? key : p);
            }
        }
        if (lane < fill) nn[(int64_t)q * k + lane] = (int32_t)(uint32_t)key;
        if (lane == 0) nn_cnt[q] = fill;
    }
}

__global__ __launch_bounds__(kBlock) void k_normals(const float* __restrict__ X, const float* __restrict__ Y,
                                                    const float* __restrict__ Z, int64_t n,
                                                    const int32_t* __restrict__ nn, const int32_t* __restrict__ nn_cnt,
                                                    int k, float vpx, float vpy, float vpz, float* __restrict__ nx,
                                                    float* __restrict__ ny, float* __restrict__ nz,
                                                    float* __restrict__ curv) {
    for (int64_t q = blockIdx.x * (int64_t)kBlock + threadIdx.x; q < n; q += (int64_t)gridDim.x * kBlock) {
        const float px = X[q], py = Y[q], pz = Z[q];
        const int cnt = fin3(px, py, pz) ? nn_cnt[q] : 0;
        if (cnt < 3) {
            nx[q] = ny[q] = nz[q] = curv[q] = __builtin_nanf("");
            continue;
        }
        float a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        const int32_t* l = nn + q * k;
        for (int t = 0; t < cnt; ++t) {
            const int j = l[t];
            const float x = X[j], y = Y[j], z = Z[j];
            a[0] += x * x;
            a[1] += x * y;
            a[2] += x * z;
            a[3] += y * y;
            a[4] += y * z;
            a[5] += z * z;
            a[6] += x;
            a[7] += y;
            a[8] += z;
        }
        const float r = 1.0f / (float)cnt;  // Eigen 3.2 `accu /= n` (A9)
#pragma unroll
        for (int t = 0; t < 9; ++t) a[t] = a[t] * r;
        float cov[9];
        cov[0] = a[0] - a[6] * a[6];
        cov[1] = a[1] - a[6] * a[7];
        cov[2] = a[2] - a[6] * a[8];
        cov[4] = a[3] - a[7] * a[7];
        cov[5] = a[4] - a[7] * a[8];
        cov[8] = a[5] - a[8] * a[8];
        cov[3] = cov[1];
        cov[6] = cov[2];
        cov[7] = cov[5];
        float ev, e[3];
        eigen33v(cov, &ev, e);
        const float tr = cov[0] + cov[4] + cov[8];
        curv[q] = tr != 0.0f ? fabsf(ev / tr) : 0.0f;
        const float vx = vpx - px, vy = vpy - py, vz = vpz - pz;
        if (vx * e[0] + vy * e[1] + vz * e[2] < 0) {
            e[0] *= -1.0f;
            e[1] *= -1.0f;
            e[2] *= -1.0f;
        }
        nx[q] = e[0];
        ny[q] = e[1];
        nz[q] = e[2];
    }
}

static int sort_cells(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, int64_t nf,
                      const NGrid& g, uint32_t** skey, uint32_t** sval) {
    hipStream_t s = ctx->stream;
    const int64_t nt = ctiles(n);
    int32_t* tc = (int32_t*)ctx->buf("nrm_tc", (size_t)(nt + 1) * 4);
    int32_t* to = (int32_t*)ctx->buf("nrm_to", (size_t)(nt + 1) * 4);
    uint32_t* k1 = (uint32_t*)ctx->buf("nrm_k1", (size_t)nf * 4);
    uint32_t* v1 = (uint32_t*)ctx->buf("nrm_v1", (size_t)nf * 4);
    uint32_t* k2 = (uint32_t*)ctx->buf("nrm_k2", (size_t)nf * 4);
    uint32_t* v2 = (uint32_t*)ctx->buf("nrm_v2", (size_t)nf * 4);
    if (!tc || !to || !k1 || !v1 || !k2 || !v2) return ctx->fail(PITT_E_NOMEM, "normals grid");
    FinitePt fp{x, y, z};
    const int gt = grid_for_tiles(nt);
    hipLaunchKernelGGL(k_pred_count<FinitePt>, dim3(gt), dim3(kBlock), 0, s, fp, n, tc);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, tc, nt, to);
    hipLaunchKernelGGL((k_pred_apply<FinitePt, WriteCellKey>), dim3(gt), dim3(kBlock), 0, s, fp,
                       WriteCellKey{x, y, z, g, k1, v1}, n, to);
    const int64_t cells = (int64_t)g.dim[0] * g.dim[1] * g.dim[2];
    int end_bit = 1;
    while (end_bit < 32 && ((int64_t)1 << end_bit) < cells) ++end_bit;
    hipcub::DoubleBuffer<uint32_t> kb(k1, k2), vb(v1, v2);
    size_t tmp_bytes = 0;
    PITT_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kb, vb, (int)nf, 0, end_bit, s));
    void* tmp = ctx->buf("nrm_sort_tmp", std::max<size_t>(tmp_bytes, 16));
    if (!tmp) return ctx->fail(PITT_E_NOMEM, "normals sort scratch");
    PITT_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kb, vb, (int)nf, 0, end_bit, s));
    *skey = kb.Current();
    *sval = vb.Current();
    return PITT_OK;
}

static NGrid make_grid(const float mn[3], const float mx[3], double h) {
    NGrid g;
    double ext = 0;
    for (int a = 0; a < 3; ++a) ext = std::max(ext, (double)mx[a] - (double)mn[a]);
    // at most 2^25 cells in the dense table
    for (;;) {
        int64_t cells = 1;
        for (int a = 0; a < 3; ++a) cells *= (int64_t)(((double)mx[a] - (double)mn[a]) / h) + 1;
        if (cells <= ((int64_t)1 << 25)) break;
        h *= 1.25;
    }
    g.h = (float)h;
    g.inv_h = (float)(1.0 / h);
    for (int a = 0; a < 3; ++a) {
        g.mn[a] = mn[a];
        g.dim[a] = (int32_t)(((double)mx[a] - (double)mn[a]) / h) + 1;
    }
    // a cell index is computed in float: a boundary may move by a few ulp of the coordinates
    g.margin = (float)(1e-5 * (ext + h) + 1e-12);
    return g;
}

static int normals_impl(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, int k,
                        const float vp[3], float* nx, float* ny, float* nz, float* curv, int32_t* nn_out,
                        int32_t* cnt_out) {
    hipStream_t s = ctx->stream;
    if (n == 0) return PITT_OK;
    constexpr int kMB = 1024;
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, kMB));
    float* part = (float*)ctx->buf("nrm_part", (size_t)kMB * 8 * 4);
    int64_t* part_n = (int64_t*)ctx->buf("nrm_part_n", (size_t)kMB * 8);
    if (!part || !part_n) return ctx->fail(PITT_E_NOMEM, "normals scratch");
    int rec = ctx->prof_begin("k_nrm_grid", (double)n * 12.0);
    hipLaunchKernelGGL(k_vox_minmax, dim3(blocks), dim3(kBlock), 0, s, x, y, z, n, part, part_n);
    float* hpart = (float*)ctx->pinned("nrm_hpart", (size_t)kMB * 8 * 4 + (size_t)kMB * 8);
    if (!hpart) return ctx->fail(PITT_E_NOMEM, "normals pinned");
    int64_t* hn = (int64_t*)(hpart + (size_t)kMB * 8);
    PITT_HIP_TRY(hipMemcpyAsync(hpart, part, (size_t)blocks * 8 * 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipMemcpyAsync(hn, part_n, (size_t)blocks * 8, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    int64_t nf = 0;
    for (int b = 0; b < blocks; ++b) {
        for (int a = 0; a < 3; ++a) {
            mn[a] = std::min(mn[a], hpart[b * 8 + a]);
            mx[a] = std::max(mx[a], hpart[b * 8 + 3 + a]);
        }
        nf += hn[b];
    }
    int32_t* cntd = cnt_out;
    if (!cntd) cntd = (int32_t*)ctx->buf("nrm_cnt", (size_t)n * 4);
    int32_t* nnd = nn_out;
    if (!nnd) nnd = (int32_t*)ctx->buf("nrm_nn", (size_t)n * k * 4);
    if (!cntd || !nnd) return ctx->fail(PITT_E_NOMEM, "normals neighbour lists");
    PITT_HIP_TRY(hipMemsetAsync(cntd, 0, (size_t)n * 4, s));
    const int kk = (int)std::min<int64_t>(k, nf);
    if (nf > 0 && kk >= 3) {
        double ext = 0;
        for (int a = 0; a < 3; ++a) ext = std::max(ext, (double)mx[a] - (double)mn[a]);
        // cell size: a pilot grid at extent / 64, then ~16 points per occupied cell (surface clouds)
        double h = std::max(ext / 64.0, 1e-6);
        NGrid g = make_grid(mn, mx, h);
        uint32_t *skey = nullptr, *sval = nullptr;
        int rc = sort_cells(ctx, x, y, z, n, nf, g, &skey, &sval);
        if (rc != PITT_OK) return rc;
        unsigned long long* runs = (unsigned long long*)ctx->buf("nrm_runs", 8);
        if (!runs) return ctx->fail(PITT_E_NOMEM, "normals runs");
        PITT_HIP_TRY(hipMemsetAsync(runs, 0, 8, s));
        hipLaunchKernelGGL(k_count_runs, dim3(grid_for_tiles(ctiles(nf))), dim3(kBlock), 0, s, skey, nf, runs);
        unsigned long long* hr = (unsigned long long*)ctx->pinned("nrm_hruns", 8);
        PITT_HIP_TRY(hipMemcpyAsync(hr, runs, 8, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        const double per = (double)nf / (double)std::max<unsigned long long>(*hr, 1ull);
        const double h2 = std::max(h * std::sqrt(16.0 / per), 1e-6);
        if (h2 < 0.8 * h || h2 > 1.25 * h) {
            g = make_grid(mn, mx, h2);
            rc = sort_cells(ctx, x, y, z, n, nf, g, &skey, &sval);
            if (rc != PITT_OK) return rc;
        }
        const int64_t cells = (int64_t)g.dim[0] * g.dim[1] * g.dim[2];
        int32_t* cbeg = (int32_t*)ctx->buf("nrm_cbeg", (size_t)cells * 4);
        int32_t* cend = (int32_t*)ctx->buf("nrm_cend", (size_t)cells * 4);
        if (!cbeg || !cend) return ctx->fail(PITT_E_NOMEM, "normals cell table");
        hipLaunchKernelGGL(k_fill_i32, dim3(std::min<int64_t>((cells + 255) / 256, 8192)), dim3(256), 0, s, cbeg, cells, -1);
        hipLaunchKernelGGL(k_cell_ranges, dim3(grid_for_tiles(ctiles(nf))), dim3(kBlock), 0, s, skey, nf, cbeg, cend);
        ctx->prof_end(rec);
        PITT_HIP_TRY(hipGetLastError());
        // the finite points in input order are the queries: sval holds them sorted by cell, which
        // keeps a block's queries spatially close
        rec = ctx->prof_begin("k_knn", (double)nf * (12.0 + 4.0 * k));
        const int kb = (int)std::min<int64_t>((nf + kNnWaves - 1) / kNnWaves, 65536);
        hipLaunchKernelGGL(k_knn<kNnMaxK>, dim3(kb), dim3(64 * kNnWaves), 0, s, x, y, z, sval, nf, g, cbeg, cend,
                           sval, k, kk, nnd, cntd);
        ctx->prof_end(rec);
        PITT_HIP_TRY(hipGetLastError());
    } else {
        ctx->prof_end(rec);
        if (nf > 0 && kk > 0 && kk < 3) {  // too few points: counts only (normals are NaN)
            // every finite point's neighbours are all finite points; PCL returns NaN normals (< 3)
        }
    }
    rec = ctx->prof_begin("k_normals", (double)n * 28.0 + (double)nf * k * 16.0);
    hipLaunchKernelGGL(k_normals, dim3(std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, 8192))),
                       dim3(kBlock), 0, s, x, y, z, n, nnd, cntd, k, vp[0], vp[1], vp[2], nx, ny, nz, curv);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    PITT_HIP_TRY(hipStreamSynchronize(s));
    return PITT_OK;
}

}  // namespace pitt

extern "C" int pitt_normal_estimation(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                      int32_t k, const float viewpoint[3], float* nx, float* ny, float* nz,
                                      float* curvature, int32_t* neighbours, int32_t* neighbour_count) {
    if (!ctx) return PITT_E_INVALID;
    if (n < 0 || (n > 0 && (!x || !y || !z || !nx || !ny || !nz || !curvature)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (k < 1 || k > pitt::kNnMaxK) return ctx->fail(PITT_E_INVALID, "k must be in [1, 64]");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    const float zero[3] = {0.0f, 0.0f, 0.0f};
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::normals_impl(ctx, x, y, z, n, k, viewpoint ? viewpoint : zero, nx, ny, nz, curvature, neighbours,
                              neighbour_count);
}
