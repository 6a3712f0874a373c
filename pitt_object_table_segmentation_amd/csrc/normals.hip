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
//                             sort, the points' coordinates in cell order, and a dense table of each
//                             cell's first sorted position (a row of cells is one contiguous range)
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
#include <hipcub/device/device_scan.hpp>

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

// points per cell (cstart = their exclusive prefix sum: the first sorted position of every cell)
__global__ void k_cell_count(const uint32_t* __restrict__ key, int64_t m, int32_t* __restrict__ cnt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        if (i == 0 || key[i - 1] != key[i]) {
            int64_t e = i + 1;
            while (e < m && key[e] == key[i]) ++e;
            cnt[key[i]] = (int32_t)(e - i);
        }
}

// the finite points' coordinates in cell order (contiguous candidate loads in k_knn)
__global__ void k_gather_sorted(const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
                                const uint32_t* __restrict__ idx, int64_t m, float* __restrict__ sx,
                                float* __restrict__ sy, float* __restrict__ sz) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t j = idx[i];
        sx[i] = X[j];
        sy[i] = Y[j];
        sz[i] = Z[j];
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
// The candidates of lane l are slots l + 64 i (i < ceil(fill / 64)).  Bisection on the distance bits
// (between the candidates' min and max) finds D, the kk-th smallest distance; ties at D are cut by the
// smallest indices (bisection on the index).  Counts are ballots + popcounts: no cross-lane LDS
// round trip per bisection step.
__device__ int nn_select(uint32_t* __restrict__ bd, int32_t* __restrict__ bi, int fill, int kk, int lane) {
    if (fill <= kk) return fill;
    constexpr int R = kNnCap / 64;
    const int ns = (fill + 63) >> 6;  // wave-uniform
    uint32_t d[R];
    int32_t ix[R];
    uint32_t dmin = 0xFFFFFFFFu, dmax = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int s = lane + 64 * i;
        const bool in = i < ns && s < fill;
        d[i] = in ? bd[s] : 0xFFFFFFFFu;
        ix[i] = in ? bi[s] : 0x7FFFFFFF;
        if (in) {
            dmin = min(dmin, d[i]);
            dmax = max(dmax, d[i]);
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        dmin = min(dmin, (uint32_t)__shfl_xor((int)dmin, o, 64));
        dmax = max(dmax, (uint32_t)__shfl_xor((int)dmax, o, 64));
    }
    auto count = [&](auto pred) {
        int c = 0;
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (i < ns) c += __builtin_popcountll(__builtin_amdgcn_ballot_w64(pred(i)));
        return c;
    };
    uint32_t lo = dmin, hi = dmax;  // finite non-negative floats: bits order = value order
    while (lo < hi) {                // smallest D with #(d <= D) >= kk
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (count([&](int i) { return d[i] <= mid; }) >= kk) hi = mid;
        else lo = mid + 1;
    }
    const uint32_t D = lo;
    const int lt = count([&](int i) { return d[i] < D; });
    const int eq = count([&](int i) { return d[i] == D; });
    int32_t I = 0x7FFFFFFF;  // indices at D kept: idx <= I
    const int need = kk - lt;
    if (eq > need) {
        int32_t a = 0, b = 0x7FFFFFFF;
        while (a < b) {
            const int32_t mid = a + ((b - a) >> 1);
            if (count([&](int i) { return d[i] == D && ix[i] <= mid; }) >= need) b = mid;
            else a = mid + 1;
        }
        I = a;
    }
    // ordered compaction of the kept slots into [0, kk)
    int base = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        if (i >= ns) break;
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
__global__ __launch_bounds__(64 * kNnWaves) void k_knn(const float* __restrict__ SX, const float* __restrict__ SY,
                                                       const float* __restrict__ SZ, int64_t nf, NGrid g,
                                                       const int32_t* __restrict__ cstart,
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
        const int q = (int)sorted_idx[qi];  // queries in cell order: a block's queries are close
        const float qx = SX[qi], qy = SY[qi], qz = SZ[qi];
        const int cx = cell_of(g, qx, 0), cy = cell_of(g, qy, 1), cz = cell_of(g, qz, 2);
        int fill = 0;
        // rings 1, 2, 4, ...: an isolated point (few neighbours near it) reaches its k-th neighbour
        // in O(log) ring scans instead of one per cell of distance
        for (int r = 1;; r = min(2 * r, rmax)) {
            fill = 0;
            const int ax0 = max(cx - r, 0), ax1 = min(cx + r, g.dim[0] - 1);
            const int ay0 = max(cy - r, 0), ay1 = min(cy + r, g.dim[1] - 1);
            const int az0 = max(cz - r, 0), az1 = min(cz + r, g.dim[2] - 1);
            // cells (ax0..ax1, b, c) are consecutive keys, so each (b, c) row of the ring is one
            // contiguous range of the cell-sorted points: its bounds for up to 64 rows are loaded
            // at once (one lane per row), then the rows are streamed in order
            const int nb = ay1 - ay0 + 1, nrows = nb * (az1 - az0 + 1);
            for (int r0 = 0; r0 < nrows; r0 += 64) {
                int rb = 0, re = 0;
                if (r0 + lane < nrows) {
                    const int b = ay0 + (r0 + lane) % nb, c = az0 + (r0 + lane) / nb;
                    const int64_t row = (int64_t)g.dim[0] * ((int64_t)b + (int64_t)g.dim[1] * c);
                    rb = cstart[row + ax0];
                    re = cstart[row + ax1 + 1];
                }
                const int nr = min(64, nrows - r0);
                for (int ri = 0; ri < nr; ++ri) {
                    const int beg = __builtin_amdgcn_readlane(rb, ri);
                    const int cnt = __builtin_amdgcn_readlane(re, ri) - beg;
                    for (int t0 = 0; t0 < cnt; t0 += 64) {
                        if (fill + 64 > kNnCap) fill = nn_select(bd, bi, fill, kk, lane);
                        const int t = beg + t0 + lane;
                        if (t0 + lane < cnt) {
                            const float dx = qx - SX[t], dy = qy - SY[t], dz = qz - SZ[t];
                            const float d2 = (dx * dx + dy * dy) + dz * dz;  // FLANN L2_Simple
                            bd[fill + lane] = __float_as_uint(d2);
                            bi[fill + lane] = (int32_t)sorted_idx[t];
                        }
                        fill += min(64, cnt - t0);
                    }
                }
            }
            const bool all = r >= rmax;
            if (fill < kk && !all) continue;
            fill = nn_select(bd, bi, fill, kk, lane);
            // the k-th distance (max of the kept) against the nearest possible outside point
            float dk = 0.0f;  // fill <= kk <= 64: one slot per lane
            if (lane < fill) dk = __uint_as_float(bd[lane]);
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
        int32_t* cstart = (int32_t*)ctx->buf("nrm_cstart", (size_t)(cells + 1) * 4);
        float* sxyz = (float*)ctx->buf("nrm_sxyz", (size_t)nf * 12);
        if (!cstart || !sxyz) return ctx->fail(PITT_E_NOMEM, "normals cell table");
        int32_t* ccnt = (int32_t*)ctx->buf("nrm_ccnt", (size_t)(cells + 1) * 4);
        if (!ccnt) return ctx->fail(PITT_E_NOMEM, "normals cell counts");
        PITT_HIP_TRY(hipMemsetAsync(ccnt, 0, (size_t)(cells + 1) * 4, s));
        hipLaunchKernelGGL(k_cell_count, dim3(grid_for_tiles(ctiles(nf))), dim3(kBlock), 0, s, skey, nf, ccnt);
        size_t scan_bytes = 0;
        PITT_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, ccnt, cstart, (int)(cells + 1), s));
        void* scan_tmp = ctx->buf("nrm_scan_tmp", std::max<size_t>(scan_bytes, 16));
        if (!scan_tmp) return ctx->fail(PITT_E_NOMEM, "normals scan scratch");
        PITT_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, ccnt, cstart, (int)(cells + 1), s));
        hipLaunchKernelGGL(k_gather_sorted, dim3(grid_for_tiles(ctiles(nf))), dim3(kBlock), 0, s, x, y, z, sval, nf,
                           sxyz, sxyz + nf, sxyz + 2 * nf);
        ctx->prof_end(rec);
        PITT_HIP_TRY(hipGetLastError());
        // the finite points in input order are the queries: sval holds them sorted by cell, which
        // keeps a block's queries spatially close
        rec = ctx->prof_begin("k_knn", (double)nf * (12.0 + 4.0 * k));
        const int kb = (int)std::min<int64_t>((nf + kNnWaves - 1) / kNnWaves, 65536);
        hipLaunchKernelGGL(k_knn<kNnMaxK>, dim3(kb), dim3(64 * kNnWaves), 0, s, sxyz, sxyz + nf, sxyz + 2 * nf, nf, g,
                           cstart, sval, k, kk, nnd, cntd);
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

// ------------------------------------------------------------------------------------------
// A batch of small clouds (a frame's clusters, pitt_classify_clusters): PCManager::estimateNormal on
// each cluster on its own, all clusters in one pass.  The k nearest finite points of a query are taken
// from its own cluster by exhaustive search (the same candidates, distances, nn_select and final
// (distance, index) sort as k_knn: identical lists), so no per-cluster grid set-up and no host round
// trip.  Clusters of more than kSegBrute points go through normals_impl one by one.
constexpr int64_t kSegBrute = 16384;

__global__ void k_seg_finite(const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
                             const int64_t* __restrict__ off, const int64_t* __restrict__ cnt, int k,
                             int32_t* __restrict__ kk) {
    const int c = blockIdx.x;
    __shared__ int part[kBlock / 64];
    int f = 0;
    for (int64_t i = threadIdx.x; i < cnt[c]; i += kBlock) {
        const int64_t j = off[c] + i;
        f += fin3(X[j], Y[j], Z[j]) ? 1 : 0;
    }
    f = wave_sum_i(f);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = f;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += part[w];
        kk[c] = t < k ? t : k;
    }
}

// one wave per query; queries numbered over the clusters (qpre: exclusive prefix of the counts)
template <int KMAX>
__global__ __launch_bounds__(64 * kNnWaves) void k_knn_seg(const float* __restrict__ X, const float* __restrict__ Y,
                                                           const float* __restrict__ Z, const int64_t* __restrict__ off,
                                                           const int64_t* __restrict__ cnt,
                                                           const int64_t* __restrict__ qpre, int nc,
                                                           const int32_t* __restrict__ kks, int k,
                                                           int32_t* __restrict__ nn, int32_t* __restrict__ nn_cnt) {
    __shared__ uint32_t s_d[kNnWaves][kNnCap];
    __shared__ int32_t s_i[kNnWaves][kNnCap];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    uint32_t* bd = s_d[w];
    int32_t* bi = s_i[w];
    const int64_t total = qpre[nc];
    for (int64_t qi = (int64_t)blockIdx.x * kNnWaves + w; qi < total; qi += (int64_t)gridDim.x * kNnWaves) {
        int lo = 0, hi = nc - 1;  // the cluster: last c with qpre[c] <= qi
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (qpre[mid] <= qi) lo = mid;
            else hi = mid - 1;
        }
        const int c = lo;
        const int64_t base = off[c], n = cnt[c];
        const int64_t q = base + (qi - qpre[c]);
        const int kk = kks[c];
        const float qx = X[q], qy = Y[q], qz = Z[q];
        if (n > kSegBrute || !fin3(qx, qy, qz) || kk < 1) {  // large clusters: normals_impl
            if (lane == 0 && n <= kSegBrute) nn_cnt[q] = 0;
            continue;
        }
        int fill = 0;
        for (int64_t t0 = 0; t0 < n; t0 += 64) {
            if (fill + 64 > kNnCap) fill = nn_select(bd, bi, fill, kk, lane);
            const int64_t t = t0 + lane;
            bool ok = false;
            float d2 = 0.0f;
            if (t < n) {
                const float px = X[base + t], py = Y[base + t], pz = Z[base + t];
                ok = fin3(px, py, pz);
                const float dx = qx - px, dy = qy - py, dz = qz - pz;
                d2 = (dx * dx + dy * dy) + dz * dz;  // FLANN L2_Simple
            }
            const uint64_t b = __builtin_amdgcn_ballot_w64(ok);
            const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            if (ok) {
                bd[fill + pre] = __float_as_uint(d2);
                bi[fill + pre] = (int32_t)(base + t);
            }
            fill += __builtin_popcountll(b);
        }
        fill = nn_select(bd, bi, fill, kk, lane);
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
        if (lane < fill) nn[q * k + lane] = (int32_t)(uint32_t)key;
        if (lane == 0) nn_cnt[q] = fill;
    }
}

// Normals of nc clusters laid out in one device SoA of n_total points (cluster c at off[c], cnt[c]
// points; other points are never neighbours and get no normal written).  off / cnt: host arrays.
int normals_batch(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n_total, const int64_t* off,
                  const int64_t* cnt, int nc, int k, const float vp[3], float* nx, float* ny, float* nz, float* curv) {
    hipStream_t s = ctx->stream;
    if (nc == 0 || n_total == 0) return PITT_OK;
    if (k < 1 || k > kNnMaxK) return ctx->fail(PITT_E_INVALID, "k must be in [1, 64]");
    int64_t* dm = (int64_t*)ctx->buf("nrmb_meta", (size_t)(3 * nc + 1) * 8);
    int64_t* hm = (int64_t*)ctx->pinned("nrmb_meta_h", (size_t)(3 * nc + 1) * 8);
    int32_t* kk = (int32_t*)ctx->buf("nrmb_kk", (size_t)nc * 4);
    int32_t* nnd = (int32_t*)ctx->buf("nrmb_nn", (size_t)n_total * k * 4);
    int32_t* cntd = (int32_t*)ctx->buf("nrmb_cnt", (size_t)n_total * 4);
    if (!dm || !hm || !kk || !nnd || !cntd) return ctx->fail(PITT_E_NOMEM, "batched normals scratch");
    for (int c = 0; c < nc; ++c) {
        hm[c] = off[c];
        hm[nc + c] = cnt[c];
    }
    hm[2 * nc] = 0;
    for (int c = 0; c < nc; ++c) hm[2 * nc + c + 1] = hm[2 * nc + c] + cnt[c];
    PITT_HIP_TRY(hipMemcpyAsync(dm, hm, (size_t)(3 * nc + 1) * 8, hipMemcpyHostToDevice, s));
    PITT_HIP_TRY(hipMemsetAsync(cntd, 0, (size_t)n_total * 4, s));
    int rec = ctx->prof_begin("k_knn_seg", (double)hm[3 * nc] * (12.0 + 4.0 * k));
    hipLaunchKernelGGL(k_seg_finite, dim3(nc), dim3(kBlock), 0, s, x, y, z, dm, dm + nc, k, kk);
    const int kb = (int)std::max<int64_t>(1, std::min<int64_t>((hm[3 * nc] + kNnWaves - 1) / kNnWaves, 65536));
    hipLaunchKernelGGL(k_knn_seg<kNnMaxK>, dim3(kb), dim3(64 * kNnWaves), 0, s, x, y, z, dm, dm + nc, dm + 2 * nc, nc,
                       kk, k, nnd, cntd);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    rec = ctx->prof_begin("k_normals", (double)n_total * 28.0);
    hipLaunchKernelGGL(k_normals, dim3(std::max<int64_t>(1, std::min<int64_t>((n_total + kBlock - 1) / kBlock, 8192))),
                       dim3(kBlock), 0, s, x, y, z, n_total, nnd, cntd, k, vp[0], vp[1], vp[2], nx, ny, nz, curv);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    // large clusters: the grid path, one at a time
    for (int c = 0; c < nc; ++c) {
        if (cnt[c] <= kSegBrute) continue;
        const int rc = normals_impl(ctx, x + off[c], y + off[c], z + off[c], cnt[c], k, vp, nx + off[c], ny + off[c],
                                    nz + off[c], curv + off[c], nullptr, nullptr);
        if (rc != PITT_OK) return rc;
    }
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
