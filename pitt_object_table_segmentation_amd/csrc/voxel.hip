// voxel.hip -- pcl::VoxelGrid<PointXYZ>::filter as called by PCManager::downSampling
// (src/point_cloud_library/pc_manager.cpp:55-67, leaf 0.01 m from :19), the first step of
// depthAcquisition (src/obj_segmentation.cpp:238); SURVEY.md s8f row 1.
//
// PCL 1.7's applyFilter (filters/impl/voxel_grid.hpp; restated in oracle/pitt_oracle.cpp):
//   1. min / max over the finite points (float);
//   2. (int64)((max - min) * inv) + 1 per axis with inv = 1.0f / leaf; a product above INT32_MAX
//      makes the filter warn and return the input cloud unchanged;
//   3. min_b = (int)floor(min * inv), div_b = max_b - min_b + 1, divb_mul = (1, div_b0, div_b0 div_b1);
//   4. idx = sum_k (int)(floor(p_k * inv_k) - (float)min_b_k) * divb_mul_k per finite point;
//   5. sort the (idx, point index) pairs by idx; one output point per run of equal idx, ascending
//      idx: the float sum of the run's points in run order, then `centroid /= n` (Eigen 3.2: times
//      1.0f / n, A9).
//
// Device pipeline (all on the context stream):
//   k_vox_minmax  -> per-block finite min / max / count            12 B per point
//   k_vox_setup   -> grid parameters (one block)
//   compaction    -> (idx, point index) of the finite points, input order   12 B read, 8 B written
//   radix sort    -> hipCUB DeviceRadixSort::SortPairs (stable) on the bits the grid needs
//   compaction    -> first position of every run of equal idx
//   k_vox_centroid -> one thread per voxel: the run's points summed in run order, times 1 / n
//
// Run order: PCL's std::sort is not stable, so its order of the points inside one voxel is
// libstdc++'s introsort permutation, and the float centroid depends on it in its last bits.
// PITT_VOXEL_ORDER_PCL reproduces that permutation (introsort.hip: the introsort partitions on the
// device, then the stable sort) -- bit-exact against PCL's order under A10; PITT_VOXEL_ORDER_STABLE
// sorts stably (ascending point index inside a voxel, faster), within the float reordering bound of
// PCL's centroids.  The voxel set, their order and every count are PCL's in both modes.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

#include <algorithm>
#include <cfloat>
#include <climits>

#include "compact.hpp"
#include "ctx.hpp"
#include "device_common.hpp"

#pragma clang fp contract(off)

namespace pitt {

struct VoxParams {
    float inv[3];
    int32_t min_b[3];
    int32_t mul[3];
    int64_t n_finite;
    int64_t cells;   // div_b0 * div_b1 * div_b2 (int64): the idx range the sort must cover
    int32_t overflow;
    int32_t pad;
};

constexpr int kVoxBlocks = 1024;

__device__ __forceinline__ bool finite3(float x, float y, float z) {
    return __builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z);
}

// per block: min/max over its finite points and their count -> part[b * 8 + {0..5, 6 (count as bits)}]
__global__ __launch_bounds__(kBlock) void k_vox_minmax(const float* __restrict__ X, const float* __restrict__ Y,
                                                       const float* __restrict__ Z, int64_t n,
                                                       float* __restrict__ part, int64_t* __restrict__ part_n) {
    __shared__ float red[6][kBlock / 64];
    __shared__ int64_t redn[kBlock / 64];
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    int64_t cnt = 0;
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const float x = X[i], y = Y[i], z = Z[i];
        if (!finite3(x, y, z)) continue;
        ++cnt;
        // Eigen's Array4f min / max: std::min(a, b) = (b < a) ? b : a
        v[0] = x < v[0] ? x : v[0];
        v[1] = y < v[1] ? y : v[1];
        v[2] = z < v[2] ? z : v[2];
        v[3] = v[3] < x ? x : v[3];
        v[4] = v[4] < y ? y : v[4];
        v[5] = v[5] < z ? z : v[5];
    }
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) v[k] = fminf(v[k], __shfl_xor(v[k], off, 64));
#pragma unroll
        for (int k = 3; k < 6; ++k) v[k] = fmaxf(v[k], __shfl_xor(v[k], off, 64));
        cnt += __shfl_xor(cnt, off, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) red[k][w] = v[k];
        redn[w] = cnt;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        float r = red[threadIdx.x][0];
        for (int j = 1; j < kBlock / 64; ++j)
            r = threadIdx.x < 3 ? fminf(r, red[threadIdx.x][j]) : fmaxf(r, red[threadIdx.x][j]);
        part[blockIdx.x * 8 + threadIdx.x] = r;
    }
    if (threadIdx.x == 0) {
        int64_t c = 0;
        for (int j = 0; j < kBlock / 64; ++j) c += redn[j];
        part_n[blockIdx.x] = c;
    }
}

// One wave: combine the block partials (min / max are order-free; the partials are finite or the
// FLT_MAX sentinels), then PCL's grid arithmetic in float / int on lane 0.
__global__ __launch_bounds__(64) void k_vox_setup(const float* __restrict__ part, const int64_t* __restrict__ part_n,
                                                  int blocks, float lx, float ly, float lz, VoxParams* __restrict__ out) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    int64_t nf = 0;
    for (int b = threadIdx.x; b < blocks; b += 64) {
        for (int k = 0; k < 3; ++k) {
            mn[k] = fminf(mn[k], part[b * 8 + k]);
            mx[k] = fmaxf(mx[k], part[b * 8 + 3 + k]);
        }
        nf += part_n[b];
    }
    for (int off = 32; off > 0; off >>= 1) {
        for (int k = 0; k < 3; ++k) {
            mn[k] = fminf(mn[k], __shfl_xor(mn[k], off, 64));
            mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], off, 64));
        }
        nf += __shfl_xor(nf, off, 64);
    }
    if (threadIdx.x != 0) return;
    VoxParams p;
    p.inv[0] = 1.0f / lx;
    p.inv[1] = 1.0f / ly;
    p.inv[2] = 1.0f / lz;
    p.n_finite = nf;
    p.overflow = 0;
    p.pad = 0;
    p.cells = 0;
    for (int k = 0; k < 3; ++k) p.min_b[k] = p.mul[k] = 0;
    if (nf > 0) {
        int64_t d[3];
        for (int k = 0; k < 3; ++k) d[k] = (int64_t)((mx[k] - mn[k]) * p.inv[k]) + 1;
        // the check PCL makes (a product of three values below ~2^31 each cannot wrap int64 here
        // unless the first two already exceed INT32_MAX)
        const bool big = d[0] > INT32_MAX || d[1] > INT32_MAX || d[2] > INT32_MAX ||
                         d[0] * d[1] > (int64_t)INT32_MAX || d[0] * d[1] * d[2] > (int64_t)INT32_MAX;
        p.overflow = big ? 1 : 0;
        if (!big) {
            int32_t div_b[3];
            for (int k = 0; k < 3; ++k) {
                p.min_b[k] = (int32_t)floorf(mn[k] * p.inv[k]);
                div_b[k] = (int32_t)floorf(mx[k] * p.inv[k]) - p.min_b[k] + 1;
            }
            p.mul[0] = 1;
            p.mul[1] = div_b[0];
            p.mul[2] = (int32_t)((uint32_t)div_b[0] * (uint32_t)div_b[1]);  // int arithmetic, wraps like x86
            p.cells = (int64_t)div_b[0] * div_b[1] * div_b[2];
        }
    }
    *out = p;
}

struct FinitePoint {
    const float *x, *y, *z;
    __device__ bool operator()(int64_t i) const { return finite3(x[i], y[i], z[i]); }
};

struct WriteVoxKey {
    const float *x, *y, *z;
    const VoxParams* p;
    uint32_t* key;
    uint32_t* val;
    __device__ void operator()(int64_t i, int64_t pos) const {
        const VoxParams& q = *p;
        const int32_t i0 = (int32_t)(floorf(x[i] * q.inv[0]) - (float)q.min_b[0]);
        const int32_t i1 = (int32_t)(floorf(y[i] * q.inv[1]) - (float)q.min_b[1]);
        const int32_t i2 = (int32_t)(floorf(z[i] * q.inv[2]) - (float)q.min_b[2]);
        // int products and sums as PCL's (two's complement wrap on overflow, as x86)
        const uint32_t idx = (uint32_t)i0 * (uint32_t)q.mul[0] + (uint32_t)i1 * (uint32_t)q.mul[1] +
                             (uint32_t)i2 * (uint32_t)q.mul[2];
        key[pos] = idx;
        val[pos] = (uint32_t)i;
    }
};

struct RunHead {
    const uint32_t* key;
    __device__ bool operator()(int64_t i) const { return i == 0 || key[i] != key[i - 1]; }
};

struct WriteStart {
    int32_t* start;
    __device__ void operator()(int64_t i, int64_t pos) const { start[pos] = (int32_t)i; }
};

// One thread per voxel v < n_vox (= run_offsets[n_tiles]): PCL's centroid of the run.
__global__ __launch_bounds__(kBlock) void k_vox_centroid(const float* __restrict__ X, const float* __restrict__ Y,
                                                         const float* __restrict__ Z,
                                                         const uint32_t* __restrict__ val,
                                                         const int32_t* __restrict__ start,
                                                         const int32_t* __restrict__ n_vox_ptr, int64_t nf,
                                                         float* __restrict__ ox, float* __restrict__ oy,
                                                         float* __restrict__ oz) {
    const int64_t n_vox = *n_vox_ptr;
    for (int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x; v < n_vox; v += (int64_t)gridDim.x * kBlock) {
        const int64_t a = start[v], b = v + 1 < n_vox ? start[v + 1] : nf;
        uint32_t j = val[a];
        float sx = X[j], sy = Y[j], sz = Z[j];
        for (int64_t k = a + 1; k < b; ++k) {
            j = val[k];
            sx += X[j];
            sy += Y[j];
            sz += Z[j];
        }
        const float r = 1.0f / (float)(b - a);
        ox[v] = sx * r;
        oy[v] = sy * r;
        oz[v] = sz * r;
    }
}

int introsort_partitions(pitt_ctx* ctx, uint32_t* key, uint32_t* val, int64_t n, int depth_limit);
int introsort_final(pitt_ctx* ctx, const uint32_t* key, const uint32_t* val, int64_t n, uint32_t* ko, uint32_t* vo);

static int voxel_impl(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, float lx, float ly,
                      float lz, int32_t order, float* ox, float* oy, float* oz, int64_t* n_out, int32_t* flags) {
    hipStream_t s = ctx->stream;
    *n_out = 0;
    if (flags) *flags = 0;
    if (n == 0) return PITT_OK;
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, kVoxBlocks));
    float* part = (float*)ctx->buf("vox_part", (size_t)kVoxBlocks * 8 * 4);
    int64_t* part_n = (int64_t*)ctx->buf("vox_part_n", (size_t)kVoxBlocks * 8);
    VoxParams* prm = (VoxParams*)ctx->buf("vox_params", sizeof(VoxParams));
    if (!part || !part_n || !prm) return ctx->fail(PITT_E_NOMEM, "voxel scratch");
    int rec = ctx->prof_begin("k_vox_minmax", (double)n * 12.0);
    hipLaunchKernelGGL(k_vox_minmax, dim3(blocks), dim3(kBlock), 0, s, x, y, z, n, part, part_n);
    ctx->prof_end(rec);
    hipLaunchKernelGGL(k_vox_setup, dim3(1), dim3(64), 0, s, part, part_n, blocks, lx, ly, lz, prm);
    PITT_HIP_TRY(hipGetLastError());
    VoxParams* hp = (VoxParams*)ctx->pinned("vox_params_h", sizeof(VoxParams));
    if (!hp) return ctx->fail(PITT_E_NOMEM, "voxel pinned");
    PITT_HIP_TRY(hipMemcpyAsync(hp, prm, sizeof(VoxParams), hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    const VoxParams P = *hp;
    if (P.n_finite == 0) return PITT_OK;
    if (P.overflow) {  // "Leaf size is too small for the input dataset": the output is the input
        PITT_HIP_TRY(hipMemcpyAsync(ox, x, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
        PITT_HIP_TRY(hipMemcpyAsync(oy, y, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
        PITT_HIP_TRY(hipMemcpyAsync(oz, z, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        *n_out = n;
        if (flags) *flags = PITT_VOXEL_OVERFLOW_COPY;
        return PITT_OK;
    }
    const int64_t nf = P.n_finite;
    // (idx, point index) of the finite points in input order
    const int64_t nt = ctiles(n);
    int32_t* tc = (int32_t*)ctx->buf("vox_tc", (size_t)(nt + 1) * 4);
    int32_t* to = (int32_t*)ctx->buf("vox_to", (size_t)(nt + 1) * 4);
    uint32_t* key = (uint32_t*)ctx->buf("vox_key", (size_t)nf * 4);
    uint32_t* val = (uint32_t*)ctx->buf("vox_val", (size_t)nf * 4);
    uint32_t* key2 = (uint32_t*)ctx->buf("vox_key2", (size_t)nf * 4);
    uint32_t* val2 = (uint32_t*)ctx->buf("vox_val2", (size_t)nf * 4);
    if (!tc || !to || !key || !val || !key2 || !val2) return ctx->fail(PITT_E_NOMEM, "voxel keys");
    const int g = grid_for_tiles(nt);
    FinitePoint fin{x, y, z};
    rec = ctx->prof_begin("k_vox_keys", (double)n * 24.0 + (double)nf * 8.0);
    hipLaunchKernelGGL(k_pred_count<FinitePoint>, dim3(g), dim3(kBlock), 0, s, fin, n, tc);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, tc, nt, to);
    hipLaunchKernelGGL((k_pred_apply<FinitePoint, WriteVoxKey>), dim3(g), dim3(kBlock), 0, s, fin,
                       WriteVoxKey{x, y, z, prm, key, val}, n, to);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    // PCL order: the partitions of libstdc++'s introsort first (introsort.hip); the stable sort then
    // gives std::sort's permutation.  Stable order: the sort alone.
    if (order == PITT_VOXEL_ORDER_PCL) {
        rec = ctx->prof_begin("vox_introsort", (double)nf * 8.0);
        const int irc = introsort_partitions(ctx, key, val, nf, -1);
        ctx->prof_end(rec);
        if (irc != PITT_OK) return irc;
    }
    const uint32_t* sk;
    const uint32_t* sv;
    if (order == PITT_VOXEL_ORDER_PCL) {  // __final_insertion_sort: every element is within 15 of its place
        rec = ctx->prof_begin("vox_final_sort", (double)nf * 16.0);
        const int frc = introsort_final(ctx, key, val, nf, key2, val2);
        ctx->prof_end(rec);
        if (frc != PITT_OK) return frc;
        sk = key2;
        sv = val2;
    } else {  // stable LSD radix sort of the keys over the bits the grid uses
        int end_bit = 1;
        while (end_bit < 32 && ((int64_t)1 << end_bit) < P.cells) ++end_bit;
        if (P.cells > (int64_t)UINT32_MAX) end_bit = 32;  // wrapped int indices: sort every bit
        hipcub::DoubleBuffer<uint32_t> kb(key, key2), vb(val, val2);
        size_t tmp_bytes = 0;
        PITT_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kb, vb, (int)nf, 0, end_bit, s));
        void* tmp = ctx->buf("vox_sort_tmp", std::max<size_t>(tmp_bytes, 16));
        if (!tmp) return ctx->fail(PITT_E_NOMEM, "voxel sort scratch");
        rec = ctx->prof_begin("vox_radix_sort", (double)nf * 16.0);
        PITT_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kb, vb, (int)nf, 0, end_bit, s));
        ctx->prof_end(rec);
        sk = kb.Current();
        sv = vb.Current();
    }
    // runs of equal idx: their first positions, ascending
    const int64_t ntf = ctiles(nf);
    int32_t* rc = (int32_t*)ctx->buf("vox_rc", (size_t)(ntf + 1) * 4);
    int32_t* ro = (int32_t*)ctx->buf("vox_ro", (size_t)(ntf + 1) * 4);
    int32_t* start = (int32_t*)ctx->buf("vox_start", (size_t)nf * 4);
    if (!rc || !ro || !start) return ctx->fail(PITT_E_NOMEM, "voxel runs");
    const int gf = grid_for_tiles(ntf);
    RunHead head{sk};
    rec = ctx->prof_begin("k_vox_runs", (double)nf * 8.0);
    hipLaunchKernelGGL(k_pred_count<RunHead>, dim3(gf), dim3(kBlock), 0, s, head, nf, rc);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, rc, ntf, ro);
    hipLaunchKernelGGL((k_pred_apply<RunHead, WriteStart>), dim3(gf), dim3(kBlock), 0, s, head, WriteStart{start},
                       nf, ro);
    ctx->prof_end(rec);
    rec = ctx->prof_begin("k_vox_centroid", (double)nf * 16.0);
    hipLaunchKernelGGL(k_vox_centroid, dim3(grid_for_tiles(ntf) * 8), dim3(kBlock), 0, s, x, y, z, sv, start,
                       ro + ntf, nf, ox, oy, oz);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    int32_t* hv = (int32_t*)ctx->pinned("vox_nvox", 16);
    if (!hv) return ctx->fail(PITT_E_NOMEM, "voxel pinned");
    PITT_HIP_TRY(hipMemcpyAsync(hv, ro + ntf, 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    *n_out = hv[0];
    return PITT_OK;
}

}  // namespace pitt

extern "C" int pitt_voxel_grid(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                               float leaf_x, float leaf_y, float leaf_z, int32_t order, float* out_x, float* out_y,
                               float* out_z, int64_t* n_out, int32_t* flags) {
    if (!ctx) return PITT_E_INVALID;
    if (order != PITT_VOXEL_ORDER_PCL && order != PITT_VOXEL_ORDER_STABLE) return ctx->fail(PITT_E_INVALID, "order");
    if (!n_out || n < 0 || (n > 0 && (!x || !y || !z || !out_x || !out_y || !out_z)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "cloud larger than 2^31 points");
    if (!(leaf_x > 0.0f) || !(leaf_y > 0.0f) || !(leaf_z > 0.0f)) return ctx->fail(PITT_E_INVALID, "leaf size");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    return pitt::voxel_impl(ctx, x, y, z, n, leaf_x, leaf_y, leaf_z, order, out_x, out_y, out_z, n_out, flags);
}

extern "C" int pitt_sort_pairs(pitt_ctx* ctx, uint32_t* key, uint32_t* val, int64_t n, int32_t depth_limit) {
    if (!ctx) return PITT_E_INVALID;
    if (n < 0 || (n > 0 && (!key || !val))) return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "more than 2^31 pairs");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    if (n < 2) return PITT_OK;
    hipStream_t s = ctx->stream;
    int rc = pitt::introsort_partitions(ctx, key, val, n, depth_limit);
    if (rc != PITT_OK) return rc;
    uint32_t* k2 = (uint32_t*)ctx->buf("sp_k2", (size_t)n * 4);
    uint32_t* v2 = (uint32_t*)ctx->buf("sp_v2", (size_t)n * 4);
    if (!k2 || !v2) return ctx->fail(PITT_E_NOMEM, "sort scratch");
    rc = pitt::introsort_final(ctx, key, val, n, k2, v2);  // __final_insertion_sort
    if (rc != PITT_OK) return rc;
    PITT_HIP_TRY(hipMemcpyAsync(key, k2, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    PITT_HIP_TRY(hipMemcpyAsync(val, v2, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    return PITT_OK;
}
