// primitives.hip -- the device side of the normal-based primitive services:
// the axis "height" post-processing that cylinder_segmentation_srv.cpp:129-189 and
// cone_segmentation_srv.cpp:129-189 run on the cloud once PCL has fitted the model:
//
//   1. the axis direction c[3..5] / |c[3..5]|, two axis points A1 = c - d, A2 = c + d (:53-79);
//   2. every point P projected on the axis: A1 + G (A2 - A1), G = dot(P - A1, A1A2) / dot(A1A2, A1A2)
//      (:141-154);
//   3. the pair (i > j) of projected points farthest apart -- float distance
//      sqrt((dx dx + dy dy) + dz dz), the first maximum in the reference's (i, j) loop order
//      (:156-171, O(n^2));
//   4. the centroid: cylinder, the midpoint of that pair (:173-176); cone, c + 3/4 height d (:173-176).
//
// Every float operation is the reference's, in source order, without FMA (restated in
// oracle/pitt_oracle.cpp: orc_axis_height).  Step 3 is exact without a square root per pair: sqrt is
// monotonic, so the height is sqrt(max s) over the pairs' squared sums s, and the pairs whose distance
// equals it are those with s >= s_lo, the smallest float whose sqrt rounds to the height.  Two passes
// over the pairs: the maximum s (an order-free float max), then the first pair (minimum i n + j) at
// or above s_lo.
//
// Kernels (one 256-point i tile x one 256-point j tile per block, j tile <= i tile, the j tile staged
// in LDS and read by broadcast ds_read_b128; per pair 3 v_sub + 3 v_mul + 2 v_add + 1 v_max):
//   k_axis_project   12 B read + 12 B written per point                 HBM
//   k_pair_max       9 VALU ops per pair, one 64-lane wave per tile pair with four i points per
//                    lane (one LDS read per four pairs), one atomic per tile pair   VALU (n^2 / 2 pairs)
//   k_pair_first     the first pair at or above s_lo, only in the tile pairs whose maximum (kept
//                    by k_pair_max) reaches it                           a few tiles
//   k_axis_final     height, indices, centroid (one thread)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "ctx.hpp"
#include "device_common.hpp"

#pragma clang fp contract(off)

namespace pitt {

struct AxisGeo {
    float c[3], d[3];  // the model's axis point and the normalised direction
    float a1[3], u[3];  // A1 and A1A2
    float gdiv;
};

constexpr int kPairTile = 256;

__global__ __launch_bounds__(256) void k_axis_project(const float* __restrict__ X, const float* __restrict__ Y,
                                                      const float* __restrict__ Z, int64_t n, AxisGeo G,
                                                      float* __restrict__ qx, float* __restrict__ qy,
                                                      float* __restrict__ qz) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float vx = X[i] - G.a1[0], vy = Y[i] - G.a1[1], vz = Z[i] - G.a1[2];
        const float g = (vx * G.u[0] + vy * G.u[1] + vz * G.u[2]) / G.gdiv;
        qx[i] = G.a1[0] + g * G.u[0];
        qy[i] = G.a1[1] + g * G.u[1];
        qz[i] = G.a1[2] + g * G.u[2];
    }
}

// tile pair t -> (ti, tj) with tj <= ti: t = ti (ti + 1) / 2 + tj
__device__ __forceinline__ void pair_tile(int64_t t, int& ti, int& tj) {
    int a = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((int64_t)(a + 1) * (a + 2) / 2 <= t) ++a;
    while ((int64_t)a * (a + 1) / 2 > t) --a;
    ti = a;
    tj = (int)(t - (int64_t)a * (a + 1) / 2);
}

// the reference's squared sum for points i and j: (dx dx + dy dy) + dz dz, d = p_i - p_j
__device__ __forceinline__ float pair_s(float xi, float yi, float zi, float xj, float yj, float zj) {
    const float ex = xi - xj, ey = yi - yj, ez = zi - zj;
    return ex * ex + ey * ey + ez * ez;
}

__device__ __forceinline__ float vmaxf(float a, float b) {  // IEEE max: a NaN operand never wins
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <bool FIRST>
__global__ __launch_bounds__(kPairTile) void k_pair_scan(const float* __restrict__ qx, const float* __restrict__ qy,
                                                         const float* __restrict__ qz, int64_t n,
                                                         const float* __restrict__ s_lo_p,
                                                         uint32_t* __restrict__ smax_bits,
                                                         unsigned long long* __restrict__ first,
                                                         float* __restrict__ tile_max) {
    __shared__ float4 jq[kPairTile];  // the j tile, one broadcast ds_read_b128 per pair
    // the second pass scans only the tile pairs whose largest s reaches the height
    if (FIRST && !(tile_max[blockIdx.x] >= *s_lo_p)) return;
    __shared__ float red[kPairTile / 64];
    __shared__ unsigned long long redk[kPairTile / 64];
    int ti, tj;
    pair_tile(blockIdx.x, ti, tj);
    const int64_t j0 = (int64_t)tj * kPairTile;
    const int t = threadIdx.x;
    if (j0 + t < n) jq[t] = make_float4(qx[j0 + t], qy[j0 + t], qz[j0 + t], 0.0f);
    __syncthreads();
    const int64_t i = (int64_t)ti * kPairTile + t;
    const int jn = (int)std::min<int64_t>(kPairTile, std::min<int64_t>(n - j0, i - j0));  // j < i, j < n
    float best = -1.0f;  // the largest s (s >= +0; NaN sums never win)
    unsigned long long key = ~0ull;
    if (i < n && jn > 0) {
        const float xi = qx[i], yi = qy[i], zi = qz[i];
        if constexpr (!FIRST) {
            if (jn == kPairTile) {  // off-diagonal tiles: a constant trip count, unrolled
#pragma unroll 16
                for (int j = 0; j < kPairTile; ++j) {
                    const float4 q = jq[j];
                    best = vmaxf(best, pair_s(xi, yi, zi, q.x, q.y, q.z));
                }
            } else {
                for (int j = 0; j < jn; ++j) {
                    const float4 q = jq[j];
                    best = vmaxf(best, pair_s(xi, yi, zi, q.x, q.y, q.z));
                }
            }
        } else {
            const float s_lo = *s_lo_p;
            for (int j = 0; j < jn; ++j) {
                const float4 q = jq[j];
                if (pair_s(xi, yi, zi, q.x, q.y, q.z) >= s_lo) {  // the first j of this i at the height
                    key = (unsigned long long)i * (unsigned long long)n + (unsigned long long)(j0 + j);
                    break;
                }
            }
        }
    }
    const int lane = t & 63, w = t >> 6;
    if constexpr (!FIRST) {
        for (int off = 32; off > 0; off >>= 1) best = vmaxf(best, __shfl_xor(best, off, 64));
        if (lane == 0) red[w] = best;
        __syncthreads();
        if (t == 0) {
            float m = red[0];
            for (int k = 1; k < kPairTile / 64; ++k) m = vmaxf(m, red[k]);
            tile_max[blockIdx.x] = m;
            if (m >= 0.0f) atomicMax(smax_bits, __float_as_uint(m) + 1u);  // 0 = no pair
        }
    } else {
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(key, off, 64);
            key = o < key ? o : key;
        }
        if (lane == 0) redk[w] = key;
        __syncthreads();
        if (t == 0) {
            unsigned long long m = redk[0];
            for (int k = 1; k < kPairTile / 64; ++k) m = redk[k] < m ? redk[k] : m;
            if (m != ~0ull) atomicMin(first, m);
        }
    }
}

// The maximum pass with four i points per thread (one 64-lane wave per tile pair): each broadcast
// ds_read_b128 of a j point feeds four pairs.
__global__ __launch_bounds__(64) void k_pair_max4(const float* __restrict__ qx, const float* __restrict__ qy,
                                                  const float* __restrict__ qz, int64_t n,
                                                  uint32_t* __restrict__ smax_bits, float* __restrict__ tile_max) {
    __shared__ float4 jq[kPairTile];
    int ti, tj;
    pair_tile(blockIdx.x, ti, tj);
    const int64_t j0 = (int64_t)tj * kPairTile, i0 = (int64_t)ti * kPairTile;
    const int lane = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t j = j0 + lane + 64 * k;
        if (j < n) jq[lane + 64 * k] = make_float4(qx[j], qy[j], qz[j], 0.0f);
    }
    __syncthreads();
    float xi[4], yi[4], zi[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = min(i0 + lane + 64 * k, n - 1);
        xi[k] = qx[i];
        yi[k] = qy[i];
        zi[k] = qz[i];
    }
    float best[4] = {-1.0f, -1.0f, -1.0f, -1.0f};
    if (tj < ti && i0 + kPairTile <= n) {  // every j < every i, all in range: a constant trip count
#pragma unroll 8
        for (int j = 0; j < kPairTile; ++j) {
            const float4 q = jq[j];
#pragma unroll
            for (int k = 0; k < 4; ++k) best[k] = vmaxf(best[k], pair_s(xi[k], yi[k], zi[k], q.x, q.y, q.z));
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = i0 + lane + 64 * k;
            const int jn = i < n ? (int)std::min<int64_t>(kPairTile, std::min<int64_t>(n - j0, i - j0)) : 0;
            for (int j = 0; j < jn; ++j) {
                const float4 q = jq[j];
                best[k] = vmaxf(best[k], pair_s(xi[k], yi[k], zi[k], q.x, q.y, q.z));
            }
        }
    }
    float b = vmaxf(vmaxf(best[0], best[1]), vmaxf(best[2], best[3]));
    for (int off = 32; off > 0; off >>= 1) b = vmaxf(b, __shfl_xor(b, off, 64));
    if (lane == 0) {
        tile_max[blockIdx.x] = b;
        if (b >= 0.0f) atomicMax(smax_bits, __float_as_uint(b) + 1u);  // 0 = no pair
    }
}

// AxisOut: height, idx1, idx2, centroid[3]
struct AxisOut {
    float height;
    int32_t idx1, idx2;
    float centroid[3];
};

__global__ void k_axis_final(const float* __restrict__ qx, const float* __restrict__ qy, const float* __restrict__ qz,
                             int64_t n, AxisGeo G, int mode, const uint32_t* __restrict__ smax_bits, const unsigned long long* __restrict__ first,
                             AxisOut* __restrict__ out) {
    AxisOut o;
    o.height = -1.0f;
    o.idx1 = o.idx2 = -1;
    if (*smax_bits) {
        o.height = sqrtf(__uint_as_float(*smax_bits - 1u));
        const unsigned long long k = *first;
        o.idx1 = (int32_t)(k / (unsigned long long)n);
        o.idx2 = (int32_t)(k % (unsigned long long)n);
    }
    if (mode == PITT_AXIS_CYLINDER) {
        const float nan = __builtin_nanf("");
        const bool ok = o.idx1 >= 0;
        o.centroid[0] = ok ? (qx[o.idx1] + qx[o.idx2]) / 2 : nan;
        o.centroid[1] = ok ? (qy[o.idx1] + qy[o.idx2]) / 2 : nan;
        o.centroid[2] = ok ? (qz[o.idx1] + qz[o.idx2]) / 2 : nan;
    } else {
        o.centroid[0] = G.c[0] + 3.0f / 4.0f * o.height * G.d[0];
        o.centroid[1] = G.c[1] + 3.0f / 4.0f * o.height * G.d[1];
        o.centroid[2] = G.c[2] + 3.0f / 4.0f * o.height * G.d[2];
    }
    *out = o;
}

// ------------------------------------------------------------------------------------------
// A batch of axis-height jobs (pitt_classify_clusters: the cylinder and cone services' post-processing
// for every cluster with a model), the same kernels' arithmetic with a job index, no host round trip
// until the results: the smallest s whose sqrt is the height (s_lo) is found on the device.
struct AxisJob {
    AxisGeo G;
    int64_t off;   // the job's points in the SoA
    int64_t qoff;  // its projected copy in the scratch (jobs may share points: a cylinder and a cone)
    int64_t n;
    int64_t tp0;   // the job's first tile pair in the tile-maximum array
    int32_t mode;
    int32_t pad;
};
struct AxisWork {
    uint32_t smax_bits;  // largest s + 1 (0: no pair)
    float s_lo;
    unsigned long long first;
};

__global__ __launch_bounds__(256) void k_axis_project_b(const float* __restrict__ X, const float* __restrict__ Y,
                                                        const float* __restrict__ Z, const AxisJob* __restrict__ jobs,
                                                        float* __restrict__ qx, float* __restrict__ qy,
                                                        float* __restrict__ qz) {
    const AxisJob& J = jobs[blockIdx.y];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < J.n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = J.off + i, q = J.qoff + i;
        const float vx = X[k] - J.G.a1[0], vy = Y[k] - J.G.a1[1], vz = Z[k] - J.G.a1[2];
        const float g = (vx * J.G.u[0] + vy * J.G.u[1] + vz * J.G.u[2]) / J.G.gdiv;
        qx[q] = J.G.a1[0] + g * J.G.u[0];
        qy[q] = J.G.a1[1] + g * J.G.u[1];
        qz[q] = J.G.a1[2] + g * J.G.u[2];
    }
}

// k_pair_scan over job blockIdx.y's tile pairs (blocks past its count return)
template <bool FIRST>
__global__ __launch_bounds__(kPairTile) void k_pair_scan_b(const float* __restrict__ qx, const float* __restrict__ qy,
                                                           const float* __restrict__ qz,
                                                           const AxisJob* __restrict__ jobs, AxisWork* __restrict__ work,
                                                           float* __restrict__ tile_max_all) {
    __shared__ float4 jq[kPairTile];
    __shared__ float red[kPairTile / 64];
    __shared__ unsigned long long redk[kPairTile / 64];
    const AxisJob& J = jobs[blockIdx.y];
    AxisWork* w = work + blockIdx.y;
    const int64_t n = J.n;
    const int64_t tiles = (n + kPairTile - 1) / kPairTile;
    if ((int64_t)blockIdx.x >= tiles * (tiles + 1) / 2) return;
    float* tile_max = tile_max_all + J.tp0;
    if (FIRST && !(w->smax_bits && tile_max[blockIdx.x] >= w->s_lo)) return;
    const float* px = qx + J.qoff;
    const float* py = qy + J.qoff;
    const float* pz = qz + J.qoff;
    int ti, tj;
    pair_tile(blockIdx.x, ti, tj);
    const int64_t j0 = (int64_t)tj * kPairTile;
    const int t = threadIdx.x;
    if (j0 + t < n) jq[t] = make_float4(px[j0 + t], py[j0 + t], pz[j0 + t], 0.0f);
    __syncthreads();
    const int64_t i = (int64_t)ti * kPairTile + t;
    const int jn = (int)std::min<int64_t>(kPairTile, std::min<int64_t>(n - j0, i - j0));
    float best = -1.0f;
    unsigned long long key = ~0ull;
    if (i < n && jn > 0) {
        const float xi = px[i], yi = py[i], zi = pz[i];
        if constexpr (!FIRST) {
            for (int j = 0; j < jn; ++j) {
                const float4 q = jq[j];
                best = vmaxf(best, pair_s(xi, yi, zi, q.x, q.y, q.z));
            }
        } else {
            const float s_lo = w->s_lo;
            for (int j = 0; j < jn; ++j) {
                const float4 q = jq[j];
                if (pair_s(xi, yi, zi, q.x, q.y, q.z) >= s_lo) {
                    key = (unsigned long long)i * (unsigned long long)n + (unsigned long long)(j0 + j);
                    break;
                }
            }
        }
    }
    const int lane = t & 63, wv = t >> 6;
    if constexpr (!FIRST) {
        for (int o = 32; o > 0; o >>= 1) best = vmaxf(best, __shfl_xor(best, o, 64));
        if (lane == 0) red[wv] = best;
        __syncthreads();
        if (t == 0) {
            float m = red[0];
            for (int k = 1; k < kPairTile / 64; ++k) m = vmaxf(m, red[k]);
            tile_max[blockIdx.x] = m;
            if (m >= 0.0f) atomicMax(&w->smax_bits, __float_as_uint(m) + 1u);
        }
    } else {
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long v = __shfl_xor(key, o, 64);
            key = v < key ? v : key;
        }
        if (lane == 0) redk[wv] = key;
        __syncthreads();
        if (t == 0) {
            unsigned long long m = redk[0];
            for (int k = 1; k < kPairTile / 64; ++k) m = redk[k] < m ? redk[k] : m;
            if (m != ~0ull) atomicMin(&w->first, m);
        }
    }
}

// per job: smax = 0, first = ~0; then s_lo, the smallest float whose (correctly rounded) sqrt is the
// height (a positive float's next value towards zero is its bit pattern minus one)
__global__ void k_axis_init_b(AxisWork* __restrict__ work, int nj) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nj) work[j] = AxisWork{0u, 0.0f, ~0ull};
}
__global__ void k_axis_slo_b(AxisWork* __restrict__ work, int nj) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nj || !work[j].smax_bits) return;
    const float smax = __uint_as_float(work[j].smax_bits - 1u);
    const float hgt = sqrtf(smax);
    float lo = smax;
    while (lo > 0.0f && sqrtf(__uint_as_float(__float_as_uint(lo) - 1u)) == hgt) lo = __uint_as_float(__float_as_uint(lo) - 1u);
    work[j].s_lo = lo;
}

__global__ void k_axis_final_b(const float* __restrict__ qx, const float* __restrict__ qy, const float* __restrict__ qz,
                               const AxisJob* __restrict__ jobs, const AxisWork* __restrict__ work, int nj,
                               AxisOut* __restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nj) return;
    const AxisJob& J = jobs[j];
    const AxisWork& w = work[j];
    AxisOut o;
    o.height = -1.0f;
    o.idx1 = o.idx2 = -1;
    if (w.smax_bits) {
        o.height = sqrtf(__uint_as_float(w.smax_bits - 1u));
        o.idx1 = (int32_t)(w.first / (unsigned long long)J.n);
        o.idx2 = (int32_t)(w.first % (unsigned long long)J.n);
    }
    if (J.mode == PITT_AXIS_CYLINDER) {
        const float nan = __builtin_nanf("");
        const bool ok = o.idx1 >= 0;
        const int64_t a = J.qoff + o.idx1, b = J.qoff + o.idx2;
        o.centroid[0] = ok ? (qx[a] + qx[b]) / 2 : nan;
        o.centroid[1] = ok ? (qy[a] + qy[b]) / 2 : nan;
        o.centroid[2] = ok ? (qz[a] + qz[b]) / 2 : nan;
    } else {
        o.centroid[0] = J.G.c[0] + 3.0f / 4.0f * o.height * J.G.d[0];
        o.centroid[1] = J.G.c[1] + 3.0f / 4.0f * o.height * J.G.d[1];
        o.centroid[2] = J.G.c[2] + 3.0f / 4.0f * o.height * J.G.d[2];
    }
    out[j] = o;
}

// the axis geometry, host float arithmetic in the reference's order (:53-79, :143-144)
static AxisGeo axis_geo(const float coef[6]) {
    AxisGeo G;
    const float norm = std::sqrt(coef[3] * coef[3] + coef[4] * coef[4] + coef[5] * coef[5]);
    for (int k = 0; k < 3; ++k) {
        G.c[k] = coef[k];
        G.d[k] = coef[3 + k] / norm;
        G.a1[k] = coef[k] + G.d[k] * -1.0f;
    }
    for (int k = 0; k < 3; ++k) G.u[k] = (coef[k] + G.d[k] * 1.0f) - G.a1[k];
    G.gdiv = G.u[0] * G.u[0] + G.u[1] * G.u[1] + G.u[2] * G.u[2];
    return G;
}

// Jobs over one device SoA of n_total points: job j = points [off[j], off[j] + n[j]), model coef6[j]
// (6 floats, host), mode[j].  Outputs (host): height, idx1, idx2, centroid per job.  One host sync.
int axis_height_batch(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n_total,
                      const int64_t* off, const int64_t* n, const float* coef6, const int32_t* mode, int nj,
                      float* height, int32_t* idx1, int32_t* idx2, float* centroid3) {
    if (nj == 0) return PITT_OK;
    hipStream_t s = ctx->stream;
    AxisJob* hj = (AxisJob*)ctx->pinned("axb_jobs_h", (size_t)nj * sizeof(AxisJob));
    AxisOut* ho = (AxisOut*)ctx->pinned("axb_out_h", (size_t)nj * sizeof(AxisOut));
    AxisJob* dj = (AxisJob*)ctx->buf("axb_jobs", (size_t)nj * sizeof(AxisJob));
    AxisWork* dw = (AxisWork*)ctx->buf("axb_work", (size_t)nj * sizeof(AxisWork));
    AxisOut* dout = (AxisOut*)ctx->buf("axb_out", (size_t)nj * sizeof(AxisOut));
    int64_t q_total = 0;
    for (int j = 0; j < nj; ++j) q_total += n[j];
    const size_t nb = (size_t)std::max<int64_t>(q_total, 1) * 4;
    float* qx = (float*)ctx->buf("axb_qx", nb);
    float* qy = (float*)ctx->buf("axb_qy", nb);
    float* qz = (float*)ctx->buf("axb_qz", nb);
    if (!hj || !ho || !dj || !dw || !dout || !qx || !qy || !qz) return ctx->fail(PITT_E_NOMEM, "axis batch scratch");
    int64_t tp_total = 0, tp_max = 0, n_max = 0, qo = 0;
    for (int j = 0; j < nj; ++j) {
        if (n[j] > 0x7fffffff || off[j] < 0 || off[j] + n[j] > n_total)
            return ctx->fail(PITT_E_INVALID, "axis height job out of range");
        hj[j].G = axis_geo(coef6 + 6 * j);
        hj[j].off = off[j];
        hj[j].qoff = qo;
        qo += n[j];
        hj[j].n = n[j];
        hj[j].tp0 = tp_total;
        hj[j].mode = mode[j];
        hj[j].pad = 0;
        const int64_t tiles = (n[j] + kPairTile - 1) / kPairTile, tp = tiles * (tiles + 1) / 2;
        tp_total += tp;
        tp_max = std::max(tp_max, tp);
        n_max = std::max(n_max, n[j]);
    }
    if (tp_max > 0x7fffffff || nj > 65535) return ctx->fail(PITT_E_INVALID, "axis height: too many jobs / tiles");
    float* tmax = (float*)ctx->buf("axb_tile_max", (size_t)std::max<int64_t>(tp_total, 1) * 4);
    if (!tmax) return ctx->fail(PITT_E_NOMEM, "axis batch tile maxima");
    PITT_HIP_TRY(hipMemcpyAsync(dj, hj, (size_t)nj * sizeof(AxisJob), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_axis_init_b, dim3((nj + 63) / 64), dim3(64), 0, s, dw, nj);
    if (n_max > 0 && tp_max > 0) {
        int rec = ctx->prof_begin("k_axis_project", (double)q_total * 24.0);
        hipLaunchKernelGGL(k_axis_project_b, dim3((unsigned)std::min<int64_t>((n_max + 255) / 256, 1024), (unsigned)nj),
                           dim3(256), 0, s, x, y, z, dj, qx, qy, qz);
        ctx->prof_end(rec);
        rec = ctx->prof_begin("k_pair_max", 0.0);
        hipLaunchKernelGGL(k_pair_scan_b<false>, dim3((unsigned)tp_max, (unsigned)nj), dim3(kPairTile), 0, s, qx, qy, qz,
                           dj, dw, tmax);
        ctx->prof_end(rec);
        hipLaunchKernelGGL(k_axis_slo_b, dim3((nj + 63) / 64), dim3(64), 0, s, dw, nj);
        rec = ctx->prof_begin("k_pair_first", 0.0);
        hipLaunchKernelGGL(k_pair_scan_b<true>, dim3((unsigned)tp_max, (unsigned)nj), dim3(kPairTile), 0, s, qx, qy, qz,
                           dj, dw, tmax);
        ctx->prof_end(rec);
    }
    hipLaunchKernelGGL(k_axis_final_b, dim3((nj + 63) / 64), dim3(64), 0, s, qx, qy, qz, dj, dw, nj, dout);
    PITT_HIP_TRY(hipGetLastError());
    PITT_HIP_TRY(hipMemcpyAsync(ho, dout, (size_t)nj * sizeof(AxisOut), hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    for (int j = 0; j < nj; ++j) {
        height[j] = ho[j].height;
        idx1[j] = ho[j].idx1;
        idx2[j] = ho[j].idx2;
        for (int k = 0; k < 3; ++k) centroid3[3 * j + k] = ho[j].centroid[k];
    }
    return PITT_OK;
}

}  // namespace pitt

extern "C" int pitt_axis_height(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                const float coef[6], int32_t mode, float* px, float* py, float* pz, float* height,
                                int32_t* idx1, int32_t* idx2, float centroid[3]) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (n < 0 || !coef || !height || !idx1 || !idx2 || !centroid || (n > 0 && (!x || !y || !z)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (mode != PITT_AXIS_CYLINDER && mode != PITT_AXIS_CONE) return ctx->fail(PITT_E_INVALID, "mode");
    if ((px || py || pz) && !(px && py && pz)) return ctx->fail(PITT_E_INVALID, "px / py / pz: all or none");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "more than 2^31 points");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    hipStream_t s = ctx->stream;
    // the axis geometry, host float arithmetic in the reference's order (scalar set-up, :53-79, :143-144)
    AxisGeo G;
    const float norm = std::sqrt(coef[3] * coef[3] + coef[4] * coef[4] + coef[5] * coef[5]);
    for (int k = 0; k < 3; ++k) {
        G.c[k] = coef[k];
        G.d[k] = coef[3 + k] / norm;
        G.a1[k] = coef[k] + G.d[k] * -1.0f;
    }
    for (int k = 0; k < 3; ++k) G.u[k] = (coef[k] + G.d[k] * 1.0f) - G.a1[k];
    G.gdiv = G.u[0] * G.u[0] + G.u[1] * G.u[1] + G.u[2] * G.u[2];
    const size_t nb = (size_t)std::max<int64_t>(n, 1) * 4;
    float* qx = px ? px : (float*)ctx->buf("ax_qx", nb);
    float* qy = py ? py : (float*)ctx->buf("ax_qy", nb);
    float* qz = pz ? pz : (float*)ctx->buf("ax_qz", nb);
    uint32_t* w = (uint32_t*)ctx->buf("ax_work", 64);  // [0] s max bits + 1 (0: no pair), [2] s_lo, [4..5] first
    AxisOut* hout = (AxisOut*)ctx->pinned("ax_out", sizeof(AxisOut) + 16);
    if (!qx || !qy || !qz || !w || !hout) return ctx->fail(PITT_E_NOMEM, "axis height scratch");
    unsigned long long* first = (unsigned long long*)(w + 4);
    AxisOut* dout = (AxisOut*)(w + 8);
    PITT_HIP_TRY(hipMemsetAsync(w, 0, 16, s));
    PITT_HIP_TRY(hipMemsetAsync(first, 0xff, 8, s));
    if (n > 0) {
        int rec = ctx->prof_begin("k_axis_project", (double)n * 24.0);
        const int g = (int)std::min<int64_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(k_axis_project, dim3(g), dim3(256), 0, s, x, y, z, n, G, qx, qy, qz);
        ctx->prof_end(rec);
        const int64_t tiles = (n + kPairTile - 1) / kPairTile;
        const int64_t tp = tiles * (tiles + 1) / 2;
        if (tp > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "axis height: too many point tiles");
        float* tmax = (float*)ctx->buf("ax_tile_max", (size_t)tp * 4);
        if (!tmax) return ctx->fail(PITT_E_NOMEM, "axis height tile maxima");
        rec = ctx->prof_begin("k_pair_max", (double)n * (double)(n - 1) / 2.0);
        if (tp >= 4096)  // enough tile pairs to fill the chip with one-wave blocks
            hipLaunchKernelGGL(k_pair_max4, dim3((unsigned)tp), dim3(64), 0, s, qx, qy, qz, n, w, tmax);
        else
            hipLaunchKernelGGL(k_pair_scan<false>, dim3((unsigned)tp), dim3(kPairTile), 0, s, qx, qy, qz, n,
                               (const float*)nullptr, w, first, tmax);
        ctx->prof_end(rec);
        PITT_HIP_TRY(hipGetLastError());
        uint32_t* hw = (uint32_t*)ctx->pinned("ax_w", 16);
        if (!hw) return ctx->fail(PITT_E_NOMEM, "axis height pinned");
        PITT_HIP_TRY(hipMemcpyAsync(hw, w, 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        if (hw[0]) {
            // s_lo: the smallest float whose (correctly rounded) sqrt is the height
            const float smax = __builtin_bit_cast(float, hw[0] - 1u);
            const float hgt = std::sqrt(smax);
            float lo = smax;
            while (lo > 0.0f && std::sqrt(std::nextafter(lo, 0.0f)) == hgt) lo = std::nextafter(lo, 0.0f);
            float* hs = (float*)ctx->pinned("ax_slo", 16);
            if (!hs) return ctx->fail(PITT_E_NOMEM, "axis height pinned");
            *hs = lo;
            PITT_HIP_TRY(hipMemcpyAsync(w + 2, hs, 4, hipMemcpyHostToDevice, s));
            rec = ctx->prof_begin("k_pair_first", (double)n * (double)(n - 1) / 2.0);
            hipLaunchKernelGGL(k_pair_scan<true>, dim3((unsigned)tp), dim3(kPairTile), 0, s, qx, qy, qz, n,
                               (const float*)(w + 2), w, first, tmax);
            ctx->prof_end(rec);
            PITT_HIP_TRY(hipGetLastError());
        }
    }
    hipLaunchKernelGGL(k_axis_final, dim3(1), dim3(1), 0, s, qx, qy, qz, n, G, (int)mode, w, first, dout);
    PITT_HIP_TRY(hipGetLastError());
    PITT_HIP_TRY(hipMemcpyAsync(hout, dout, sizeof(AxisOut), hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    *height = hout->height;
    *idx1 = hout->idx1;
    *idx2 = hout->idx2;
    for (int k = 0; k < 3; ++k) centroid[k] = hout->centroid[k];
    return PITT_OK;
}

// Host-memory form: a PointXYZ cloud (16-byte stride) staged into the context's device buffers.
extern "C" int pitt_axis_height_host(pitt_ctx* ctx, const float* xyz16, int64_t n, const float coef[6], int32_t mode,
                                     float* height, int32_t* idx1, int32_t* idx2, float centroid[3]) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (n < 0 || (n > 0 && !xyz16)) return ctx->fail(PITT_E_INVALID, "null argument");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    const size_t nb = (size_t)std::max<int64_t>(n, 1) * 4;
    float* d = (float*)ctx->buf("ax_hsoa", nb * 3);
    if (!d) return ctx->fail(PITT_E_NOMEM, "axis height staging");
    std::vector<float> soa((size_t)std::max<int64_t>(n, 1) * 3);
    for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) soa[(size_t)(k * n + i)] = xyz16[4 * i + k];
    if (n > 0) PITT_HIP_TRY(hipMemcpyAsync(d, soa.data(), (size_t)n * 12, hipMemcpyHostToDevice, ctx->stream));
    return pitt_axis_height(ctx, d, d + n, d + 2 * n, n, coef, mode, nullptr, nullptr, nullptr, height, idx1, idx2,
                            centroid);
}
