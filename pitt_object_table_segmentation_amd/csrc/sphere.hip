// sphere.hip -- the sphere service's seg.segment (sphere_segmentation_srv.cpp:57-73; SURVEY.md s8f
// row 4).  SACSegmentationFromNormals with SACMODEL_SPHERE falls through to the plain
// SampleConsensusModelSphere (the normals are not used): RANSAC over 4-point samples with the radius
// limits, then optimizeModelCoefficients and the final selectWithinDistance.
//
// PCL 1.7 semantics (restated in oracle/pitt_oracle.cpp: orc_sphere_segment):
//   getSamples         drawIndexSample with 4 draws per attempt (A2); isSampleGood accepts every sample;
//   computeModel...    Cramer's rule with Eigen 3.2's 4 x 4 determinant (Costabel's expansion, float),
//                      m11 == 0 -> the attempt is skipped (skipped_count);
//   countWithinDistance 0 for a model outside the radius limits, else
//                      |sqrtf((x - a)^2 + (y - b)^2 + (z - c)^2) - r| < threshold (A4 float threshold);
//   computeModel       the plane path's loop with w^4 (strict > first-best, k, max_skip = 10 x max_it);
//   optimize...        more than 4 inliers: a least-squares refinement of ||p - c|| - r.  PCL runs
//                      Eigen's float Levenberg-Marquardt with numerical differences (stopping at its
//                      sqrt(eps) tolerances); this runs a double Levenberg-Marquardt on device sums to
//                      the optimum -- the coefficients match PCL's within that tolerance, not bit for bit.
//
// Device pipeline: k_sph_model (one thread per attempt: the 4 x 4 determinants), k_sph_count per
// chunk of attempts (one 2048-point tile x one hypothesis per block, ballot counts), the RANSAC replay
// on the host over the chunk's counts (scalar control), compaction of the inliers, and for the
// refinement k_lm<SphLmModel> (lm.hpp): the whole Levenberg-Marquardt iteration in one resident grid
// (deterministic sums).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "compact.hpp"
#include "ctx.hpp"
#include "device_common.hpp"
#include "lm.hpp"

#pragma clang fp contract(off)

namespace pitt {

__device__ __forceinline__ float sph_det4_helper(const float* m, int j, int k, int a, int b) {
    return (m[j * 4 + 0] * m[k * 4 + 1] - m[k * 4 + 0] * m[j * 4 + 1]) *
           (m[a * 4 + 2] * m[b * 4 + 3] - m[b * 4 + 2] * m[a * 4 + 3]);
}

// Eigen 3.2 determinant_impl<4>, terms left to right
__device__ __forceinline__ float sph_det4(const float* m) {
    return sph_det4_helper(m, 0, 1, 2, 3) - sph_det4_helper(m, 0, 2, 1, 3) + sph_det4_helper(m, 0, 3, 1, 2) +
           sph_det4_helper(m, 1, 2, 0, 3) - sph_det4_helper(m, 1, 3, 0, 2) + sph_det4_helper(m, 2, 3, 0, 1);
}

// flag: 0 = m11 == 0 (skipped), 1 = a model inside the radius limits, 2 = outside (counts 0)
__global__ void k_sph_model(const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
                            const int32_t* __restrict__ table, int A, double rmin, double rmax,
                            float4* __restrict__ coef, int32_t* __restrict__ flag) {
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= A) return;
    float px[4], py[4], pz[4], t[16];
    for (int i = 0; i < 4; ++i) {
        const int s = table[4 * a + i];
        px[i] = X[s];
        py[i] = Y[s];
        pz[i] = Z[s];
    }
    for (int i = 0; i < 4; ++i) t[i * 4 + 0] = px[i], t[i * 4 + 1] = py[i], t[i * 4 + 2] = pz[i], t[i * 4 + 3] = 1.0f;
    const float m11 = sph_det4(t);
    if (m11 == 0) {
        flag[a] = 0;
        coef[a] = make_float4(0, 0, 0, 0);
        return;
    }
    for (int i = 0; i < 4; ++i) t[i * 4 + 0] = px[i] * px[i] + py[i] * py[i] + pz[i] * pz[i];
    const float m12 = sph_det4(t);
    for (int i = 0; i < 4; ++i) t[i * 4 + 1] = t[i * 4 + 0], t[i * 4 + 0] = px[i];
    const float m13 = sph_det4(t);
    for (int i = 0; i < 4; ++i) t[i * 4 + 2] = t[i * 4 + 1], t[i * 4 + 1] = py[i];
    const float m14 = sph_det4(t);
    for (int i = 0; i < 4; ++i)
        t[i * 4 + 0] = t[i * 4 + 2], t[i * 4 + 1] = px[i], t[i * 4 + 2] = py[i], t[i * 4 + 3] = pz[i];
    const float m15 = sph_det4(t);
    float4 c;
    c.x = 0.5f * m12 / m11;
    c.y = 0.5f * m13 / m11;
    c.z = 0.5f * m14 / m11;
    c.w = sqrtf(c.x * c.x + c.y * c.y + c.z * c.z - m15 / m11);
    coef[a] = c;
    const bool bad = (rmin != -DBL_MAX && (double)c.w < rmin) || (rmax != DBL_MAX && (double)c.w > rmax);
    flag[a] = bad ? 2 : 1;
}

__device__ __forceinline__ bool sph_in(float x, float y, float z, float4 c, float t) {
    const float dx = x - c.x, dy = y - c.y, dz = z - c.z;
    return fabsf(sqrtf(dx * dx + dy * dy + dz * dz) - c.w) < t;
}

// counts[a - a0] for attempts [a0, a0 + gridDim.y): blockIdx.x = 2048-point tile
__global__ __launch_bounds__(256) void k_sph_count(const float* __restrict__ X, const float* __restrict__ Y,
                                                   const float* __restrict__ Z, int64_t n,
                                                   const float4* __restrict__ coef, const int32_t* __restrict__ flag,
                                                   int a0, float t, int32_t* __restrict__ counts) {
    const int a = a0 + blockIdx.y;
    if (flag[a] != 1) return;
    const float4 c = coef[a];
    __shared__ int part[4];
    int cnt = 0;
    const int64_t base = (int64_t)blockIdx.x * 2048;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        const bool in = i < n && sph_in(X[i], Y[i], Z[i], c, t);
        cnt += __popcll(__ballot(in));
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(counts + blockIdx.y, part[0] + part[1] + part[2] + part[3]);
}

struct SphIn {
    const float *x, *y, *z;
    float4 c;
    float t;
    __device__ bool operator()(int64_t i) const { return sph_in(x[i], y[i], z[i], c, t); }
};
struct WriteIdx {
    int32_t* out;
    __device__ void operator()(int64_t i, int64_t pos) const { out[pos] = (int32_t)i; }
};

// Levenberg-Marquardt over the inliers' residuals ||p - c|| - r in double (lm.hpp's resident grid, 100
// iterations, no diagonal floor), the coefficients written back as floats.
struct SphLmModel {
    static constexpr int N = 4;
    static constexpr int kMaxIt = 100;
    static constexpr double kDiagEps = 0.0;
    static constexpr int64_t kSmall = 2048;
    using Out = float4;
    __device__ double aux(const double*) const { return 0.0; }
    float4 start;
    __device__ void init(double* v) const {
        v[0] = start.x, v[1] = start.y, v[2] = start.z, v[3] = start.w;
    }
    __device__ void residual(const double* v, float px, float py, float pz, double* J, double* f) const {
        const double dx = (double)px - v[0], dy = (double)py - v[1], dz = (double)pz - v[2];
        const double d = sqrt(dx * dx + dy * dy + dz * dz);
        *f = d - v[3];
        J[0] = d > 0 ? -dx / d : 0.0;
        J[1] = d > 0 ? -dy / d : 0.0;
        J[2] = d > 0 ? -dz / d : 0.0;
        J[3] = -1.0;
    }
    __device__ void finish(const double* xv, float4* out) const {
        *out = make_float4((float)xv[0], (float)xv[1], (float)xv[2], (float)xv[3]);
    }
};

}  // namespace pitt

extern "C" int pitt_sphere_segment(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                   const pitt_sphere_params* p, int32_t* inliers, int64_t* n_inliers, float coef_out[4],
                                   int32_t* hypotheses) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (!p || !n_inliers || !coef_out || n < 0 || (n > 0 && (!x || !y || !z || !inliers)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "more than 2^31 points");
    if (p->max_iterations < 0 || !(p->probability > 0 && p->probability < 1))
        return ctx->fail(PITT_E_INVALID, "max_iterations / probability");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    *n_inliers = 0;
    if (hypotheses) *hypotheses = 0;
    for (int k = 0; k < 4; ++k) coef_out[k] = 0;
    if (n < 4) return PITT_NO_MODEL;  // getSamples: "Can not select 4 unique points"
    hipStream_t s = ctx->stream;
    const float t = float_threshold(p->threshold);
    // attempts: every iteration draws once; skipped draws (m11 == 0) are at most max_skip
    const int64_t max_skip = (int64_t)p->max_iterations * 10;
    const int64_t A = (int64_t)p->max_iterations + 1 + max_skip;
    if (A > (1 << 24)) return ctx->fail(PITT_E_INVALID, "max_iterations too large");
    const std::vector<int32_t>& tab = sampler_table(ctx, n, p->seed, A, 4);
    int32_t* dtab = (int32_t*)ctx->buf("sph_table", (size_t)A * 16);
    float4* dcoef = (float4*)ctx->buf("sph_coef", (size_t)A * 16);
    int32_t* dflag = (int32_t*)ctx->buf("sph_flag", (size_t)A * 4);
    int32_t* dcnt = (int32_t*)ctx->buf("sph_cnt", (size_t)A * 4);
    const int64_t nt = ctiles(n);
    int32_t* tc = (int32_t*)ctx->buf("sph_tc", (size_t)(nt + 1) * 4);
    int32_t* to = (int32_t*)ctx->buf("sph_to", (size_t)(nt + 1) * 4);
    double* part = (double*)ctx->buf("sph_part", 64);
    if (!dtab || !dcoef || !dflag || !dcnt || !tc || !to || !part) return ctx->fail(PITT_E_NOMEM, "sphere scratch");
    PITT_HIP_TRY(hipMemcpyAsync(dtab, tab.data(), (size_t)A * 16, hipMemcpyHostToDevice, s));
    int rec = ctx->prof_begin("k_sph_model", (double)A * 48.0);
    hipLaunchKernelGGL(k_sph_model, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, s, x, y, z, dtab, (int)A,
                       p->radius_min, p->radius_max, dcoef, dflag);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    std::vector<int32_t> hflag((size_t)A), hcnt;
    PITT_HIP_TRY(hipMemcpyAsync(hflag.data(), dflag, (size_t)A * 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    // RandomSampleConsensus::computeModel over chunks of attempts (32, 64, 128, then 256 at a time)
    int iterations = 0, n_best = -INT32_MAX;
    double k = 1.0;
    const double log_probability = std::log(1.0 - p->probability);
    const double one_over_indices = 1.0 / (double)n;
    int64_t skipped = 0;
    int best = -1;
    int64_t a = 0;
    int chunk = 32;
    bool done = false;
    while (!done && a < A) {
        const int64_t a1 = std::min<int64_t>(A, a + chunk);
        const int nh = (int)(a1 - a);
        PITT_HIP_TRY(hipMemsetAsync(dcnt + a, 0, (size_t)nh * 4, s));
        rec = ctx->prof_begin("k_sph_count", (double)nh * (double)n * 12.0);
        hipLaunchKernelGGL(k_sph_count, dim3((unsigned)nt, (unsigned)nh), dim3(256), 0, s, x, y, z, n, dcoef, dflag,
                           (int)a, t, dcnt + a);
        ctx->prof_end(rec);
        PITT_HIP_TRY(hipGetLastError());
        hcnt.resize((size_t)nh);
        PITT_HIP_TRY(hipMemcpyAsync(hcnt.data(), dcnt + a, (size_t)nh * 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        for (int64_t i = a; i < a1; ++i) {
            if (!(iterations < k && skipped < max_skip)) {
                done = true;
                break;
            }
            if (hflag[(size_t)i] == 0) {
                ++skipped;
                continue;
            }
            const int n_in = hcnt[(size_t)(i - a)];  // 0 for a model outside the radius limits
            if (n_in > n_best) {
                n_best = n_in;
                best = (int)i;
                const double w = (double)n_best * one_over_indices;
                double p_no = 1.0 - std::pow(w, 4.0);
                p_no = std::max(std::numeric_limits<double>::epsilon(), p_no);
                p_no = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no);
                k = log_probability / std::log(p_no);
            }
            ++iterations;
            if (iterations > p->max_iterations) {
                done = true;
                break;
            }
        }
        a = a1;
        chunk = std::min(chunk * 2, 256);
    }
    if (hypotheses) *hypotheses = iterations;
    if (best < 0) return PITT_NO_MODEL;
    float4 bc;
    PITT_HIP_TRY(hipMemcpy(&bc, dcoef + best, 16, hipMemcpyDeviceToHost));
    int32_t* hto = (int32_t*)ctx->pinned("sph_to_h", 16);
    if (!hto) return ctx->fail(PITT_E_NOMEM, "sphere pinned");
    const int g = grid_for_tiles(nt);
    // selectWithinDistance (none for a model outside the radius limits)
    auto select = [&](float4 c) -> int {
        const bool valid = !((p->radius_min != -DBL_MAX && (double)c.w < p->radius_min) ||
                             (p->radius_max != DBL_MAX && (double)c.w > p->radius_max));
        if (!valid) {
            *n_inliers = 0;
            return PITT_OK;
        }
        SphIn pred{x, y, z, c, t};
        hipLaunchKernelGGL(k_pred_count<SphIn>, dim3(g), dim3(kBlock), 0, s, pred, n, tc);
        hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, tc, nt, to);
        hipLaunchKernelGGL((k_pred_apply<SphIn, WriteIdx>), dim3(g), dim3(kBlock), 0, s, pred, WriteIdx{inliers}, n, to);
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipMemcpyAsync(hto, to + nt, 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        *n_inliers = hto[0];
        return PITT_OK;
    };
    int rc = select(bc);
    if (rc != PITT_OK) return rc;
    float out[4] = {bc.x, bc.y, bc.z, bc.w};
    if (p->optimize && *n_inliers > 4) {
        // Levenberg-Marquardt in double, the whole iteration in one 1024-thread block (the oracle's
        // sphere_refine; fixed reduction order, so the same bits on every run)
        float4* dref = (float4*)part;
        rec = ctx->prof_begin("k_sph_lm", (double)*n_inliers * 12.0);
        const int lrc = launch_lm(ctx, s, SphLmModel{bc}, x, y, z, inliers, *n_inliers, dref);
        if (lrc != PITT_OK) return lrc;
        ctx->prof_end(rec);
        PITT_HIP_TRY(hipGetLastError());
        float4* hr = (float4*)ctx->pinned("sph_ref_h", 16);
        if (!hr) return ctx->fail(PITT_E_NOMEM, "sphere pinned");
        PITT_HIP_TRY(hipMemcpyAsync(hr, dref, 16, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        out[0] = hr->x;
        out[1] = hr->y;
        out[2] = hr->z;
        out[3] = hr->w;
        rc = select(make_float4(out[0], out[1], out[2], out[3]));
        if (rc != PITT_OK) return rc;
    }
    for (int r = 0; r < 4; ++r) coef_out[r] = out[r];
    return PITT_OK;
}

// Host-memory form (the service handlers' PointXYZ clouds, 16-byte stride): the cloud is staged into
// the context's device SoA buffers, the inliers copied back.
extern "C" int pitt_sphere_segment_host(pitt_ctx* ctx, const float* xyz16, int64_t n,
                                        const pitt_sphere_params* params, int32_t* inliers, int64_t* n_inliers,
                                        float coef[4], int32_t* hypotheses) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (n < 0 || (n > 0 && (!xyz16 || !inliers)) || !n_inliers || !coef) return ctx->fail(PITT_E_INVALID, "null argument");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    const size_t nb = (size_t)std::max<int64_t>(n, 1) * 4;
    float* dx = (float*)ctx->buf("sph_hx", nb);
    float* dy = (float*)ctx->buf("sph_hy", nb);
    float* dz = (float*)ctx->buf("sph_hz", nb);
    int32_t* di = (int32_t*)ctx->buf("sph_hi", nb);
    if (!dx || !dy || !dz || !di) return ctx->fail(PITT_E_NOMEM, "sphere staging");
    std::vector<float> soa((size_t)n * 3);
    for (int64_t i = 0; i < n; ++i) {
        soa[(size_t)i] = xyz16[4 * i];
        soa[(size_t)(n + i)] = xyz16[4 * i + 1];
        soa[(size_t)(2 * n + i)] = xyz16[4 * i + 2];
    }
    hipStream_t s = ctx->stream;
    if (n > 0) {
        PITT_HIP_TRY(hipMemcpyAsync(dx, soa.data(), (size_t)n * 4, hipMemcpyHostToDevice, s));
        PITT_HIP_TRY(hipMemcpyAsync(dy, soa.data() + n, (size_t)n * 4, hipMemcpyHostToDevice, s));
        PITT_HIP_TRY(hipMemcpyAsync(dz, soa.data() + 2 * n, (size_t)n * 4, hipMemcpyHostToDevice, s));
    }
    const int rc = pitt_sphere_segment(ctx, dx, dy, dz, n, params, di, n_inliers, coef, hypotheses);
    if (rc < 0) return rc;
    if (*n_inliers > 0) {
        PITT_HIP_TRY(hipMemcpyAsync(inliers, di, (size_t)*n_inliers * 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
    }
    return rc;
}
