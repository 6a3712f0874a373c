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
//   optimize...        more than 4 inliers: Eigen's float Levenberg-Marquardt with numerical
//                      differences on fvec = sqrtf(|p - c|^2) - r (elm.hpp, bit for bit the oracle's
//                      pcl_lm_sphere).
//
// Device pipeline: k_sph_model (one thread per attempt: the 4 x 4 determinants), k_sph_count per
// chunk of attempts (one 2048-point tile x one hypothesis per block, ballot counts), the RANSAC replay
// on the host over the chunk's counts (scalar control), compaction of the inliers, and for the
// refinement k_elm<ElmSphere> (elm.hpp): the whole float Levenberg-Marquardt in one block per cloud.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "compact.hpp"
#include "ctx.hpp"
#include "device_common.hpp"
#include "elm.hpp"
#include "prim_ransac.hpp"

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
__device__ __forceinline__ void sph_count_block(const float* __restrict__ X, const float* __restrict__ Y,
                                                const float* __restrict__ Z, int64_t n, const float4* __restrict__ coef,
                                                const int32_t* __restrict__ flag, int a, float t,
                                                int32_t* __restrict__ count, int64_t base) {
    if (flag[a] != 1) return;
    const float4 c = coef[a];
    __shared__ int part[4];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        const bool in = i < n && sph_in(X[i], Y[i], Z[i], c, t);
        cnt += __popcll(__ballot(in));
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(count, part[0] + part[1] + part[2] + part[3]);
}
__global__ __launch_bounds__(256) void k_sph_count(const float* __restrict__ X, const float* __restrict__ Y,
                                                   const float* __restrict__ Z, int64_t n,
                                                   const float4* __restrict__ coef, const int32_t* __restrict__ flag,
                                                   int a0, float t, int32_t* __restrict__ counts) {
    sph_count_block(X, Y, Z, n, coef, flag, a0 + (int)blockIdx.y, t, counts + blockIdx.y, (int64_t)blockIdx.x * 2048);
}
// Several clouds' chunks in one launch: blockIdx.z = the job, blocks past its cloud or its attempts exit.
__global__ __launch_bounds__(256) void k_sph_count_multi(const CountJob<float4>* __restrict__ jobs, float t) {
    const CountJob<float4>& j = jobs[blockIdx.z];
    const int64_t base = (int64_t)blockIdx.x * 2048;
    if ((int)blockIdx.y >= j.nh || base >= j.cl.n) return;
    sph_count_block(j.cl.x, j.cl.y, j.cl.z, j.cl.n, j.coef, j.flag, j.a0 + (int)blockIdx.y, t, j.counts + blockIdx.y, base);
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

// prim_ransac.hpp traits of the sphere service
struct SphPrep {
    int32_t valid;
};
struct SphModel {
    using Coef = float4;
    using Prep = SphPrep;
    static constexpr int kSample = 4;
    static constexpr const char* kName = "k_sph";
    static constexpr double kModelBytes = 48.0, kCountBytes = 12.0;
    static constexpr bool kDevicePrep = false;
    int max_iterations;
    double probability;
    uint32_t seed;
    int optimize;
    double rmin, rmax;
    float t;
    static void to_out(const float4& c, float* o) {
        o[0] = c.x, o[1] = c.y, o[2] = c.z, o[3] = c.w;
    }
    void launch_model(hipStream_t s, const PrimCloud& c, const int32_t* tab, int A, float4* coef, int32_t* flag) const {
        hipLaunchKernelGGL(k_sph_model, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, s, c.x, c.y, c.z, tab, A, rmin,
                           rmax, coef, flag);
    }
    static constexpr int kCountSpan = 2048;
    void launch_count_multi(hipStream_t s, const CountJob<float4>* jobs, int nj, int bx, int nh) const {
        hipLaunchKernelGGL(k_sph_count_multi, dim3((unsigned)bx, (unsigned)nh, (unsigned)nj), dim3(256), 0, s, jobs, t);
    }
    void launch_count(hipStream_t s, const PrimCloud& c, const float4* coef, const int32_t* flag, int a0, int nh,
                      int32_t* cnt) const {
        hipLaunchKernelGGL(k_sph_count, dim3((unsigned)ctiles(c.n), (unsigned)nh), dim3(256), 0, s, c.x, c.y, c.z, c.n,
                           coef, flag, a0, t, cnt);
    }
    // selectWithinDistance: none for a model outside the radius limits
    void prep_host(const float4& c, SphPrep* p) const {
        p->valid = !((rmin != -DBL_MAX && (double)c.w < rmin) || (rmax != DBL_MAX && (double)c.w > rmax));
    }
    void launch_prep(hipStream_t, const float4&, SphPrep*) const {}
    static bool prep_valid(const SphPrep& p) { return p.valid != 0; }
    using SelPred = SphIn;
    using SelAct = WriteIdx;
    SphIn sel_pred(const PrimCloud& c, const float4& m, const SphPrep&) const { return SphIn{c.x, c.y, c.z, m, t}; }
    static WriteIdx sel_act(const PrimCloud& c) { return WriteIdx{c.inliers}; }
    void launch_select(hipStream_t s, const PrimCloud& c, const float4& m, const SphPrep& q, int32_t* tc, int32_t* to,
                       int g) const {
        SphIn pred = sel_pred(c, m, q);
        hipLaunchKernelGGL(k_pred_count<SphIn>, dim3(g), dim3(kBlock), 0, s, pred, c.n, tc);
        hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, tc, ctiles(c.n), to);
        hipLaunchKernelGGL((k_pred_apply<SphIn, WriteIdx>), dim3(g), dim3(kBlock), 0, s, pred, WriteIdx{c.inliers}, c.n,
                           to);
    }
    // more than 4 inliers (sac_model_sphere.hpp: "Not enough inliers" below): PCL's float
    // Levenberg-Marquardt on the sphere's OptimizationFunctor (elm.hpp), bit-exact with the oracle
    using Elm = ElmSphere;
    static int refine_kind(int64_t n_inliers) { return n_inliers > 4 ? 1 : 0; }
    void launch_normalize(hipStream_t, const float4&, float4*) const {}
};

SphModel sph_model(const pitt_sphere_params* p) {
    return SphModel{p->max_iterations, p->probability, p->seed, p->optimize, p->radius_min, p->radius_max,
                    float_threshold(p->threshold)};
}

// A batch of sphere services: one host synchronisation per phase.
int sphere_batch(pitt_ctx* ctx, const pitt_sphere_params* p, const PrimCloud* cl, int nc, PrimResult* res) {
    return prim_ransac_batch(ctx, sph_model(p), cl, nc, res);
}
// The same as a run of prim_ransac_lockstep (pitt_classify_clusters).
std::unique_ptr<PrimRunBase> sphere_run(pitt_ctx* ctx, const pitt_sphere_params* p, const PrimCloud* cl, int nc,
                                        PrimResult* res) {
    return std::make_unique<PrimRun<SphModel>>(ctx, sph_model(p), cl, nc, res);
}

}  // namespace pitt

extern "C" int pitt_sphere_segment(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                   const pitt_sphere_params* p, int32_t* inliers, int64_t* n_inliers, float coef_out[4],
                                   int32_t* hypotheses) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (!p || !n_inliers || !coef_out || n < 0 || (n > 0 && (!x || !y || !z || !inliers)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    *n_inliers = 0;
    if (hypotheses) *hypotheses = 0;
    for (int k = 0; k < 4; ++k) coef_out[k] = 0;
    const PrimCloud c{x, y, z, nullptr, nullptr, nullptr, n, inliers};
    PrimResult r;
    const int rc = sphere_batch(ctx, p, &c, 1, &r);
    if (rc != PITT_OK) return rc;
    if (hypotheses) *hypotheses = r.hypotheses;
    if (r.status != PITT_OK) return r.status;
    *n_inliers = r.n_inliers;
    for (int k = 0; k < 4; ++k) coef_out[k] = r.coef[k];
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
