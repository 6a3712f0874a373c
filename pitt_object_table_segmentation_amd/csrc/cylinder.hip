// cylinder.hip -- the cylinder service's seg.segment (cylinder_segmentation_srv.cpp:110-126; SURVEY.md
// s8f row 4): SampleConsensusModelCylinder with normals, RANSAC over 2-point samples, the radius limits,
// the normal-weighted distance, optimize, the final selection.  The axis "height" post-processing that
// follows in the service is pitt_axis_height (primitives.hip).
//
// PCL 1.7 semantics (restated in oracle/pitt_oracle.cpp: orc_cylinder_segment); Eigen::Vector4f math is
// element-wise float, dot / squaredNorm reduced in SSE2 order (A3), normalize() times 1 / norm (A9),
// normalized() divided by it:
//   computeModel...    identical points (|dx|, |dy|, |dz| <= FLT_EPSILON) -> skip; the closest points of
//                      the two normal lines (a, b, c, d, e; den < 1e-8 -> the parallel case), line_pt =
//                      p1 + n1 + sc n1, line_dir = normalize(p2 + tc n2 - line_pt), r = sqrt of
//                      sqrPointToLineDistance(p1) (double sqrt of the float quotient), outside the radius
//                      limits -> skip;
//   countWithinDistance |w * d_normal + (1 - w) * d_euclid| < threshold in double, d_euclid = |point-to-axis
//                      distance - r|, d_normal = min(angle, pi - angle) between the normal and the radial
//                      direction (getAngle3D: acos of the clamped dot of the normalized vectors);
//   computeModel       the plane loop with w^2;
//   optimize           Eigen's float Levenberg-Marquardt with numerical differences on OptimizationFunctor's
//                      residual (float)(sqrPointToLineDistance - r^2) over the inliers (elm.hpp, bit for bit
//                      the oracle's pcl_lm_cylinder), the direction normalised as a Vector3f afterwards.
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
#include "vec4.hpp"

#pragma clang fp contract(off)

namespace pitt {

using CylCoef = Coef7;

__global__ void k_cyl_model(const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
                            const float* __restrict__ NX, const float* __restrict__ NY, const float* __restrict__ NZ,
                            const int32_t* __restrict__ table, int A, double rmin, double rmax,
                            CylCoef* __restrict__ coef, int32_t* __restrict__ flag) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A) return;
    const int a = table[2 * t], b = table[2 * t + 1];
    const float eps = FLT_EPSILON;
    CylCoef out = {};
    int ok = 1;
    if (fabsf(X[a] - X[b]) <= eps && fabsf(Y[a] - Y[b]) <= eps && fabsf(Z[a] - Z[b]) <= eps) {
        ok = 0;
    } else {
        const CV4 p1 = cv4(X[a], Y[a], Z[a]), p2 = cv4(X[b], Y[b], Z[b]);
        const CV4 n1 = cv4(NX[a], NY[a], NZ[a]), n2 = cv4(NX[b], NY[b], NZ[b]);
        const CV4 w = csub(cadd(n1, p1), p2);
        const float A_ = cdot(n1, n1), B = cdot(n1, n2), C = cdot(n2, n2), D = cdot(n1, w), E = cdot(n2, w);
        const float den = A_ * C - B * B;
        float sc, tc;
        if (den < 1e-8) {
            sc = 0.0f;
            tc = (B > C ? D / B : E / C);
        } else {
            sc = (B * E - C * D) / den;
            tc = (A_ * E - B * D) / den;
        }
        const CV4 lp = cadd(cadd(p1, n1), cmul(sc, n1));
        const CV4 ld = cnormalize(csub(cadd(p2, cmul(tc, n2)), lp));
        for (int k = 0; k < 3; ++k) out.c[k] = lp.v[k], out.c[3 + k] = ld.v[k];
        out.c[6] = (float)sqrt(csqr_pt_line(p1, lp, ld));
        if (out.c[6] > rmax || out.c[6] < rmin) ok = 0;
    }
    coef[t] = out;
    flag[t] = ok;
}

// getAngle3D's normalized() under Eigen 3.2 (a zero vector divides: NaN, never an inlier) or
// Eigen >= 3.3 (a zero vector stays zero: the angle is pi/2), as the cone's
__device__ __forceinline__ CV4 cyl_normalized_e(CV4 a, int eigen33) {
    if (eigen33 && !(cdot(a, a) > 0.0f)) return a;
    return cnormalized(a);
}

__device__ __forceinline__ bool cyl_in(float x, float y, float z, float nx, float ny, float nz, const CylCoef& m,
                                       double w, double th, int eigen33) {
    const CV4 lp = cv4(m.c[0], m.c[1], m.c[2]), ld = cv4(m.c[3], m.c[4], m.c[5]);
    const float ptdotdir = cdot(lp, ld), dirdotdir = 1.0f / cdot(ld, ld);
    const CV4 pt = cv4(x, y, z), nn = cv4(nx, ny, nz);
    const double d_euclid = fabs(sqrt(csqr_pt_line(pt, lp, ld)) - (double)m.c[6]);
    const float k = (cdot(pt, ld) - ptdotdir) * dirdotdir;
    const CV4 dir = cnormalize(csub(pt, cadd(lp, cmul(k, ld))));
    double rad = cdot(cyl_normalized_e(nn, eigen33), cyl_normalized_e(dir, eigen33));
    if (rad < -1.0) rad = -1.0;
    else if (rad > 1.0) rad = 1.0;
    double d_normal = fabs(acos(rad));
    const double alt = M_PI - d_normal;
    d_normal = alt < d_normal ? alt : d_normal;  // std::min
    return fabs(w * d_normal + (1 - w) * d_euclid) < th;
}

__device__ __forceinline__ bool cyl_valid(const CylCoef& m, double rmin, double rmax) {
    return !((rmin != -DBL_MAX && m.c[6] < rmin) || (rmax != DBL_MAX && m.c[6] > rmax));
}

__device__ __forceinline__ void cyl_count_block(const float* __restrict__ X, const float* __restrict__ Y,
                                                const float* __restrict__ Z, const float* __restrict__ NX,
                                                const float* __restrict__ NY, const float* __restrict__ NZ, int64_t n,
                                                const CylCoef* __restrict__ coef, const int32_t* __restrict__ flag,
                                                int a, double w, double th, int eigen33, double rmin, double rmax,
                                                int32_t* __restrict__ count, int64_t base) {
    if (flag[a] != 1) return;
    const CylCoef m = coef[a];
    if (!cyl_valid(m, rmin, rmax)) return;
    __shared__ int part[4];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        const bool in = i < n && cyl_in(X[i], Y[i], Z[i], NX[i], NY[i], NZ[i], m, w, th, eigen33);
        cnt += __popcll(__ballot(in));
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(count, part[0] + part[1] + part[2] + part[3]);
}
__global__ __launch_bounds__(256) void k_cyl_count(const float* __restrict__ X, const float* __restrict__ Y,
                                                   const float* __restrict__ Z, const float* __restrict__ NX,
                                                   const float* __restrict__ NY, const float* __restrict__ NZ,
                                                   int64_t n, const CylCoef* __restrict__ coef,
                                                   const int32_t* __restrict__ flag, int a0, double w, double th,
                                                   int eigen33, double rmin, double rmax,
                                                   int32_t* __restrict__ counts) {
    cyl_count_block(X, Y, Z, NX, NY, NZ, n, coef, flag, a0 + (int)blockIdx.y, w, th, eigen33, rmin, rmax,
                    counts + blockIdx.y, (int64_t)blockIdx.x * 1024);
}
// Several clouds' chunks in one launch: blockIdx.z = the job, blocks past its cloud or its attempts exit.
__global__ __launch_bounds__(256) void k_cyl_count_multi(const CountJob<CylCoef>* __restrict__ jobs, double w,
                                                         double th, int eigen33, double rmin, double rmax) {
    const CountJob<CylCoef>& j = jobs[blockIdx.z];
    const int64_t base = (int64_t)blockIdx.x * 1024;
    if ((int)blockIdx.y >= j.nh || base >= j.cl.n) return;
    cyl_count_block(j.cl.x, j.cl.y, j.cl.z, j.cl.nx, j.cl.ny, j.cl.nz, j.cl.n, j.coef, j.flag, j.a0 + (int)blockIdx.y,
                    w, th, eigen33, rmin, rmax, j.counts + blockIdx.y, base);
}

struct CylIn {
    const float *x, *y, *z, *nx, *ny, *nz;
    CylCoef m;
    double w, th;
    int eigen33;
    __device__ bool operator()(int64_t i) const {
        return cyl_in(x[i], y[i], z[i], nx[i], ny[i], nz[i], m, w, th, eigen33);
    }
};
struct CylWriteIdx {
    int32_t* out;
    __device__ void operator()(int64_t i, int64_t pos) const { out[pos] = (int32_t)i; }
};

// prim_ransac.hpp traits of the cylinder service
struct CylPrep {
    int32_t valid;
};
struct CylModel {
    using Coef = CylCoef;
    using Prep = CylPrep;
    static constexpr int kSample = 2;
    static constexpr const char* kName = "k_cyl";
    static constexpr double kModelBytes = 48.0, kCountBytes = 24.0;
    static constexpr bool kDevicePrep = false;
    int max_iterations;
    double probability;
    uint32_t seed;
    int optimize;
    double rmin, rmax, w, th;
    int eigen33;
    static void to_out(const CylCoef& c, float* o) {
        for (int k = 0; k < 7; ++k) o[k] = c.c[k];
    }
    void launch_model(hipStream_t s, const PrimCloud& c, const int32_t* tab, int A, CylCoef* coef, int32_t* flag) const {
        hipLaunchKernelGGL(k_cyl_model, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, s, c.x, c.y, c.z, c.nx, c.ny,
                           c.nz, tab, A, rmin, rmax, coef, flag);
    }
    static constexpr int kCountSpan = 1024;
    void launch_count_multi(hipStream_t s, const CountJob<CylCoef>* jobs, int nj, int bx, int nh) const {
        hipLaunchKernelGGL(k_cyl_count_multi, dim3((unsigned)bx, (unsigned)nh, (unsigned)nj), dim3(256), 0, s, jobs, w, th,
                           eigen33, rmin, rmax);
    }
    void launch_count(hipStream_t s, const PrimCloud& c, const CylCoef* coef, const int32_t* flag, int a0, int nh,
                      int32_t* cnt) const {
        hipLaunchKernelGGL(k_cyl_count, dim3((unsigned)((c.n + 1023) / 1024), (unsigned)nh), dim3(256), 0, s, c.x, c.y,
                           c.z, c.nx, c.ny, c.nz, c.n, coef, flag, a0, w, th, eigen33, rmin, rmax, cnt);
    }
    // selectWithinDistance: none for a model outside the radius limits
    void prep_host(const CylCoef& m, CylPrep* p) const {
        p->valid = !((rmin != -DBL_MAX && m.c[6] < rmin) || (rmax != DBL_MAX && m.c[6] > rmax));
    }
    void launch_prep(hipStream_t, const CylCoef&, CylPrep*) const {}
    static bool prep_valid(const CylPrep& p) { return p.valid != 0; }
    using SelPred = CylIn;
    using SelAct = CylWriteIdx;
    CylIn sel_pred(const PrimCloud& c, const CylCoef& m, const CylPrep&) const {
        return CylIn{c.x, c.y, c.z, c.nx, c.ny, c.nz, m, w, th, eigen33};
    }
    static CylWriteIdx sel_act(const PrimCloud& c) { return CylWriteIdx{c.inliers}; }
    void launch_select(hipStream_t s, const PrimCloud& c, const CylCoef& m, const CylPrep& q, int32_t* tc, int32_t* to,
                       int g) const {
        CylIn pred = sel_pred(c, m, q);
        hipLaunchKernelGGL(k_pred_count<CylIn>, dim3(g), dim3(kBlock), 0, s, pred, c.n, tc);
        hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, tc, ctiles(c.n), to);
        hipLaunchKernelGGL((k_pred_apply<CylIn, CylWriteIdx>), dim3(g), dim3(kBlock), 0, s, pred,
                           CylWriteIdx{c.inliers}, c.n, to);
    }
    // any inliers: PCL's float Levenberg-Marquardt (7 or more: Eigen's LM refuses m < n, the model then
    // stays and only the direction is normalised)
    using Elm = ElmCylinder;
    static int refine_kind(int64_t n_inliers) { return n_inliers >= 7 ? 1 : n_inliers > 0 ? 2 : 0; }
    void launch_normalize(hipStream_t s, const Coef7& bc, Coef7* out) const {
        hipLaunchKernelGGL(k_lm7_normalize_dir<>, dim3(1), dim3(1), 0, s, bc, out);
    }
};

static CylModel cyl_model(const pitt_cylinder_params* p) {
    return CylModel{p->max_iterations, p->probability, p->seed, p->optimize, p->radius_min, p->radius_max,
                    p->normal_distance_weight, p->threshold, (int)p->eigen33};
}
// A batch of cylinder services: one host synchronisation per phase.
int cylinder_batch(pitt_ctx* ctx, const pitt_cylinder_params* p, const PrimCloud* cl, int nc, PrimResult* res) {
    return prim_ransac_batch(ctx, cyl_model(p), cl, nc, res);
}
// The same as a run of prim_ransac_lockstep (pitt_classify_clusters).
std::unique_ptr<PrimRunBase> cylinder_run(pitt_ctx* ctx, const pitt_cylinder_params* p, const PrimCloud* cl, int nc,
                                          PrimResult* res) {
    return std::make_unique<PrimRun<CylModel>>(ctx, cyl_model(p), cl, nc, res);
}

}  // namespace pitt

extern "C" int pitt_cylinder_segment(pitt_ctx* ctx, const float* x, const float* y, const float* z, const float* nx,
                                     const float* ny, const float* nz, int64_t n, const pitt_cylinder_params* p,
                                     int32_t* inliers, int64_t* n_inliers, float coef_out[7], int32_t* hypotheses) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (!p || !n_inliers || !coef_out || n < 0 || (n > 0 && (!x || !y || !z || !nx || !ny || !nz || !inliers)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    *n_inliers = 0;
    if (hypotheses) *hypotheses = 0;
    for (int k = 0; k < 7; ++k) coef_out[k] = 0;
    const PrimCloud c{x, y, z, nx, ny, nz, n, inliers};
    PrimResult r;
    const int rc = cylinder_batch(ctx, p, &c, 1, &r);
    if (rc != PITT_OK) return rc;
    if (hypotheses) *hypotheses = r.hypotheses;
    if (r.status != PITT_OK) return r.status;
    *n_inliers = r.n_inliers;
    for (int k = 0; k < 7; ++k) coef_out[k] = r.coef[k];
    return PITT_OK;
}

// Host-memory form (the service handlers' clouds): points as PointXYZ (16-byte stride), normals as
// (nx, ny, nz) triples; staged into the context's device buffers, the inliers copied back.
extern "C" int pitt_cylinder_segment_host(pitt_ctx* ctx, const float* xyz16, const float* normals3, int64_t n,
                                          const pitt_cylinder_params* params, int32_t* inliers, int64_t* n_inliers,
                                          float coef[7], int32_t* hypotheses) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (n < 0 || (n > 0 && (!xyz16 || !normals3 || !inliers)) || !n_inliers || !coef)
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    const size_t nb = (size_t)std::max<int64_t>(n, 1) * 4;
    float* d = (float*)ctx->buf("cyl_hsoa", nb * 6);
    int32_t* di = (int32_t*)ctx->buf("cyl_hi", nb);
    if (!d || !di) return ctx->fail(PITT_E_NOMEM, "cylinder staging");
    std::vector<float> soa((size_t)std::max<int64_t>(n, 1) * 6);
    for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            soa[(size_t)(k * n + i)] = xyz16[4 * i + k];
            soa[(size_t)((3 + k) * n + i)] = normals3[3 * i + k];
        }
    hipStream_t s = ctx->stream;
    if (n > 0) PITT_HIP_TRY(hipMemcpyAsync(d, soa.data(), (size_t)n * 24, hipMemcpyHostToDevice, s));
    const int rc = pitt_cylinder_segment(ctx, d, d + n, d + 2 * n, d + 3 * n, d + 4 * n, d + 5 * n, n, params, di,
                                         n_inliers, coef, hypotheses);
    if (rc < 0) return rc;
    if (*n_inliers > 0) {
        PITT_HIP_TRY(hipMemcpyAsync(inliers, di, (size_t)*n_inliers * 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
    }
    return rc;
}
