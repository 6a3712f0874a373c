// cone.hip -- the cone service's seg.segment (cone_segmentation_srv.cpp:111-127):
// SampleConsensusModelCone with normals, RANSAC over 3-point samples, the opening-angle limits, the eps
// angle, the normal-weighted distance, optimize, the final selection.  The axis "height" post-processing
// that follows in the service is pitt_axis_height (primitives.hip, PITT_AXIS_CONE).
//
// PCL 1.7 semantics (restated in oracle/pitt_oracle.cpp: orc_cone_segment); Vector4f math as vec4.hpp:
//   computeModel...    ortho_ij = n_i x n_j, apex = (d1 o23 + d2 o31 + d3 o12) / (n1 . o23) with
//                      d_i = p_i . n_i; axis = normalize((np2 - np1) x (np3 - np1)), np_i = apex +
//                      (p_i - apex) / |p_i - apex|; angle = (acosf + acosf + acosf) / 3 of the unit offsets
//                      against the axis; outside [min_angle, max_angle] -> skip;
//   isModelValid       the eps angle of the direction against `axis` (getAngle3D), the angle limits;
//   countWithinDistance |w * d_normal + (1 - w) * d_euclid| < threshold in double: d_euclid = |axis
//                      distance - tan(angle) |apex - proj||, d_normal = min(a, pi - a) of the angle between
//                      the normal and sinf(angle) * unit(apex - proj) + cosf(angle) * unit(p - proj);
//   computeModel       the plane loop with w^3;
//   optimize           Eigen's float Levenberg-Marquardt with numerical differences on OptimizationFunctor's
//                      residual (float)(sqrPointToLineDistance(p, apex, dir) - (tanf(a) |apex - proj(p)|)^2)
//                      (elm.hpp, bit for bit the oracle's pcl_lm_cone), the direction normalised afterwards.
// A7: acosf / sinf / cosf / tanf are taken as correctly rounded -- (float) of the double function, here and
// in the oracle -- so host libm and the device's agree except for values within 2^-29 of a rounding boundary.
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

__device__ __forceinline__ float acosf_cr(float a) { return (float)acos((double)a); }
__device__ __forceinline__ float sinf_cr(float a) { return (float)sin((double)a); }
__device__ __forceinline__ float cosf_cr(float a) { return (float)cos((double)a); }

// getAngle3D under Eigen 3.2 (normalized() divides: a zero vector gives NaN) or >= 3.3 (keeps it zero)
__device__ __forceinline__ CV4 cnormalized_e(CV4 a, int eigen33) {
    if (eigen33 && !(cdot(a, a) > 0.0f)) return a;
    return cnormalized(a);
}
__device__ __forceinline__ double cangle3d(CV4 a, CV4 b, int eigen33) {
    double rad = cdot(cnormalized_e(a, eigen33), cnormalized_e(b, eigen33));
    if (rad < -1.0) rad = -1.0;
    else if (rad > 1.0) rad = 1.0;
    return acos(rad);
}

struct ConeCfg {
    double w, th, amin, amax, eps;
    float ax, ay, az;
    int eigen33;
};

__global__ void k_cone_model(const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
                             const float* __restrict__ NX, const float* __restrict__ NY, const float* __restrict__ NZ,
                             const int32_t* __restrict__ table, int A, double amin, double amax,
                             Coef7* __restrict__ coef, int32_t* __restrict__ flag) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A) return;
    CV4 p[3], nn[3];
    for (int q = 0; q < 3; ++q) {
        const int id = table[3 * t + q];
        p[q] = cv4(X[id], Y[id], Z[id]);
        nn[q] = cv4(NX[id], NY[id], NZ[id]);
    }
    const CV4 o12 = ccross3(nn[0], nn[1]), o23 = ccross3(nn[1], nn[2]), o31 = ccross3(nn[2], nn[0]);
    const float den = cdot(nn[0], o23);
    const float d1 = cdot(p[0], nn[0]), d2 = cdot(p[1], nn[1]), d3 = cdot(p[2], nn[2]);
    const CV4 num = cadd(cadd(cmul(d1, o23), cmul(d2, o31)), cmul(d3, o12));
    const CV4 apex = cv4(num.v[0] / den, num.v[1] / den, num.v[2] / den, num.v[3] / den);
    CV4 ap[3], np[3];
    for (int q = 0; q < 3; ++q) {
        ap[q] = csub(p[q], apex);
        np[q] = cadd(apex, cnormalized(ap[q]));
    }
    const CV4 axis = cnormalize(ccross3(csub(np[1], np[0]), csub(np[2], np[0])));
    float acc = 0.0f;
    for (int q = 0; q < 3; ++q) acc = acc + acosf_cr(cdot(cnormalize(ap[q]), axis));
    Coef7 out = {};
    for (int k = 0; k < 3; ++k) out.c[k] = apex.v[k], out.c[3 + k] = axis.v[k];
    out.c[6] = acc / 3.0f;
    // PCL also tests angle != -+DBL_MAX first: always true for a float, so dropped
    const int ok = !(out.c[6] < amin) && !(out.c[6] > amax);
    coef[t] = out;
    flag[t] = ok;
}

__device__ __forceinline__ bool cone_valid(const Coef7& m, const ConeCfg& c) {
    if (c.eps > 0.0) {
        double d = fabs(cangle3d(cv4(c.ax, c.ay, c.az), cv4(m.c[3], m.c[4], m.c[5]), c.eigen33));
        const double alt = M_PI - d;
        d = alt < d ? alt : d;  // std::min
        if (d > c.eps) return false;
    }
    return !(m.c[6] < c.amin) && !(m.c[6] > c.amax);  // the -+DBL_MAX guards: always true for a float
}

// per-model constants of countWithinDistance, hoisted out of the point loop
struct ConeModel {
    CV4 apex, ad;
    float apexdotdir, dirdotdir, sa, ca;
    double tana;
};
__device__ __forceinline__ ConeModel cone_model(const Coef7& m) {
    ConeModel q;
    q.apex = cv4(m.c[0], m.c[1], m.c[2]);
    q.ad = cv4(m.c[3], m.c[4], m.c[5]);
    q.apexdotdir = cdot(q.apex, q.ad);
    q.dirdotdir = 1.0f / cdot(q.ad, q.ad);
    q.sa = sinf_cr(m.c[6]);
    q.ca = cosf_cr(m.c[6]);
    q.tana = tan((double)m.c[6]);
    return q;
}

__device__ __forceinline__ bool cone_in(float x, float y, float z, float nx, float ny, float nz, const ConeModel& q,
                                        const ConeCfg& c) {
    const CV4 pt = cv4(x, y, z), nn = cv4(nx, ny, nz);
    const float k = (cdot(pt, q.ad) - q.apexdotdir) * q.dirdotdir;
    const CV4 proj = cadd(q.apex, cmul(k, q.ad));
    const CV4 dir = cnormalize(csub(pt, proj));
    CV4 h = csub(q.apex, proj);
    const double radius = q.tana * (double)sqrtf(cdot(h, h));
    h = cnormalize(h);
    const CV4 cn = cadd(cmul(q.sa, h), cmul(q.ca, dir));
    const double d_euclid = fabs(sqrt(csqr_pt_line(pt, q.apex, q.ad)) - radius);
    double d_normal = fabs(cangle3d(nn, cn, c.eigen33));
    const double alt = M_PI - d_normal;
    d_normal = alt < d_normal ? alt : d_normal;
    return fabs(c.w * d_normal + (1 - c.w) * d_euclid) < c.th;
}

__device__ __forceinline__ void cone_count_block(const float* __restrict__ X, const float* __restrict__ Y,
                                                 const float* __restrict__ Z, const float* __restrict__ NX,
                                                 const float* __restrict__ NY, const float* __restrict__ NZ, int64_t n,
                                                 const Coef7* __restrict__ coef, const int32_t* __restrict__ flag,
                                                 int a, const ConeCfg& cfg, int32_t* __restrict__ count,
                                                 int64_t base) {
    if (flag[a] != 1) return;
    const Coef7 m = coef[a];
    if (!cone_valid(m, cfg)) return;
    const ConeModel q = cone_model(m);
    __shared__ int part[4];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        const bool in = i < n && cone_in(X[i], Y[i], Z[i], NX[i], NY[i], NZ[i], q, cfg);
        cnt += __popcll(__ballot(in));
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(count, part[0] + part[1] + part[2] + part[3]);
}
__global__ __launch_bounds__(256) void k_cone_count(const float* __restrict__ X, const float* __restrict__ Y,
                                                    const float* __restrict__ Z, const float* __restrict__ NX,
                                                    const float* __restrict__ NY, const float* __restrict__ NZ,
                                                    int64_t n, const Coef7* __restrict__ coef,
                                                    const int32_t* __restrict__ flag, int a0, ConeCfg cfg,
                                                    int32_t* __restrict__ counts) {
    cone_count_block(X, Y, Z, NX, NY, NZ, n, coef, flag, a0 + (int)blockIdx.y, cfg, counts + blockIdx.y,
                     (int64_t)blockIdx.x * 1024);
}
// Several clouds' chunks in one launch: blockIdx.z = the job, blocks past its cloud or its attempts exit.
__global__ __launch_bounds__(256) void k_cone_count_multi(const CountJob<Coef7>* __restrict__ jobs, ConeCfg cfg) {
    const CountJob<Coef7>& j = jobs[blockIdx.z];
    const int64_t base = (int64_t)blockIdx.x * 1024;
    if ((int)blockIdx.y >= j.nh || base >= j.cl.n) return;
    cone_count_block(j.cl.x, j.cl.y, j.cl.z, j.cl.nx, j.cl.ny, j.cl.nz, j.cl.n, j.coef, j.flag, j.a0 + (int)blockIdx.y,
                     cfg, j.counts + blockIdx.y, base);
}

struct ConeIn {
    const float *x, *y, *z, *nx, *ny, *nz;
    ConeModel q;
    ConeCfg c;
    __device__ bool operator()(int64_t i) const { return cone_in(x[i], y[i], z[i], nx[i], ny[i], nz[i], q, c); }
};
struct ConeWriteIdx {
    int32_t* out;
    __device__ void operator()(int64_t i, int64_t pos) const { out[pos] = (int32_t)i; }
};

// selectWithinDistance's isModelValid and the predicate's model constants, from one device thread (the eps
// check and the constants need the device's acos / sin / cos / tan, as the counting kernel evaluates them)
struct ConePrep {
    ConeModel q;
    int32_t valid;
};
__global__ void k_cone_prepare(Coef7 m, ConeCfg cfg, ConePrep* out) {
    ConePrep r;
    r.q = cone_model(m);
    r.valid = cone_valid(m, cfg) ? 1 : 0;
    *out = r;
}

// The same for several clouds' models (device coefficients), cloud c where sel[c] >= 0.
__global__ void k_cone_prepare_multi(const Coef7* __restrict__ m, const int32_t* __restrict__ sel, int nc, ConeCfg cfg,
                                     ConePrep* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc || sel[c] < 0) return;
    const Coef7 mc = m[c];
    ConePrep r;
    r.q = cone_model(mc);
    r.valid = cone_valid(mc, cfg) ? 1 : 0;
    out[c] = r;
}

// prim_ransac.hpp traits of the cone service
struct ConeModelT {
    using Coef = Coef7;
    using Prep = ConePrep;
    static constexpr int kSample = 3;
    static constexpr const char* kName = "k_cone";
    static constexpr double kModelBytes = 72.0, kCountBytes = 24.0;
    static constexpr bool kDevicePrep = true;  // isModelValid and the model constants need device math
    int max_iterations;
    double probability;
    uint32_t seed;
    int optimize;
    ConeCfg cfg;
    static void to_out(const Coef7& c, float* o) {
        for (int k = 0; k < 7; ++k) o[k] = c.c[k];
    }
    void launch_model(hipStream_t s, const PrimCloud& c, const int32_t* tab, int A, Coef7* coef, int32_t* flag) const {
        hipLaunchKernelGGL(k_cone_model, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, s, c.x, c.y, c.z, c.nx, c.ny,
                           c.nz, tab, A, cfg.amin, cfg.amax, coef, flag);
    }
    static constexpr int kCountSpan = 1024;
    void launch_count_multi(hipStream_t s, const CountJob<Coef7>* jobs, int nj, int bx, int nh) const {
        hipLaunchKernelGGL(k_cone_count_multi, dim3((unsigned)bx, (unsigned)nh, (unsigned)nj), dim3(256), 0, s, jobs, cfg);
    }
    void launch_count(hipStream_t s, const PrimCloud& c, const Coef7* coef, const int32_t* flag, int a0, int nh,
                      int32_t* cnt) const {
        hipLaunchKernelGGL(k_cone_count, dim3((unsigned)((c.n + 1023) / 1024), (unsigned)nh), dim3(256), 0, s, c.x,
                           c.y, c.z, c.nx, c.ny, c.nz, c.n, coef, flag, a0, cfg, cnt);
    }
    void prep_host(const Coef7&, ConePrep*) const {}
    void launch_prep(hipStream_t s, const Coef7& m, ConePrep* out) const {
        hipLaunchKernelGGL(k_cone_prepare, dim3(1), dim3(1), 0, s, m, cfg, out);
    }
    void launch_prep_multi(hipStream_t s, const Coef7* m, const int32_t* sel, int nc, ConePrep* out) const {
        hipLaunchKernelGGL(k_cone_prepare_multi, dim3((unsigned)((nc + 63) / 64)), dim3(64), 0, s, m, sel, nc, cfg, out);
    }
    static bool prep_valid(const ConePrep& p) { return p.valid != 0; }
    using SelPred = ConeIn;
    using SelAct = ConeWriteIdx;
    ConeIn sel_pred(const PrimCloud& c, const Coef7&, const ConePrep& q) const {
        return ConeIn{c.x, c.y, c.z, c.nx, c.ny, c.nz, q.q, cfg};
    }
    static ConeWriteIdx sel_act(const PrimCloud& c) { return ConeWriteIdx{c.inliers}; }
    void launch_select(hipStream_t s, const PrimCloud& c, const Coef7& m, const ConePrep& q, int32_t* tc, int32_t* to,
                       int g) const {
        ConeIn pred = sel_pred(c, m, q);
        hipLaunchKernelGGL(k_pred_count<ConeIn>, dim3(g), dim3(kBlock), 0, s, pred, c.n, tc);
        hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, tc, ctiles(c.n), to);
        hipLaunchKernelGGL((k_pred_apply<ConeIn, ConeWriteIdx>), dim3(g), dim3(kBlock), 0, s, pred,
                           ConeWriteIdx{c.inliers}, c.n, to);
    }
    // any inliers: PCL's float Levenberg-Marquardt (fewer than 7: the model unchanged, its direction
    // normalised)
    using Elm = ElmCone;
    static int refine_kind(int64_t n_inliers) { return n_inliers >= 7 ? 1 : n_inliers > 0 ? 2 : 0; }
    void launch_normalize(hipStream_t s, const Coef7& bc, Coef7* out) const {
        hipLaunchKernelGGL(k_lm7_normalize_dir<>, dim3(1), dim3(1), 0, s, bc, out);
    }
};

static ConeModelT cone_model_t(const pitt_cone_params* p) {
    return ConeModelT{p->max_iterations, p->probability, p->seed, p->optimize,
                      ConeCfg{p->normal_distance_weight, p->threshold, p->min_angle, p->max_angle, p->eps_angle,
                              p->axis[0], p->axis[1], p->axis[2], p->eigen33}};
}
// A batch of cone services: one host synchronisation per phase.
int cone_batch(pitt_ctx* ctx, const pitt_cone_params* p, const PrimCloud* cl, int nc, PrimResult* res) {
    return prim_ransac_batch(ctx, cone_model_t(p), cl, nc, res);
}
// The same as a run of prim_ransac_lockstep (pitt_classify_clusters).
std::unique_ptr<PrimRunBase> cone_run(pitt_ctx* ctx, const pitt_cone_params* p, const PrimCloud* cl, int nc,
                                      PrimResult* res) {
    return std::make_unique<PrimRun<ConeModelT>>(ctx, cone_model_t(p), cl, nc, res);
}

}  // namespace pitt

extern "C" int pitt_cone_segment(pitt_ctx* ctx, const float* x, const float* y, const float* z, const float* nx,
                                 const float* ny, const float* nz, int64_t n, const pitt_cone_params* p,
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
    const int rc = cone_batch(ctx, p, &c, 1, &r);
    if (rc != PITT_OK) return rc;
    if (hypotheses) *hypotheses = r.hypotheses;
    if (r.status != PITT_OK) return r.status;
    *n_inliers = r.n_inliers;
    for (int k = 0; k < 7; ++k) coef_out[k] = r.coef[k];
    return PITT_OK;
}

// Host-memory form (the service handlers' clouds): points as PointXYZ (16-byte stride), normals as
// (nx, ny, nz) triples; staged into the context's device buffers, the inliers copied back.
extern "C" int pitt_cone_segment_host(pitt_ctx* ctx, const float* xyz16, const float* normals3, int64_t n,
                                      const pitt_cone_params* params, int32_t* inliers, int64_t* n_inliers,
                                      float coef[7], int32_t* hypotheses) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (n < 0 || (n > 0 && (!xyz16 || !normals3 || !inliers)) || !n_inliers || !coef)
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    const size_t nb = (size_t)std::max<int64_t>(n, 1) * 4;
    float* d = (float*)ctx->buf("cone_hsoa", nb * 6);
    int32_t* di = (int32_t*)ctx->buf("cone_hi", nb);
    if (!d || !di) return ctx->fail(PITT_E_NOMEM, "cone staging");
    std::vector<float> soa((size_t)std::max<int64_t>(n, 1) * 6);
    for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            soa[(size_t)(k * n + i)] = xyz16[4 * i + k];
            soa[(size_t)((3 + k) * n + i)] = normals3[3 * i + k];
        }
    hipStream_t s = ctx->stream;
    if (n > 0) PITT_HIP_TRY(hipMemcpyAsync(d, soa.data(), (size_t)n * 24, hipMemcpyHostToDevice, s));
    const int rc = pitt_cone_segment(ctx, d, d + n, d + 2 * n, d + 3 * n, d + 4 * n, d + 5 * n, n, params, di,
                                     n_inliers, coef, hypotheses);
    if (rc < 0) return rc;
    if (*n_inliers > 0) {
        PITT_HIP_TRY(hipMemcpyAsync(inliers, di, (size_t)*n_inliers * 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
    }
    return rc;
}
