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
//   optimize           the double Levenberg-Marquardt of lm.hpp on f = |v|^2 - (1 + tan^2 a) (u.v)^2 / |u|^2
//                      (v = apex - p: the functor's residual by Lagrange's identity); PCL runs Eigen's float
//                      LM: equal within its tolerance, not bit for bit.
// A7: acosf / sinf / cosf are taken as correctly rounded -- (float) of the double function, here and in
// the oracle -- so host libm and the device's agree except for values within 2^-29 of a rounding boundary.
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

__global__ __launch_bounds__(256) void k_cone_count(const float* __restrict__ X, const float* __restrict__ Y,
                                                    const float* __restrict__ Z, const float* __restrict__ NX,
                                                    const float* __restrict__ NY, const float* __restrict__ NZ,
                                                    int64_t n, const Coef7* __restrict__ coef,
                                                    const int32_t* __restrict__ flag, int a0, ConeCfg cfg,
                                                    int32_t* __restrict__ counts) {
    const int a = a0 + blockIdx.y;
    if (flag[a] != 1) return;
    const Coef7 m = coef[a];
    if (!cone_valid(m, cfg)) return;
    const ConeModel q = cone_model(m);
    __shared__ int part[4];
    int cnt = 0;
    const int64_t base = (int64_t)blockIdx.x * 1024;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        const bool in = i < n && cone_in(X[i], Y[i], Z[i], NX[i], NY[i], NZ[i], q, cfg);
        cnt += __popcll(__ballot(in));
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(counts + blockIdx.y, part[0] + part[1] + part[2] + part[3]);
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

struct ConeResidual {
    static constexpr int64_t kSmall = 2048;  // one block measured slower than the grid at 4k inliers
    __device__ static double aux(const double* q) { return tan(q[6]); }  // q[7] below
    __device__ void operator()(const double* q, float px, float py, float pz, double J[7], double* f) const {
        const double vx = q[0] - px, vy = q[1] - py, vz = q[2] - pz;
        const double ux = q[3], uy = q[4], uz = q[5];
        const double s = ux * ux + uy * uy + uz * uz, g = ux * vx + uy * vy + uz * vz;
        const double t = q[7], K = 1.0 + t * t;
        *f = (vx * vx + vy * vy + vz * vz) - K * g * g / s;
        const double a = 2.0 * K * g / s;
        J[0] = 2.0 * vx - a * ux;
        J[1] = 2.0 * vy - a * uy;
        J[2] = 2.0 * vz - a * uz;
        J[3] = -a * (vx - g * ux / s);
        J[4] = -a * (vy - g * uy / s);
        J[5] = -a * (vz - g * uz / s);
        J[6] = -(g * g / s) * 2.0 * t * K;
    }
};

}  // namespace pitt

extern "C" int pitt_cone_segment(pitt_ctx* ctx, const float* x, const float* y, const float* z, const float* nx,
                                 const float* ny, const float* nz, int64_t n, const pitt_cone_params* p,
                                 int32_t* inliers, int64_t* n_inliers, float coef_out[7], int32_t* hypotheses) {
    using namespace pitt;
    if (!ctx) return PITT_E_INVALID;
    if (!p || !n_inliers || !coef_out || n < 0 || (n > 0 && (!x || !y || !z || !nx || !ny || !nz || !inliers)))
        return ctx->fail(PITT_E_INVALID, "null argument");
    if (n > 0x7fffffff) return ctx->fail(PITT_E_INVALID, "more than 2^31 points");
    if (p->max_iterations < 0 || !(p->probability > 0 && p->probability < 1))
        return ctx->fail(PITT_E_INVALID, "max_iterations / probability");
    if (hipSetDevice(ctx->device) != hipSuccess) return ctx->fail(PITT_E_HIP, "hipSetDevice");
    *n_inliers = 0;
    if (hypotheses) *hypotheses = 0;
    for (int k = 0; k < 7; ++k) coef_out[k] = 0;
    if (n < 3) return PITT_NO_MODEL;  // getSamples: "Can not select 3 unique points"
    hipStream_t s = ctx->stream;
    const ConeCfg cfg{p->normal_distance_weight, p->threshold, p->min_angle, p->max_angle, p->eps_angle,
                      p->axis[0], p->axis[1], p->axis[2], p->eigen33};
    const int64_t max_skip = (int64_t)p->max_iterations * 10;
    const int64_t A = (int64_t)p->max_iterations + 1 + max_skip;
    if (A > (1 << 24)) return ctx->fail(PITT_E_INVALID, "max_iterations too large");
    const std::vector<int32_t>& tab = sampler_table(ctx, n, p->seed, A, 3);
    int32_t* dtab = (int32_t*)ctx->buf("cone_table", (size_t)A * 12);
    Coef7* dcoef = (Coef7*)ctx->buf("cone_coef", (size_t)A * sizeof(Coef7));
    int32_t* dflag = (int32_t*)ctx->buf("cone_flag", (size_t)A * 4);
    int32_t* dcnt = (int32_t*)ctx->buf("cone_cnt", (size_t)A * 4);
    const int64_t nt = ctiles(n);
    int32_t* tc = (int32_t*)ctx->buf("cone_tc", (size_t)(nt + 1) * 4);
    int32_t* to = (int32_t*)ctx->buf("cone_to", (size_t)(nt + 1) * 4);
    Coef7* dref = (Coef7*)ctx->buf("cone_ref", sizeof(Coef7));
    ConePrep* dprep = (ConePrep*)ctx->buf("cone_prep", sizeof(ConePrep));
    if (!dtab || !dcoef || !dflag || !dcnt || !tc || !to || !dref || !dprep)
        return ctx->fail(PITT_E_NOMEM, "cone scratch");
    PITT_HIP_TRY(hipMemcpyAsync(dtab, tab.data(), (size_t)A * 12, hipMemcpyHostToDevice, s));
    int rec = ctx->prof_begin("k_cone_model", (double)A * 72.0);
    hipLaunchKernelGGL(k_cone_model, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, s, x, y, z, nx, ny, nz, dtab,
                       (int)A, p->min_angle, p->max_angle, dcoef, dflag);
    ctx->prof_end(rec);
    PITT_HIP_TRY(hipGetLastError());
    std::vector<int32_t> hflag((size_t)A), hcnt;
    PITT_HIP_TRY(hipMemcpyAsync(hflag.data(), dflag, (size_t)A * 4, hipMemcpyDeviceToHost, s));
    PITT_HIP_TRY(hipStreamSynchronize(s));
    // RandomSampleConsensus::computeModel replayed over chunks of device counts
    int iterations = 0, n_best = -INT32_MAX;
    double k = 1.0;
    const double log_probability = std::log(1.0 - p->probability);
    const double one_over_indices = 1.0 / (double)n;
    int64_t skipped = 0;
    int best = -1;
    int64_t a = 0;
    int chunk = 32;
    bool done = false;
    const int64_t ntc = (n + 1023) / 1024;
    while (!done && a < A) {
        const int64_t a1 = std::min<int64_t>(A, a + chunk);
        const int nh = (int)(a1 - a);
        PITT_HIP_TRY(hipMemsetAsync(dcnt + a, 0, (size_t)nh * 4, s));
        rec = ctx->prof_begin("k_cone_count", (double)nh * (double)n * 24.0);
        hipLaunchKernelGGL(k_cone_count, dim3((unsigned)ntc, (unsigned)nh), dim3(256), 0, s, x, y, z, nx, ny, nz, n,
                           dcoef, dflag, (int)a, cfg, dcnt + a);
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
            const int n_in = hcnt[(size_t)(i - a)];
            if (n_in > n_best) {
                n_best = n_in;
                best = (int)i;
                const double w = (double)n_best * one_over_indices;
                double p_no = 1.0 - std::pow(w, 3.0);
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
    Coef7 bc;
    PITT_HIP_TRY(hipMemcpy(&bc, dcoef + best, sizeof bc, hipMemcpyDeviceToHost));
    int32_t* hto = (int32_t*)ctx->pinned("cone_to_h", 16);
    Coef7* href = (Coef7*)ctx->pinned("cone_ref_h", sizeof(Coef7));
    ConePrep* hprep = (ConePrep*)ctx->pinned("cone_prep_h", sizeof(ConePrep));
    if (!hto || !href || !hprep) return ctx->fail(PITT_E_NOMEM, "cone pinned");
    const int g = grid_for_tiles(nt);
    auto select = [&](const Coef7& m) -> int {
        *n_inliers = 0;
        hipLaunchKernelGGL(k_cone_prepare, dim3(1), dim3(1), 0, s, m, cfg, dprep);
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipMemcpyAsync(hprep, dprep, sizeof(ConePrep), hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        if (!hprep->valid) return PITT_OK;
        ConeIn pred{x, y, z, nx, ny, nz, hprep->q, cfg};
        hipLaunchKernelGGL(k_pred_count<ConeIn>, dim3(g), dim3(kBlock), 0, s, pred, n, tc);
        hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, s, tc, nt, to);
        hipLaunchKernelGGL((k_pred_apply<ConeIn, ConeWriteIdx>), dim3(g), dim3(kBlock), 0, s, pred,
                           ConeWriteIdx{inliers}, n, to);
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipMemcpyAsync(hto, to + nt, 4, hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        *n_inliers = hto[0];
        return PITT_OK;
    };
    int rc = select(bc);
    if (rc != PITT_OK) return rc;
    Coef7 outc = bc;
    if (p->optimize && *n_inliers > 0) {
        if (*n_inliers >= 7) {
            rec = ctx->prof_begin("k_cone_lm", (double)*n_inliers * 12.0);
            const int lrc = launch_lm7(ctx, s, ConeResidual{}, x, y, z, inliers, *n_inliers, bc, dref);
            if (lrc != PITT_OK) return lrc;
            ctx->prof_end(rec);
        } else {
            hipLaunchKernelGGL(k_lm7_normalize_dir<>, dim3(1), dim3(1), 0, s, bc, dref);
        }
        PITT_HIP_TRY(hipGetLastError());
        PITT_HIP_TRY(hipMemcpyAsync(href, dref, sizeof(Coef7), hipMemcpyDeviceToHost, s));
        PITT_HIP_TRY(hipStreamSynchronize(s));
        outc = *href;
        rc = select(outc);
        if (rc != PITT_OK) return rc;
    }
    for (int r = 0; r < 7; ++r) coef_out[r] = outc.c[r];
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
