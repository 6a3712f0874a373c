// elm.hpp -- PCL 1.7's optimizeModelCoefficients for the sphere, cylinder and cone models on the device:
//
//     Eigen::NumericalDiff<OptimizationFunctor> num_diff (functor);
//     Eigen::LevenbergMarquardt<Eigen::NumericalDiff<OptimizationFunctor>, float> lm (num_diff);
//     lm.minimize (optimized_coefficients);
//
// (sac_model_sphere.hpp / sac_model_cylinder.hpp / sac_model_cone.hpp, reached from the services'
// setOptimizeCoefficients (true): sphere_segmentation_srv.cpp:61,73, cylinder_segmentation_srv.cpp:114,126,
// cone_segmentation_srv.cpp:115,127).  Eigen 3.2's unsupported NonLinearOptimization module is MINPACK's
// lmdif: a forward-difference Jacobian, ColPivHouseholderQR, lmpar / qrsolv for the Levenberg-Marquardt
// parameter and the step-bound / ratio logic, all in float with Eigen's defaults (factor 100, maxfev 400,
// ftol = xtol = sqrt(FLT_EPSILON), gtol 0).  The oracle restates it from Eigen's published source
// (oracle/eigen_lm.hpp); this is the same algorithm in the same float operation order, so the refined
// coefficients -- and therefore the final inlier sets -- are the oracle's bit for bit.
//
// Float order (A3, SSE2 build without FMA): dense sums are Eigen's LinearVectorizedTraversal redux (two
// 4-lane packet accumulators, predux (a0 + a2) + (a1 + a3), a scalar tail); the Householder GEMV is the
// row-major kernel (scalar head to the rhs's 16-byte boundary, one packet accumulator, scalar tail);
// blueNorm is sequential over three ranges; stableNorm sums 4096-element blocks scaled by the running max.
//
// Layout.  One 256-thread block per refinement (a batch: every cluster's refinement of one model kind in
// one launch).  Per job a float workspace of (N + 2) m in HBM: the Jacobian (column-major, N x m; the QR
// runs in place on it), then f(x) and the trial residuals (swapped on an accepted step).  The m-sized
// elementwise work (residuals, the Jacobian, the Householder updates) runs on all 256 threads.  Every
// m-sized sum is a serial float chain in Eigen's order, so those run on wave 0's lanes: the redux's 8
// packet chains, the GEMV's 4 per column (all columns at once), blueNorm's one per column.  The
// n-sized control (lmpar, qrsolv, the step logic) runs on thread 0 from LDS.  The chains bound the
// kernel: about 5.5 m dependent adds per outer iteration.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <string>
#include <vector>

#include "ctx.hpp"
#include "vec4.hpp"

#pragma clang fp contract(off)

namespace pitt {

constexpr int kElmThreads = 256;
constexpr int kElmMaxN = 7;

struct Coef7 {  // the cylinder / cone models: point (apex), direction, radius (opening angle)
    float c[7];
    float pad;
};

// fewer residuals than parameters (m < 7): Eigen's LM returns ImproperInputParameters and leaves the model;
// optimizeModelCoefficients still normalises the direction (Vector3f: a0 + (a1 + a2), times 1 / norm)
template <int = 0>  // a template, so the header can be included by several translation units
__global__ void k_lm7_normalize_dir(Coef7 m, Coef7* out) {
    const float u0 = m.c[3], u1 = m.c[4], u2 = m.c[5];
    const float r = 1.0f / sqrtf(u0 * u0 + (u1 * u1 + u2 * u2));
    m.c[3] = u0 * r;
    m.c[4] = u1 * r;
    m.c[5] = u2 * r;
    *out = m;
}

// Eigen::LevenbergMarquardtSpace::Status
enum ElmStatus {
    kElmImproper = 0,
    kElmRelReduction = 1,
    kElmRelError = 2,
    kElmCosinus = 4,
    kElmMaxFev = 5,
    kElmFtol = 6,
    kElmXtol = 7,
    kElmGtol = 8,
    kElmRunning = -1
};

struct ElmJob {
    const float *x, *y, *z;  // the cloud (device SoA)
    const int32_t* inl;      // the inlier indices (device), m of them
    int64_t m;
    float* work;             // (N + 2) * m floats
    float start[8];          // the winning model
    float* out;              // N floats: the refined model (direction normalised for the 7-parameter models)
    int32_t* info;           // optional: [status, nfev]
};

// ---- scalar helpers (one thread) -------------------------------------------------------------------
__device__ __forceinline__ float elm_max(float a, float b) { return (a < b) ? b : a; }  // std::max
__device__ __forceinline__ float elm_min(float a, float b) { return (b < a) ? b : a; }  // std::min

// Eigen 3.2 redux of a float expression (the oracle's redux_sum), sequentially in one thread.
template <class G>
__device__ float elm_redux1(int size, G g) {
    if (size <= 0) return 0.0f;
    const int asz2 = (size / 8) * 8, asz = (size / 4) * 4;
    float res;
    if (asz) {
        float p0[4], p1[4];
        for (int l = 0; l < 4; ++l) p0[l] = g(l);
        if (asz > 4) {
            for (int l = 0; l < 4; ++l) p1[l] = g(4 + l);
            for (int i = 8; i < asz2; i += 8)
                for (int l = 0; l < 4; ++l) {
                    p0[l] = p0[l] + g(i + l);
                    p1[l] = p1[l] + g(i + 4 + l);
                }
            for (int l = 0; l < 4; ++l) p0[l] = p0[l] + p1[l];
            if (asz > asz2)
                for (int l = 0; l < 4; ++l) p0[l] = p0[l] + g(asz2 + l);
        }
        res = (p0[0] + p0[2]) + (p0[1] + p0[3]);
        for (int i = asz; i < size; ++i) res = res + g(i);
    } else {
        res = g(0);
        for (int i = 1; i < size; ++i) res = res + g(i);
    }
    return res;
}

// MatrixBase::blueNorm's machine constants for float.
struct ElmBlue {
    float b1, b2, s1m, s2m, rbig, overfl, relerr;
};
__device__ __forceinline__ ElmBlue elm_blue_consts() {
    ElmBlue c;
    c.b1 = ldexpf(1.0f, -63);   // -((1 - min_exponent) / 2), min_exponent = -125
    c.b2 = ldexpf(1.0f, 52);    // (max_exponent + 1 - digits) / 2 = (128 + 1 - 24) / 2
    c.s1m = ldexpf(1.0f, 63);   // (2 - min_exponent) / 2
    c.s2m = ldexpf(1.0f, -76);  // -((max_exponent + digits) / 2)
    c.rbig = FLT_MAX;
    c.overfl = c.rbig * c.s2m;
    c.relerr = sqrtf(ldexpf(1.0f, -23));  // sqrt(pow(2, 1 - digits))
    return c;
}
// blueNorm's finish from the three range sums.
__device__ __forceinline__ float elm_blue_finish(const ElmBlue& c, float asml, float amed, float abig) {
    if (abig > 0.0f) {
        abig = sqrtf(abig);
        if (abig > c.overfl) return c.rbig;
        if (amed > 0.0f) {
            abig = abig / c.s2m;
            amed = sqrtf(amed);
        } else {
            return abig / c.s2m;
        }
    } else if (asml > 0.0f) {
        if (amed > 0.0f) {
            abig = sqrtf(amed);
            amed = sqrtf(asml) / c.s1m;
        } else {
            return sqrtf(asml) / c.s1m;
        }
    } else {
        return sqrtf(amed);
    }
    asml = elm_min(abig, amed);
    abig = elm_max(abig, amed);
    if (asml <= abig * c.relerr) return abig;
    const float q = asml / abig;
    return abig * sqrtf(1.0f + q * q);
}
// One element of blueNorm's sequential loop (the three range sums; + 0 leaves a sum unchanged, as every
// sum is +0 or positive).
__device__ __forceinline__ void elm_blue_step(const ElmBlue& c, float ab2, float v, float& asml, float& amed,
                                              float& abig) {
    const float ax = fabsf(v);
    const bool big = ax > ab2;
    const bool sml = !big && ax < c.b1;
    const float tb = ax * c.s2m, ts = ax * c.s1m;
    abig = abig + (big ? tb * tb : 0.0f);
    asml = asml + (sml ? ts * ts : 0.0f);
    amed = amed + ((big || sml) ? 0.0f : ax * ax);
}
__device__ float elm_blue1(const float* v, int n) {  // blueNorm of a short vector, one thread
    const ElmBlue c = elm_blue_consts();
    const float ab2 = c.b2 / (float)n;
    float asml = 0.0f, amed = 0.0f, abig = 0.0f;
    for (int i = 0; i < n; ++i) elm_blue_step(c, ab2, v[i], asml, amed, abig);
    return elm_blue_finish(c, asml, amed, abig);
}
// stableNorm of a short vector (n < 4096: one block), one thread.
__device__ float elm_stable1(const float* v, int n) {
    float mx = fabsf(v[0]);
    for (int i = 1; i < n; ++i) mx = elm_max(mx, fabsf(v[i]));
    float scale = 0.0f, inv = 1.0f, ssq = 0.0f;
    if (mx > scale) {
        const float r = scale / mx;
        ssq = ssq * (r * r);
        scale = mx;
        inv = 1.0f / scale;
    }
    ssq = ssq + elm_redux1(n, [&](int i) {
              const float t = v[i] * inv;
              return t * t;
          });
    return scale * sqrtf(ssq);
}

// ---- wave-level chains (every lane of the calling wave calls them) ----------------------------------
// a + g(i) + g(i + S) + ... over i < end, in that order (one dependent add per element).  Eight elements
// per step, the next step's eight loads issued before this step's adds, so the adds cover the LDS latency.
// 32-bit indices (m < 2^31): 64-bit compares and address arithmetic would double the loop's issue cost.
template <int S, class G>
__device__ __forceinline__ float elm_chain(int i, int end, float a, G g) {
    constexpr int U = 8;
    if (i + (U - 1) * S < end) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = g(i + u * S);
        for (i += U * S; i + (U - 1) * S < end; i += U * S) {
            float w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = g(i + u * S);
#pragma unroll
            for (int u = 0; u < U; ++u) a = a + v[u];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = w[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) a = a + v[u];
    }
    for (; i < end; i += S) a = a + g(i);
    return a;
}

// Eigen's redux (elm_redux_wave below) of up to eight sums at once: lanes 8 q .. 8 q + 7 run sum q's
// eight packet-lane chains over its own sz elements g(i) (sz = 0: no sum), and lane 8 q returns it.
template <class G>
__device__ __forceinline__ float elm_redux_wave8(int64_t size, G g, int lane) {
    const int sz = (int)size;
    const int l = lane & 7, base = lane & ~7;
    const int asz2 = (sz / 8) * 8, asz = (sz / 4) * 4;
    float acc = 0.0f;
    if (asz > 4) acc = elm_chain<8>(8 + l, asz2, g(l), g);
    else if (asz == 4 && l < 4) acc = g(l);
    const float p1 = __shfl(acc, base + ((l + 4) & 7), 64);
    if (asz > 4 && l < 4) {
        acc = acc + p1;
        if (asz > asz2) acc = acc + g(asz2 + l);
    }
    const float a0 = __shfl(acc, base, 64), a1 = __shfl(acc, base + 1, 64), a2 = __shfl(acc, base + 2, 64),
                a3 = __shfl(acc, base + 3, 64);
    float res = 0.0f;
    if (l == 0) {
        if (asz) {
            res = (a0 + a2) + (a1 + a3);
            for (int i = asz; i < sz; ++i) res = res + g(i);
        } else if (sz > 0) {
            res = elm_chain<1>(1, sz, g(0), g);
        }
    }
    return res;
}

// ---- the single-sum form (wave 0 of the block; every lane of the wave calls it) ---------------------
// Eigen's redux over g(0 .. size-1): lanes 0-7 run the two packets' 8 lane chains; the sum on lane 0.
template <class G>
__device__ __forceinline__ float elm_redux_wave(int64_t size64, G g, int lane) {
    const int size = (int)size64;
    const int asz2 = (size / 8) * 8, asz = (size / 4) * 4;
    float acc = 0.0f;
    if (asz > 4) {
        if (lane < 8) acc = elm_chain<8>(8 + lane, asz2, g(lane), g);
        const float p1 = __shfl(acc, (lane + 4) & 63, 64);
        if (lane < 4) {
            acc = acc + p1;
            if (asz > asz2) acc = acc + g(asz2 + lane);
        }
    } else if (asz == 4) {
        if (lane < 4) acc = g(lane);
    }
    const float a0 = __shfl(acc, 0, 64), a1 = __shfl(acc, 1, 64), a2 = __shfl(acc, 2, 64), a3 = __shfl(acc, 3, 64);
    float res = 0.0f;
    if (lane == 0) {
        if (asz) {
            res = (a0 + a2) + (a1 + a3);
            for (int i = asz; i < size; ++i) res = res + g(i);
        } else if (size > 0) {
            res = elm_chain<1>(1, size, g(0), g);
        }
    }
    return res;
}

// ---- the refinement -----------------------------------------------------------------------------------
template <class F>
struct ElmShared {
    static constexpr int N = F::N;
    using Pre = typename F::Pre;
    Pre pre[N + 1];                 // the Jacobian's N perturbed models, then the trial model
    float x[N], diag[N], wa1[N], wa2[N], wa3[N], qtf[N], colnorm[N], hstep[N], hc[N], sq[N];
    float R[N][N];                  // R(r, c) = R[c][r]: the QR's top n x n block (column-major)
    float lmS[N][N];                // lmpar's working copy of R for qrsolv (thread 0; in LDS rather than scratch)
#ifdef PITT_ELM_PROF
    unsigned long long prof_qrsolv;
    int prof_lmpar_iter;
#endif
    int perm[N], transp[N];
    float maxpivot;
    int nonzero_pivots;
    float bc[8];                    // broadcast scalars
    int ibc[8];
    // LevenbergMarquardt's state (thread 0)
    float fnorm, par, delta, xnorm, temp, gnorm;
    int nfev, iter, status, cur;    // cur: which of the two residual buffers holds f(x)
};

// ColPivHouseholderQR<MatrixXf>::compute on the Jacobian in place (A: column-major, m x N), the oracle's
// ColPivQR::compute, fused with householderQ().adjoint() * w (m floats, the oracle's ColPivQR::apply_qt):
// reflector k is applied to w right after it is formed -- later steps never touch column k, and apply_qt
// applies the reflectors to w in the same order k = 0, 1, ... -- so w's dot product (Eigen's redux, wave
// 1) runs beside the block GEMV's (the row-major kernel's order, wave 0).  The pivot column's recomputed
// norm and the reflector's tail norm are taken in one pass (the swap only moves the column).  Every thread
// of the block calls it.
#ifdef PITT_ELM_PROF
#define PITT_QR_T(k)                             \
    do {                                         \
        const unsigned long long t_ = clock64(); \
        qp[k] += t_ - qt;                        \
        qt = t_;                                 \
    } while (0)
#else
#define PITT_QR_T(k) \
    do {             \
    } while (0)
#endif
template <class F, class B>
__device__ __forceinline__ void elm_qr(float* A, int64_t m, float* w, ElmShared<F>& s, B&& wave1_first,
                                       unsigned long long* qp = nullptr) {
    constexpr int N = F::N;
#ifdef PITT_ELM_PROF
    unsigned long long qt = clock64();
#else
    (void)qp;
#endif
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr float kEps = FLT_EPSILON;
    // column squared norms: lanes 8 j .. 8 j + 7 for column j, all columns at once
    if (wave == 0) {
        const int q = lane >> 3;
        const float* col = A + (int64_t)(q < N ? q : 0) * m;
        const float r = elm_redux_wave8(q < N ? m : 0, [&](int i) { const float v = col[i]; return v * v; }, lane);
        if ((lane & 7) == 0 && q < N) s.sq[q] = r;
    }
    if (wave == 1) wave1_first(lane);  // the caller's work beside the column norms (the blue norms)
    __syncthreads();
    if (tid == 0) {
        float mx = s.sq[0];
        for (int k = 1; k < N; ++k) mx = elm_max(mx, s.sq[k]);
        s.bc[0] = mx * (kEps * kEps) / (float)m;  // threshold_helper
        s.nonzero_pivots = N;
        s.maxpivot = 0.0f;
        int big = 0;  // the first pivot: the first maximum of the squared norms
        for (int j = 1; j < N; ++j)
            if (s.sq[j] > s.sq[big]) big = j;
        s.ibc[0] = big;
    }
    __syncthreads();
    PITT_QR_T(0);
    const float threshold_helper = s.bc[0];
    for (int k = 0; k < N; ++k) {
        const int big = s.ibc[0];
        const int64_t len = m - k;
        if (wave == 0) {
            // lanes 0-7: the pivot column's norm from row k, recomputed; lanes 8-15: makeHouseholderInPlace's
            // tail norm, rows k + 1.. of the same column (column k once swapped)
            const int q = lane >> 3;
            const float* col = A + (int64_t)big * m + k + (q == 1 ? 1 : 0);
            const int64_t sz = q == 0 ? len : (q == 1 ? len - 1 : 0);
            const float r = elm_redux_wave8(sz, [&](int i) { const float v = col[i]; return v * v; }, lane);
            const float tail_sq = __shfl(r, 8, 64);
            if (lane == 0) {
                const float bigsq = r;
                s.sq[big] = bigsq;
                if (s.nonzero_pivots == N && bigsq < threshold_helper * (float)(m - k)) s.nonzero_pivots = k;
                s.transp[k] = big;
                if (k != big) {
                    const float t = s.sq[k];
                    s.sq[k] = s.sq[big];
                    s.sq[big] = t;
                }
                const float c0 = A[(int64_t)big * m + k];
                float tau, beta, den = 1.0f;
                int zero = 0;
                if (tail_sq == 0.0f) {
                    tau = 0.0f;
                    beta = c0;
                    zero = 1;
                } else {
                    beta = sqrtf(c0 * c0 + tail_sq);
                    if (c0 >= 0.0f) beta = -beta;
                    den = c0 - beta;
                    tau = (beta - c0) / beta;
                }
                s.hc[k] = tau;
                s.bc[1] = tau;
                s.bc[2] = beta;
                s.bc[3] = den;
                s.ibc[1] = zero;
                if (fabsf(beta) > s.maxpivot) s.maxpivot = fabsf(beta);
            }
        }
        __syncthreads();
        PITT_QR_T(1);
        const float tau = s.bc[1], beta = s.bc[2], den = s.bc[3];
        const bool zero = s.ibc[1] != 0;
        {  // columns k and big swapped (all rows); column k's essential part scaled, beta on the diagonal
            float* a = A + (int64_t)k * m;
            float* b = A + (int64_t)big * m;
            for (int64_t r = tid; r < m; r += kElmThreads) {
                float nk = b[r];
                if (k != big) b[r] = a[r];
                if (r > k) nk = zero ? 0.0f : nk / den;
                else if (r == k) nk = beta;
                a[r] = nk;
            }
        }
        __syncthreads();
        PITT_QR_T(2);
        // applyHouseholderOnTheLeft to the block A(k.., k+1..): tmp_c = essential^T * bottom (row-major GEMV
        // order: head to the essential vector's 16-byte boundary, one packet, tail), lanes 4 c + l of wave 0;
        // and to w: tmp_w = essential . w(k+1..) + w(k) (Eigen's redux), wave 1
        const int cols = N - k - 1;
        const int64_t rows = m - k;
        if (rows == 1) {
            if (tid == 0) {
                for (int c = 0; c < cols; ++c) A[(int64_t)(k + 1 + c) * m + k] = A[(int64_t)(k + 1 + c) * m + k] * (1.0f - tau);
                w[k] = w[k] * (1.0f - tau);
            }
        } else {
            const float* ess = A + (int64_t)k * m + k + 1;
            const int64_t depth = rows - 1;
            if (wave == 0 && cols > 0) {
                const int64_t ess_off = (int64_t)k * m + k + 1;
                int64_t as = (4 - (ess_off % 4)) % 4;
                if (as > depth) as = depth;
                const int64_t asize = as + ((depth - as) & ~(int64_t)3);
                const int c = lane >> 2, l = lane & 3;
                float pk = 0.0f;
                if (c < cols) {
                    const float* col = A + (int64_t)(k + 1 + c) * m + k + 1;
                    pk = elm_chain<4>((int)(as + l), (int)asize, 0.0f, [&](int j) { return col[j] * ess[j]; });
                }
                const int b = lane & ~3;
                const float q0 = __shfl(pk, b, 64), q1 = __shfl(pk, b + 1, 64), q2 = __shfl(pk, b + 2, 64),
                            q3 = __shfl(pk, b + 3, 64);
                if (c < cols && l == 0) {
                    const float* col = A + (int64_t)(k + 1 + c) * m + k + 1;
                    float tmp = 0.0f;
                    for (int64_t jj = 0; jj < as; ++jj) tmp = tmp + col[jj] * ess[jj];
                    if (asize > as) tmp = tmp + ((q0 + q2) + (q1 + q3));
                    for (int64_t jj = asize; jj < depth; ++jj) tmp = tmp + col[jj] * ess[jj];
                    float* top = A + (int64_t)(k + 1 + c) * m + k;
                    tmp = tmp + *top;
                    *top = *top - tau * tmp;
                    s.wa3[c] = tmp;  // scratch: tmp_c (wa3 is free during the QR)
                }
            }
            if (wave == 1) {
                const float* wb = w + k + 1;
                const float tw = elm_redux_wave(depth, [&](int i) { return ess[i] * wb[i]; }, lane);
                if (lane == 0) {
                    const float tmp = tw + w[k];
                    w[k] = w[k] - tau * tmp;
                    s.bc[4] = tmp;
                }
            }
            __syncthreads();
            PITT_QR_T(3);
            const float tmpw = s.bc[4];
            for (int c = 0; c < cols; ++c) {
                float* col = A + (int64_t)(k + 1 + c) * m + k + 1;
                const float tc = s.wa3[c];
                for (int64_t i = tid; i < depth; i += kElmThreads) col[i] = col[i] - (tau * ess[i]) * tc;
            }
            for (int64_t i = tid; i < depth; i += kElmThreads) w[k + 1 + i] = w[k + 1 + i] - (tau * ess[i]) * tmpw;
        }
        __syncthreads();
        PITT_QR_T(4);
        if (tid == 0) {  // the norms downdated, the next pivot
            for (int j = k + 1; j < N; ++j) {
                const float r = A[(int64_t)j * m + k];
                s.sq[j] = s.sq[j] - r * r;
            }
            if (k + 1 < N) {
                int nb = k + 1;
                for (int j = k + 2; j < N; ++j)
                    if (s.sq[j] > s.sq[nb]) nb = j;
                s.ibc[0] = nb;
            }
        }
        __syncthreads();
        PITT_QR_T(5);
    }
    if (tid == 0) {
        for (int k = 0; k < N; ++k) s.perm[k] = k;
        for (int k = 0; k < N; ++k) {
            const int t = s.perm[k];
            s.perm[k] = s.perm[s.transp[k]];
            s.perm[s.transp[k]] = t;
        }
    }
    // the top n x n block for the scalar control
    for (int e = tid; e < N * N; e += kElmThreads) s.R[e / N][e % N] = A[(int64_t)(e / N) * m + (e % N)];
    __syncthreads();
}

// stableNorm of an m-vector (4096-element blocks scaled by the running max): every thread calls it; the
// value is returned to all of them.
template <class F>
__device__ __forceinline__ float elm_stable_block(const float* v, int64_t n, ElmShared<F>& s, float* red) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float scale = 0.0f, inv = 1.0f, ssq = 0.0f;
    for (int64_t bi = 0; bi < n; bi += 4096) {
        const int64_t len = n - bi < 4096 ? n - bi : 4096;
        // maxCoeff with std::max: a NaN first element stays, later NaNs never win
        float mx = 0.0f;
        for (int64_t i = tid; i < len; i += kElmThreads) {
            const float a = fabsf(v[bi + i]);
            if (a > mx) mx = a;
        }
        for (int off = 32; off > 0; off >>= 1) {
            const float o = __shfl_xor(mx, off, 64);
            if (o > mx) mx = o;
        }
        if (lane == 0) red[wave] = mx;
        __syncthreads();
        if (tid == 0) {
            float t = red[0];
            for (int w = 1; w < kElmThreads / 64; ++w)
                if (red[w] > t) t = red[w];
            const float first = fabsf(v[bi]);
            s.bc[0] = first != first ? first : t;
        }
        __syncthreads();
        mx = s.bc[0];
        if (mx > scale) {
            const float r = scale / mx;
            ssq = ssq * (r * r);
            scale = mx;
            inv = 1.0f / scale;
        }
        if (wave == 0) {
            const float* vb = v + bi;
            const float sum = elm_redux_wave(len, [&](int i) { const float t = vb[i] * inv; return t * t; }, lane);
            if (lane == 0) s.bc[1] = sum;
        }
        __syncthreads();
        ssq = ssq + s.bc[1];
        __syncthreads();
    }
    return scale * sqrtf(ssq);
}

// JacobiRotation::makeGivens (real)
__device__ void elm_givens(float p, float q, float* c, float* s) {
    if (q == 0.0f) {
        *c = p < 0.0f ? -1.0f : 1.0f;
        *s = 0.0f;
    } else if (p == 0.0f) {
        *c = 0.0f;
        *s = q < 0.0f ? 1.0f : -1.0f;
    } else if (fabsf(p) > fabsf(q)) {
        const float t = q / p;
        float u = sqrtf(1.0f + t * t);
        if (p < 0.0f) u = -u;
        *c = 1.0f / u;
        *s = -t * *c;
    } else {
        const float t = p / q;
        float u = sqrtf(1.0f + t * t);
        if (q < 0.0f) u = -u;
        *s = -1.0f / u;
        *c = -t * *s;
    }
}

// qrsolv (Eigen 3.2 NonLinearOptimization/qrsolv.h), one thread; S: n x n column-major copy of R.
template <int N>
__device__ void elm_qrsolv(float (&S)[N][N], const int* ipvt, const float* diag, const float* qtb, float* x,
                           float* sdiag) {
    float wa[N];
#pragma unroll
    for (int j = 0; j < N; ++j) wa[j] = qtb[j];
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] = S[j][j];
    // the Givens eliminations on a register copy of S (every index below is a compile-time constant once
    // the loops are unrolled, so S, sdiag and wa stay in VGPRs instead of one LDS round trip per access)
    float Sr[N][N], sd[N];
#pragma unroll
    for (int c = 0; c < N; ++c)
#pragma unroll
        for (int r = 0; r < N; ++r) Sr[c][r] = r > c ? S[r][c] : S[c][r];  // strictly lower = upper^T
#pragma unroll
    for (int k = 0; k < N; ++k) sd[k] = sdiag[k];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const int l = ipvt[j];
        if (diag[l] == 0.0f) break;
#pragma unroll
        for (int k = j; k < N; ++k) sd[k] = 0.0f;
        sd[j] = diag[l];
        float qtbpj = 0.0f;
#pragma unroll
        for (int k = j; k < N; ++k) {
            float gc, gs;
            elm_givens(-Sr[k][k], sd[k], &gc, &gs);
            Sr[k][k] = gc * Sr[k][k] + gs * sd[k];
            const float temp = gc * wa[k] + gs * qtbpj;
            qtbpj = -gs * wa[k] + gc * qtbpj;
            wa[k] = temp;
#pragma unroll
            for (int i = k + 1; i < N; ++i) {
                const float t2 = gc * Sr[k][i] + gs * sd[i];
                sd[i] = -gs * Sr[k][i] + gc * sd[i];
                Sr[k][i] = t2;
            }
        }
    }
#pragma unroll
    for (int c = 0; c < N; ++c)
#pragma unroll
        for (int r = 0; r < N; ++r) S[c][r] = Sr[c][r];
#pragma unroll
    for (int k = 0; k < N; ++k) sdiag[k] = sd[k];
    int nsing = 0;
    while (nsing < N && sdiag[nsing] != 0.0f) ++nsing;
    for (int j = nsing; j < N; ++j) wa[j] = 0.0f;
    // S.topLeftCorner(nsing, nsing).transpose().triangularView<Upper>() x = wa: U(i, j) = S(j, i)
    for (int k = 0; k < nsing; ++k) {
        const int i = nsing - k - 1;
        if (k > 0) wa[i] = wa[i] - elm_redux1(k, [&](int t) { return S[i][i + 1 + t] * wa[i + 1 + t]; });
        wa[i] = wa[i] / S[i][i];
    }
    for (int j = 0; j < N; ++j) {
        sdiag[j] = S[j][j];
        S[j][j] = x[j];
    }
    for (int j = 0; j < N; ++j) x[ipvt[j]] = wa[j];
}

// lmpar2 (Eigen 3.2 NonLinearOptimization/lmpar.h), one thread.
template <class F>
__device__ void elm_lmpar(ElmShared<F>& s, const float* qtb, float delta, float& par, float* x) {
    constexpr int N = F::N;
    const float dwarf = FLT_MIN;
    float wa1[N], wa2[N];
    for (int j = 0; j < N; ++j) wa1[j] = qtb[j];
    // rank(): pivots above maxpivot * eps * diagonalSize
    const float th = fabsf(s.maxpivot) * (FLT_EPSILON * (float)N);
    int rank = 0;
    for (int i = 0; i < s.nonzero_pivots; ++i) rank += fabsf(s.R[i][i]) > th ? 1 : 0;
    for (int j = rank; j < N; ++j) wa1[j] = 0.0f;
    for (int k = 0; k < rank; ++k) {  // R(0..rank) upper solve, column-major panel from the last column
        const int i = rank - k - 1;
        if (wa1[i] != 0.0f) {
            wa1[i] = wa1[i] / s.R[i][i];
            for (int t = 0; t < i; ++t) wa1[t] = wa1[t] - wa1[i] * s.R[i][t];
        }
    }
    for (int i = 0; i < N; ++i) x[s.perm[i]] = wa1[i];
    int iter = 0;
    for (int j = 0; j < N; ++j) wa2[j] = s.diag[j] * x[j];
    float dxnorm = elm_blue1(wa2, N);
    float fp = dxnorm - delta;
    if (fp <= 0.1f * delta) {
        par = 0.0f;
        return;
    }
    float parl = 0.0f;
    if (rank == N) {
        for (int i = 0; i < N; ++i) {
            const int pi = s.perm[i];
            wa1[i] = (s.diag[pi] * wa2[pi]) / dxnorm;
        }
        for (int i = 0; i < N; ++i) {  // R^T lower solve (row-major view)
            if (i > 0) wa1[i] = wa1[i] - elm_redux1(i, [&](int t) { return s.R[i][t] * wa1[t]; });
            wa1[i] = wa1[i] / s.R[i][i];
        }
        const float temp = elm_blue1(wa1, N);
        parl = fp / delta / temp / temp;
    }
    for (int j = 0; j < N; ++j)
        wa1[j] = elm_redux1(j + 1, [&](int i) { return s.R[j][i] * qtb[i]; }) / s.diag[s.perm[j]];
    const float gnorm = elm_stable1(wa1, N);
    float paru = gnorm / delta;
    if (paru == 0.0f) paru = dwarf / elm_min(delta, 0.1f);
    par = elm_max(par, parl);
    par = elm_min(par, paru);
    if (par == 0.0f) par = gnorm / dxnorm;
    float(&S)[N][N] = s.lmS;
    for (int c = 0; c < N; ++c)
        for (int r = 0; r < N; ++r) S[c][r] = s.R[c][r];
    float sdiag[N];
    while (true) {
        ++iter;
        if (par == 0.0f) par = elm_max(dwarf, 0.001f * paru);
        const float sp = sqrtf(par);
        for (int j = 0; j < N; ++j) wa1[j] = sp * s.diag[j];
#ifdef PITT_ELM_PROF
        const unsigned long long tq0 = clock64();
#endif
        elm_qrsolv<N>(S, s.perm, wa1, qtb, x, sdiag);
#ifdef PITT_ELM_PROF
        s.prof_qrsolv += clock64() - tq0;
        ++s.prof_lmpar_iter;
#endif
        for (int j = 0; j < N; ++j) wa2[j] = s.diag[j] * x[j];
        dxnorm = elm_blue1(wa2, N);
        float temp = fp;
        fp = dxnorm - delta;
        if (fabsf(fp) <= 0.1f * delta || (parl == 0.0f && fp <= temp && temp < 0.0f) || iter == 10) break;
        for (int i = 0; i < N; ++i) {
            const int pi = s.perm[i];
            wa1[i] = s.diag[pi] * (wa2[pi] / dxnorm);
        }
        for (int j = 0; j < N; ++j) {
            wa1[j] = wa1[j] / sdiag[j];
            temp = wa1[j];
            for (int i = j + 1; i < N; ++i) wa1[i] = wa1[i] - S[j][i] * temp;
        }
        temp = elm_blue1(wa1, N);
        const float parc = fp / delta / temp / temp;
        if (fp > 0.0f) parl = elm_max(parl, par);
        if (fp < 0.0f) paru = elm_min(paru, par);
        par = elm_max(parl, par + parc);
    }
    if (iter == 0) par = 0.0f;
}

// The residuals of `pre` at every inlier.
template <class F>
__device__ __forceinline__ void elm_eval(const ElmJob& j, const typename F::Pre& pre, float* out) {
    for (int64_t i = threadIdx.x; i < j.m; i += kElmThreads) {
        const int32_t id = j.inl[i];
        out[i] = F::eval(pre, j.x[id], j.y[id], j.z[id]);
    }
}

// The workspace ((N + 2) m floats: the Jacobian, f(x) and the trial residuals) lives in LDS when the
// batch's largest job fits (k_elm<F, true>: the launch's dynamic LDS holds it), else in HBM (ElmJob::work).
// Every m-long serial chain of the LM reads it: from LDS a chain step waits ~100 cycles for its operand,
// from L2/HBM several hundred.
extern __shared__ float elm_dyn[];
constexpr size_t kElmLdsMax = 144 * 1024;  // dynamic LDS budget per block (of the CU's 160 KB)

// LDS: the Jacobian and both residual vectors live in dynamic LDS ((N + 2) m floats <= kElmLdsMax), every
// pointer into them derived from elm_dyn so that the chains read them with ds_read (a pointer that may be
// either LDS or HBM compiles to flat loads, about twice the latency); otherwise in the job's HBM workspace.
template <class F, bool LDS>
__global__ __launch_bounds__(kElmThreads) void k_elm(const ElmJob* __restrict__ jobs) {
    constexpr int N = F::N;
    __shared__ ElmShared<F> s;
    __shared__ float red[kElmThreads / 64];
    const ElmJob j = jobs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t m = j.m;
    if (m < N) {  // minimizeInit: ImproperInputParameters, the model unchanged
        if (tid == 0) {
            F::finish(j.start, j.out);
            if (j.info) j.info[0] = kElmImproper, j.info[1] = 0;
        }
        return;
    }
    float* const ws = LDS ? elm_dyn : j.work;
    float* fjac = ws;
    float* rbuf[2] = {ws + (int64_t)N * m, ws + (int64_t)(N + 1) * m};
    constexpr float factor = 100.0f;
    const float ftol = sqrtf(FLT_EPSILON), xtol = sqrtf(FLT_EPSILON), gtol = 0.0f, eps = FLT_EPSILON;
    constexpr int maxfev = 400;
    const float neps = sqrtf(elm_max(0.0f, FLT_EPSILON));  // NumericalDiff: sqrt(max(epsfcn, eps))
    if (tid == 0) {
#ifdef PITT_ELM_PROF
        s.prof_qrsolv = 0;
        s.prof_lmpar_iter = 0;
#endif
        for (int k = 0; k < N; ++k) s.x[k] = j.start[k];
        F::prep(s.x, s.pre[N]);
        s.cur = 0;
        s.nfev = 1;
        s.par = 0.0f;
        s.delta = 0.0f;
        s.xnorm = 0.0f;
        s.temp = 0.0f;
        s.iter = 1;
        s.status = kElmRunning;
    }
    __syncthreads();
    elm_eval<F>(j, s.pre[N], rbuf[0]);
    __syncthreads();
    {
        const float fn = elm_stable_block(rbuf[0], m, s, red);
        if (tid == 0) s.fnorm = fn;
    }
    __syncthreads();
#ifdef PITT_ELM_PROF  // per-phase cycles of thread 0 (s_memtime), printed at the end
    unsigned long long qprof[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long pc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt = clock64();
    int n_outer = 0, n_inner = 0;
#define PITT_ELM_T(k)                          \
    do {                                       \
        const unsigned long long t_ = clock64(); \
        pc[k] += t_ - pt;                      \
        pt = t_;                               \
    } while (0)
#else
#define PITT_ELM_T(k) \
    do {              \
    } while (0)
#endif
    while (true) {
#ifdef PITT_ELM_PROF
        ++n_outer;
#endif
        float* fvec = rbuf[s.cur];
        float* wa4 = rbuf[s.cur ^ 1];
        // NumericalDiff<Forward>::df: column c = (f(x + h_c e_c) - f(x)) / h_c, h_c = sqrt(eps) |x_c| (or sqrt(eps))
        if (tid < N) {
            float h = neps * fabsf(s.x[tid]);
            if (h == 0.0f) h = neps;
            float q[N];
            for (int k = 0; k < N; ++k) q[k] = s.x[k];
            q[tid] = q[tid] + h;
            s.hstep[tid] = h;
            F::prep(q, s.pre[tid]);
            if (tid == 0) s.ibc[3] = 0;
        }
        __syncthreads();
        // the Jacobian, each column's "every element in blueNorm's middle range" test (bit c of ibc[3] set
        // when some element is not: too big, too small but nonzero, or NaN), and wa4 = f(x) for Q^T f
        {
            const ElmBlue bc = elm_blue_consts();
            const float ab2 = bc.b2 / (float)m;
            int outside = 0;
            for (int64_t i = tid; i < m; i += kElmThreads) {
                const int32_t id = j.inl[i];
                const float px = j.x[id], py = j.y[id], pz = j.z[id];
                const float f0 = fvec[i];
#pragma unroll
                for (int c = 0; c < N; ++c) {
                    const float v = (F::eval(s.pre[c], px, py, pz) - f0) / s.hstep[c];
                    fjac[(int64_t)c * m + i] = v;
                    const float ax = fabsf(v);
                    if (!(ax <= ab2 && (ax >= bc.b1 || ax == 0.0f))) outside |= 1 << c;
                }
                wa4[i] = f0;
            }
            if (outside) atomicOr(&s.ibc[3], outside);
        }
        __syncthreads();
        PITT_ELM_T(0);
        if (tid == 0) s.nfev += N + 1;
        // the columns' blue norms (wa2), wave 1 lane c for column c while wave 0 takes the QR's column norms:
        // a column with every element in the middle range sums only ax^2 (the other two sums stay +0, and a
        // zero element adds +0 to whichever sum takes it), one dependent add per element
        auto blue = [&](int ln) {
            if (ln >= N) return;
            const float* col = fjac + (int64_t)ln * m;
            float r;
            if (!((s.ibc[3] >> ln) & 1)) {
                r = sqrtf(elm_chain<1>(0, (int)m, 0.0f, [&](int i) { const float v = col[i]; return v * v; }));
            } else {
                const ElmBlue c = elm_blue_consts();
                const float ab2 = c.b2 / (float)m;
                float asml = 0.0f, amed = 0.0f, abig = 0.0f;
                int64_t i = 0;
                for (; i + 3 < m; i += 4) {
                    const float v0 = col[i], v1 = col[i + 1], v2 = col[i + 2], v3 = col[i + 3];
                    elm_blue_step(c, ab2, v0, asml, amed, abig);
                    elm_blue_step(c, ab2, v1, asml, amed, abig);
                    elm_blue_step(c, ab2, v2, asml, amed, abig);
                    elm_blue_step(c, ab2, v3, asml, amed, abig);
                }
                for (; i < m; ++i) elm_blue_step(c, ab2, col[i], asml, amed, abig);
                r = elm_blue_finish(c, asml, amed, abig);
            }
            s.colnorm[ln] = r;
        };
        PITT_ELM_T(1);
        // the QR, with qtf = (Q^T f)(0..n) formed in wa4 on the way
#ifdef PITT_ELM_PROF
        elm_qr<F>(fjac, m, wa4, s, blue, qprof);
#else
        elm_qr<F>(fjac, m, wa4, s, blue);
#endif
        PITT_ELM_T(2);
        if (tid == 0 && s.iter == 1) {
            for (int k = 0; k < N; ++k) s.diag[k] = s.colnorm[k] == 0.0f ? 1.0f : s.colnorm[k];
            float dx[N];
            for (int k = 0; k < N; ++k) dx[k] = s.diag[k] * s.x[k];
            s.xnorm = elm_stable1(dx, N);
            s.delta = factor * s.xnorm;
            if (s.delta == 0.0f) s.delta = factor;
        }
        PITT_ELM_T(3);
        if (tid == 0) {
            for (int k = 0; k < N; ++k) s.qtf[k] = wa4[k];
            float gnorm = 0.0f;
            if (s.fnorm != 0.0f)
                for (int c = 0; c < N; ++c) {
                    const float w = s.colnorm[s.perm[c]];
                    if (w != 0.0f) {
                        const float fn = s.fnorm;
                        const float d = elm_redux1(c + 1, [&](int i) { return s.R[c][i] * (s.qtf[i] / fn); });
                        gnorm = elm_max(gnorm, fabsf(d / w));
                    }
                }
            s.gnorm = gnorm;
            if (gnorm <= gtol) s.status = kElmCosinus;
            else
                for (int k = 0; k < N; ++k) s.diag[k] = elm_max(s.diag[k], s.colnorm[k]);
        }
        __syncthreads();
        if (s.status != kElmRunning) break;
        // the inner loop: trial steps until one is accepted (ratio >= 1e-4) or a test stops
        while (true) {
#ifdef PITT_ELM_PROF
            ++n_inner;
#endif
            PITT_ELM_T(4);
            if (tid == 0) {
                float step[N];
                elm_lmpar<F>(s, s.qtf, s.delta, s.par, step);
                for (int k = 0; k < N; ++k) s.wa1[k] = -step[k];
                for (int k = 0; k < N; ++k) s.wa2[k] = s.x[k] + s.wa1[k];
                float dp[N];
                for (int k = 0; k < N; ++k) dp[k] = s.diag[k] * s.wa1[k];
                s.bc[6] = elm_stable1(dp, N);  // pnorm
                if (s.iter == 1) s.delta = elm_min(s.delta, s.bc[6]);
                F::prep(s.wa2, s.pre[N]);
            }
            __syncthreads();
            PITT_ELM_T(5);
            float* trial = rbuf[s.cur ^ 1];
            elm_eval<F>(j, s.pre[N], trial);
            __syncthreads();
            PITT_ELM_T(6);
            const float fnorm1 = elm_stable_block(trial, m, s, red);
            PITT_ELM_T(7);
            if (tid == 0) {
                ++s.nfev;
                const float pnorm = s.bc[6];
                float actred = -1.0f;
                if (0.1f * fnorm1 < s.fnorm) {
                    const float q = fnorm1 / s.fnorm;
                    actred = 1.0f - q * q;
                }
                // wa3 = R * (P^-1 * wa1): Eigen's upper TRMV, column by column
                float pw[N];
                for (int i = 0; i < N; ++i) pw[i] = s.wa1[s.perm[i]];
                for (int r = 0; r < N; ++r) s.wa3[r] = 0.0f;
                for (int i = 0; i < N; ++i)
                    for (int r = 0; r <= i; ++r) s.wa3[r] = s.wa3[r] + pw[i] * s.R[i][r];
                const float t1 = elm_stable1(s.wa3, N) / s.fnorm;
                const float temp1 = t1 * t1;
                const float t2 = sqrtf(s.par) * pnorm / s.fnorm;
                const float temp2 = t2 * t2;
                const float prered = temp1 + temp2 / 0.5f;
                const float dirder = -(temp1 + temp2);
                float ratio = 0.0f;
                if (prered != 0.0f) ratio = actred / prered;
                if (ratio <= 0.25f) {
                    if (actred >= 0.0f) s.temp = 0.5f;
                    if (actred < 0.0f) s.temp = 0.5f * dirder / (dirder + 0.5f * actred);
                    if (0.1f * fnorm1 >= s.fnorm || s.temp < 0.1f) s.temp = 0.1f;
                    s.delta = s.temp * elm_min(s.delta, pnorm / 0.1f);
                    s.par = s.par / s.temp;
                } else if (!(s.par != 0.0f && ratio < 0.75f)) {
                    s.delta = pnorm / 0.5f;
                    s.par = 0.5f * s.par;
                }
                if (ratio >= 1e-4f) {  // accepted: x, f(x) and the norms move to the trial point
                    for (int k = 0; k < N; ++k) s.x[k] = s.wa2[k];
                    float dx[N];
                    for (int k = 0; k < N; ++k) dx[k] = s.diag[k] * s.x[k];
                    s.cur ^= 1;
                    s.xnorm = elm_stable1(dx, N);
                    s.fnorm = fnorm1;
                    ++s.iter;
                }
                int st = kElmRunning;
                if (fabsf(actred) <= ftol && prered <= ftol && 0.5f * ratio <= 1.0f) st = kElmRelReduction;
                else if (s.delta <= xtol * s.xnorm) st = kElmRelError;
                else if (s.nfev >= maxfev) st = kElmMaxFev;
                else if (fabsf(actred) <= eps && prered <= eps && 0.5f * ratio <= 1.0f) st = kElmFtol;
                else if (s.delta <= eps * s.xnorm) st = kElmXtol;
                else if (s.gnorm <= eps) st = kElmGtol;
                s.status = st;
                s.ibc[2] = (st == kElmRunning && ratio < 1e-4f) ? 1 : 0;  // another trial step
            }
            __syncthreads();
            if (!s.ibc[2]) break;
        }
        PITT_ELM_T(4);
        if (s.status != kElmRunning) break;
    }
#ifdef PITT_ELM_PROF
    if (tid == 0)
        printf("PITT_ELM_PROF N %d m %lld outer %d inner %d nfev %d status %d cycles: jacobian %llu qr %llu post %llu "
               "lmpar %llu (qrsolv %llu in %d iterations) eval %llu stable %llu logic %llu | qr: norms %llu pivnorm %llu "
               "swap %llu gemv %llu update %llu downdate %llu\n",
               N, (long long)m, n_outer, n_inner, s.nfev, s.status, pc[0], pc[2], pc[3], pc[5], s.prof_qrsolv,
               s.prof_lmpar_iter, pc[6], pc[7], pc[4], qprof[0], qprof[1], qprof[2], qprof[3], qprof[4], qprof[5]);
#endif
#undef PITT_ELM_T
    if (tid == 0) {
        F::finish(s.x, j.out);
        if (j.info) j.info[0] = s.status, j.info[1] = s.nfev;
    }
}

// One launch for a batch of refinements of one model kind (one block each).
template <class F>
inline int launch_elm_batch(pitt_ctx* ctx, hipStream_t s, std::vector<ElmJob>& jobs, const char* name) {
    if (jobs.empty()) return PITT_OK;
    size_t words = 0;
    int64_t m_max = 0;
    for (const ElmJob& jb : jobs) {
        words += (size_t)(F::N + 2) * (size_t)jb.m + 64;
        m_max = std::max<int64_t>(m_max, jb.m);
    }
    const size_t lds_bytes = (size_t)(F::N + 2) * (size_t)m_max * sizeof(float);
    const int lds = lds_bytes <= kElmLdsMax ? 1 : 0;
    if (lds) {
        static bool attr_set = false;  // once per kernel instantiation (one per model kind)
        if (!attr_set) {
            PITT_HIP_TRY(hipFuncSetAttribute((const void*)k_elm<F, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)kElmLdsMax));
            attr_set = true;
        }
    }
    float* work = (float*)ctx->buf(std::string(name) + "_elm_work", words * 4);
    const size_t bytes = jobs.size() * sizeof(ElmJob);
    auto* h = (ElmJob*)ctx->pinned(std::string(name) + "_elm_jobs_h", bytes);
    auto* d = (ElmJob*)ctx->buf(std::string(name) + "_elm_jobs", bytes);
    if (!work || !h || !d) return ctx->fail(PITT_E_NOMEM, "lm scratch");
    size_t off = 0;
    for (ElmJob& jb : jobs) {
        jb.work = work + off;
        off += (size_t)(F::N + 2) * (size_t)jb.m + 64;
    }
    std::copy(jobs.begin(), jobs.end(), h);
    PITT_HIP_TRY(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    if (lds)
        hipLaunchKernelGGL((k_elm<F, true>), dim3((unsigned)jobs.size()), dim3(kElmThreads), lds_bytes, s, d);
    else
        hipLaunchKernelGGL((k_elm<F, false>), dim3((unsigned)jobs.size()), dim3(kElmThreads), 0, s, d);
    PITT_HIP_TRY(hipGetLastError());
#ifdef PITT_SYNC_CHECK
    ctx->check_canaries(name);
#endif
    return PITT_OK;
}

// ---- the three models' OptimizationFunctors (sac_model_{sphere,cylinder,cone}.h), as the oracle's
// pcl_lm_* restate them ---------------------------------------------------------------------------------
// sphere: fvec[i] = sqrtf(cen_t.dot(cen_t)) - x[3], cen_t = (p - x[0..2], 0) (Vector4f dot, SSE2 order)
struct ElmSphere {
    static constexpr int N = 4;
    struct Pre {
        float q[4];
    };
    __device__ static void prep(const float* q, Pre& p) {
        for (int k = 0; k < 4; ++k) p.q[k] = q[k];
    }
    __device__ static float eval(const Pre& p, float px, float py, float pz) {
        const float cx = px - p.q[0], cy = py - p.q[1], cz = pz - p.q[2];
        return sqrtf((cx * cx + cz * cz) + (cy * cy + 0.0f * 0.0f)) - p.q[3];
    }
    __device__ static void finish(const float* x, float* out) {
        for (int k = 0; k < 4; ++k) out[k] = x[k];
    }
};
// line_dir.normalize() after the 7-parameter models' LM (Vector3f: a0 + (a1 + a2), times 1 / norm)
__device__ __forceinline__ void elm_finish7(const float* x, float* out) {
    for (int k = 0; k < 7; ++k) out[k] = x[k];
    const float r = 1.0f / sqrtf(x[3] * x[3] + (x[4] * x[4] + x[5] * x[5]));
    out[3] = x[3] * r;
    out[4] = x[4] * r;
    out[5] = x[5] * r;
}
// cylinder: fvec[i] = (float)(sqrPointToLineDistance(pt, line_pt, line_dir) - x[6] * x[6])
struct ElmCylinder {
    static constexpr int N = 7;
    struct Pre {
        CV4 lp, ld;
        float r2;
    };
    __device__ static void prep(const float* q, Pre& p) {
        p.lp = cv4(q[0], q[1], q[2], 0.0f);
        p.ld = cv4(q[3], q[4], q[5], 0.0f);
        p.r2 = q[6] * q[6];
    }
    __device__ static float eval(const Pre& p, float px, float py, float pz) {
        return (float)(csqr_pt_line(cv4(px, py, pz, 0.0f), p.lp, p.ld) - (double)p.r2);
    }
    __device__ static void finish(const float* x, float* out) { elm_finish7(x, out); }
};
// cone: fvec[i] = (float)(sqrPointToLineDistance(pt, apex, dir) - r * r), r = tanf(x[6]) |apex - proj(pt)|
// (A7: tanf as the correctly rounded float of the double tan)
struct ElmCone {
    static constexpr int N = 7;
    struct Pre {
        CV4 apex, ad;
        float apexdotdir, dirdotdir, ta;
    };
    __device__ static void prep(const float* q, Pre& p) {
        p.apex = cv4(q[0], q[1], q[2], 0.0f);
        p.ad = cv4(q[3], q[4], q[5], 0.0f);
        p.apexdotdir = cdot(p.apex, p.ad);
        p.dirdotdir = 1.0f / cdot(p.ad, p.ad);
        p.ta = (float)tan((double)q[6]);
    }
    __device__ static float eval(const Pre& p, float px, float py, float pz) {
        const CV4 pt = cv4(px, py, pz, 0.0f);
        const float k = (cdot(pt, p.ad) - p.apexdotdir) * p.dirdotdir;
        const CV4 proj = cadd(p.apex, cmul(k, p.ad));
        const CV4 h = csub(p.apex, proj);
        const float rad = p.ta * sqrtf(cdot(h, h));
        return (float)(csqr_pt_line(pt, p.apex, p.ad) - (double)(rad * rad));
    }
    __device__ static void finish(const float* x, float* out) { elm_finish7(x, out); }
};

}  // namespace pitt
