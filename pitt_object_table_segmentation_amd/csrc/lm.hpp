// lm.hpp -- the oracle's lm_solve<N> (oracle/pitt_oracle.cpp) on the device: Levenberg-Marquardt in double
// with Marquardt damping (lambda * diag, x10 / x0.1, stop when no damping lowers the cost, the step falls
// below 1e-10 relative, accepted or rejected, or the iteration cap passes) over a model's residual summed over an inlier list by a
// small resident grid (deterministic sums: per lane, then a fixed wave, block and grid order).  Used by the
// sphere (sphere.hip, 4 parameters), cylinder (cylinder.hip) and cone (cone.hip) services (7 parameters).
//
// A model P provides: N, kMaxIt, kDiagEps (added to the damped diagonal), kSmall (inlier counts up to it
// run as one block, measured per model), init(v), aux(v) (a per-evaluation constant handed to the
// residual as v[N]), residual(v, px, py, pz, J[N], &f) and finish(xv, out) -- the float coefficients as
// PCL's optimizeModelCoefficients writes them.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "ctx.hpp"

#pragma clang fp contract(off)

namespace pitt {

struct Coef7 {
    float c[7];
    float pad;
};

constexpr int kLmThreads = 256;  // one wave per SIMD: the 36 double accumulators stay in VGPRs
constexpr int kLmMaxN = 7;
constexpr int kLmMaxSums = kLmMaxN * (kLmMaxN + 1) / 2 + kLmMaxN + 1;
constexpr int kLmMaxBlocks = 64;
template <int N>
constexpr int lm_sums() { return N * (N + 1) / 2 + N + 1; }  // co-resident on any idle MI355X (256 CUs): the grid barrier needs it

// Shared between the blocks of one k_lm7 launch (device scratch; bar zeroed before the launch).
struct LmGlobal {
    double part[kLmMaxBlocks][kLmMaxSums];
    double xn[kLmMaxN];
    int32_t state;  // 0 evaluate xn, 3 stop
    uint32_t bar;
};

// Grid barrier over a monotonically rising arrival counter: barrier j waits for j * gridDim.x arrivals.
// Agent-scope release / acquire make the blocks' writes visible across the XCDs' L2s.
__device__ __forceinline__ void lm_grid_sync(uint32_t* bar, uint32_t& target) {
    __syncthreads();
    target += gridDim.x;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        // poll relaxed (no cache invalidation per poll), then one acquire fence
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// This block's share of J^T J (upper triangle), J^T f and f^T f at v, in a fixed order: per lane over the
// points gid, gid + G * 256, ...; then the wave (xor shuffles), then the four waves in order.
template <class P>
__device__ void lm_partial(const P& prm, const float* X, const float* Y, const float* Z, const int32_t* inl,
                           int64_t m, const double* v, double (*red)[kLmMaxSums], double* out, int blk, int nblk) {
    constexpr int N = P::N, S = lm_sums<N>();
    double acc[S];
#pragma unroll
    for (int q = 0; q < S; ++q) acc[q] = 0;
    double w[N + 1];  // the point, then the model's per-evaluation constant (aux: e.g. the cone's tan)
#pragma unroll
    for (int q = 0; q < N; ++q) w[q] = v[q];
    w[N] = prm.aux(v);
    for (int64_t k = (int64_t)blk * kLmThreads + threadIdx.x; k < m; k += (int64_t)nblk * kLmThreads) {
        const int id = inl[k];
        double J[N], f;
        prm.residual(w, X[id], Y[id], Z[id], J, &f);
        int t = 0;
#pragma unroll
        for (int a = 0; a < N; ++a)
#pragma unroll
            for (int b = a; b < N; ++b) acc[t++] += J[a] * J[b];
#pragma unroll
        for (int a = 0; a < N; ++a) acc[N * (N + 1) / 2 + a] += J[a] * f;
        acc[S - 1] += f * f;
    }
#pragma unroll
    for (int q = 0; q < S; ++q) {
        double t = acc[q];
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][q] = t;
    }
    __syncthreads();
    if (threadIdx.x < S) {
        double t = 0;
        for (int w = 0; w < kLmThreads / 64; ++w) t += red[w][threadIdx.x];
        out[threadIdx.x] = t;
    }
}

// Block 0: the grid's partial sums, loaded by all its threads at once into LDS, then summed per entry over
// the blocks in order.
template <int S>
__device__ void lm_reduce_grid(const LmGlobal* g, double* stage, double* out) {
    const int G = (int)gridDim.x;
    for (int e = threadIdx.x; e < G * S; e += kLmThreads) stage[e] = g->part[e / S][e % S];
    __syncthreads();
    if (threadIdx.x < S) {
        double t = 0;
        for (int b = 0; b < G; ++b) t += stage[b * S + threadIdx.x];
        out[threadIdx.x] = t;
    }
}

// The damped N x N system of the oracle's lm_solve<N> (M = J^T J + lambda diag + eps, rhs -J^T f), Gaussian
// elimination with partial pivoting in its exact operation order, fully unrolled so M stays in registers
// (the pivot row swap is a select per element).  false when a pivot is 0.
template <int N>
__device__ __forceinline__ bool lm_solve_dev(const double* sums, double lambda, double eps, double dl[N]) {
    double M[N][N + 1];
    int t = 0;
#pragma unroll
    for (int a = 0; a < N; ++a)
#pragma unroll
        for (int b = a; b < N; ++b) {
            M[a][b] = sums[t];
            M[b][a] = sums[t];
            ++t;
        }
#pragma unroll
    for (int a = 0; a < N; ++a) {
        M[a][a] += lambda * M[a][a] + eps;
        M[a][N] = -sums[N * (N + 1) / 2 + a];
    }
#pragma unroll
    for (int col = 0; col < N; ++col) {
        int piv = col;
        double best = fabs(M[col][col]);
#pragma unroll
        for (int r = col + 1; r < N; ++r) {
            const double v = fabs(M[r][col]);
            if (v > best) best = v, piv = r;
        }
        if (best == 0) return false;
#pragma unroll
        for (int r = col + 1; r < N; ++r) {
            const bool sw = piv == r;
#pragma unroll
            for (int k = 0; k <= N; ++k) {
                const double a = M[col][k], b = M[r][k];
                M[col][k] = sw ? b : a;
                M[r][k] = sw ? a : b;
            }
        }
#pragma unroll
        for (int r = col + 1; r < N; ++r) {
            const double f = M[r][col] / M[col][col];
#pragma unroll
            for (int k = col; k <= N; ++k) M[r][k] -= f * M[col][k];
        }
    }
#pragma unroll
    for (int r = N - 1; r >= 0; --r) {
        double acc = M[r][N];
#pragma unroll
        for (int k = r + 1; k < N; ++k) acc -= M[r][k] * dl[k];
        dl[r] = acc / M[r][r];
    }
    return true;
}

// Block-shared state of one Levenberg-Marquardt run (GRID: the partial-sum staging of a multi-block run).
template <int N, bool GRID>
struct LmShared {
    static constexpr int S = lm_sums<N>();
    double red[kLmThreads / 64][kLmMaxSums];
    double stage[GRID ? kLmMaxBlocks * S : 1];
    double cur[S], trial[S];
    double xv[N], xn[N], dl[N];  // block 0's current point, the trial point it publishes, their step
    int32_t st_s;
};

// The oracle's lm_solve<N> (oracle/pitt_oracle.cpp, sphere_refine / lm_solve) on nblk resident blocks
// (blk = this block's index).  Block 0's thread 0 runs the scalar control (Marquardt damping x10 / x0.1,
// accept on a lower cost, stop when no damping lowers it, the step dl (accepted or rejected) falls below
// 1e-10 relative to the trial point -- the oracle's measure -- or P::kMaxIt iterations pass); every block
// sums its share of the residuals at each trial point.  One block (`one`): partial sums straight into
// LDS, __syncthreads for the barriers.  Several (GRID): two grid barriers per evaluation, after the trial
// point is published and after the partial sums are written (block 0 reduces them in order).
template <class P, bool GRID>
__device__ void lm_run(const P& prm, const float* __restrict__ X, const float* __restrict__ Y,
                       const float* __restrict__ Z, const int32_t* __restrict__ inl, int64_t m, LmGlobal* g,
                       typename P::Out* out, bool one, int blk, int nblk, LmShared<P::N, GRID>& sh) {
    constexpr int N = P::N, S = lm_sums<N>();
    double v0[N];
    prm.init(v0);
    uint32_t target = 0;
    lm_partial(prm, X, Y, Z, inl, m, v0, sh.red, one ? sh.cur : g->part[blk], blk, nblk);
    const bool ctl = blk == 0;
    if constexpr (GRID) {
        if (!one) {
            lm_grid_sync(&g->bar, target);
            if (ctl) lm_reduce_grid<S>(g, sh.stage, sh.cur);
        }
    }
    if (ctl && threadIdx.x < N) sh.xv[threadIdx.x] = v0[threadIdx.x];
    // control state (block 0, thread 0)
    double lambda = 1e-3;
    int it = 0;
    bool have_trial = false;
    for (;;) {
        if (ctl) __syncthreads();
        if (ctl && threadIdx.x == 0) {
            bool stop = false;
            if (have_trial) {
                double rs = 0, rx = 0;  // the step and the trial point, as the oracle measures them
                for (int r = 0; r < N; ++r) {
                    rs += sh.dl[r] * sh.dl[r];
                    rx += sh.xn[r] * sh.xn[r];
                }
                const bool small = sqrt(rs / (rx + 1e-300)) < 1e-10;
                if (sh.trial[S - 1] < sh.cur[S - 1]) {  // accepted: the end of an outer iteration
                    for (int r = 0; r < N; ++r) sh.xv[r] = sh.xn[r];
                    for (int q = 0; q < S; ++q) sh.cur[q] = sh.trial[q];
                    lambda *= 0.1;
                    ++it;
                    stop = small || it >= P::kMaxIt;
                } else {  // a rejected step below 1e-10 relative cannot change the float result: stop
                    stop = small;
                    lambda *= 10;
                }
            }
            if (!stop && !(lambda < 1e10)) stop = true;  // no damping lowered the cost
            double dl[N];
            if (!stop && !lm_solve_dev<N>(sh.cur, lambda, P::kDiagEps, dl)) stop = true;
            if (!stop)
                for (int r = 0; r < N; ++r) {
                    sh.dl[r] = dl[r];
                    sh.xn[r] = sh.xv[r] + dl[r];
                    if constexpr (GRID)
                        if (!one) g->xn[r] = sh.xn[r];
                }
            sh.st_s = stop ? 3 : 0;
            if constexpr (GRID)
                if (!one) g->state = sh.st_s;
        }
        double vn[N];
        if (one) {
            __syncthreads();
            if (sh.st_s == 3) break;
#pragma unroll
            for (int k = 0; k < N; ++k) vn[k] = sh.xn[k];
            lm_partial(prm, X, Y, Z, inl, m, vn, sh.red, sh.trial, blk, nblk);
        } else if constexpr (GRID) {
            lm_grid_sync(&g->bar, target);
            if (__hip_atomic_load(&g->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3) break;
#pragma unroll
            for (int k = 0; k < N; ++k) vn[k] = __hip_atomic_load(&g->xn[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lm_partial(prm, X, Y, Z, inl, m, vn, sh.red, g->part[blk], blk, nblk);
            lm_grid_sync(&g->bar, target);
            if (ctl) lm_reduce_grid<S>(g, sh.stage, sh.trial);
        }
        have_trial = true;
    }
    if (ctl && threadIdx.x == 0) prm.finish(sh.xv, out);
}

template <class P>
__global__ __launch_bounds__(kLmThreads) void k_lm(P prm, const float* __restrict__ X, const float* __restrict__ Y,
                                                   const float* __restrict__ Z, const int32_t* __restrict__ inl,
                                                   int64_t m, LmGlobal* __restrict__ g, typename P::Out* __restrict__ out) {
    __shared__ LmShared<P::N, true> sh;
    lm_run<P, true>(prm, X, Y, Z, inl, m, g, out, gridDim.x == 1, (int)blockIdx.x, (int)gridDim.x, sh);
}

// One refinement per block (pitt_classify_clusters: every cluster's model of one kind at once); each
// block runs the one-block form of k_lm on its job, so a job's result is the single launch's bit for bit.
template <class P>
struct LmJob {
    P prm;
    const float *x, *y, *z;
    const int32_t* inl;
    int64_t m;
    typename P::Out* out;
};
template <class P>
__global__ __launch_bounds__(kLmThreads) void k_lm_batch(const LmJob<P>* __restrict__ jobs) {
    __shared__ LmShared<P::N, false> sh;
    const LmJob<P> j = jobs[blockIdx.x];
    lm_run<P, false>(j.prm, j.x, j.y, j.z, j.inl, j.m, nullptr, j.out, true, 0, 1, sh);
}

// Host side: G = ceil(m / 1024) blocks (at most kLmMaxBlocks, and no more than can be resident at once:
// the grid barrier needs every block running), the barrier counter zeroed on the stream.
template <class P>
inline int launch_lm(pitt_ctx* ctx, hipStream_t s, const P& prm, const float* x, const float* y, const float* z,
                     const int32_t* inl, int64_t m, typename P::Out* out, const char* scratch = "lm_global") {
    // scratch: one LmGlobal per stream that may run a grid refinement (its barrier and partial sums)
    LmGlobal* g = (LmGlobal*)ctx->buf(scratch, sizeof(LmGlobal));
    if (!g) return ctx->fail(PITT_E_NOMEM, "lm scratch");
    // up to P::kSmall inliers one block (no grid barrier: two device-memory round trips per evaluation
    // cost more than the 256 threads' extra points), above that one block per 1024 inliers
    int G = m <= P::kSmall ? 1 : (int)std::min<int64_t>(kLmMaxBlocks, (m + 1023) / 1024);
    if (G > 1) {
        static int resident = -1;  // blocks of k_lm<P> the device holds at once
        if (resident < 0) {
            int per_cu = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&k_lm<P>),
                                                             kLmThreads, 0) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess)
                return ctx->fail(PITT_E_HIP, "lm occupancy query");
            resident = per_cu * cus;
        }
        if (resident < 1) return ctx->fail(PITT_E_HIP, "lm kernel cannot be resident");
        G = std::min(G, resident);
    }
    PITT_HIP_TRY(hipMemsetAsync(&g->bar, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_lm<P>, dim3(G), dim3(kLmThreads), 0, s, prm, x, y, z, inl, m, g, out);
    PITT_HIP_TRY(hipGetLastError());
    return PITT_OK;
}

// A batch of one-block refinements (every job's m <= P::kSmall) in one launch.
template <class P>
inline int launch_lm_batch(pitt_ctx* ctx, hipStream_t s, const std::vector<LmJob<P>>& jobs, const char* name) {
    if (jobs.empty()) return PITT_OK;
    const size_t bytes = jobs.size() * sizeof(LmJob<P>);
    auto* h = (LmJob<P>*)ctx->pinned(std::string(name) + "_lmjobs_h", bytes);
    auto* d = (LmJob<P>*)ctx->buf(std::string(name) + "_lmjobs", bytes);
    if (!h || !d) return ctx->fail(PITT_E_NOMEM, "lm batch scratch");
    std::copy(jobs.begin(), jobs.end(), h);
    PITT_HIP_TRY(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_lm_batch<P>, dim3((unsigned)jobs.size()), dim3(kLmThreads), 0, s, d);
    PITT_HIP_TRY(hipGetLastError());
    return PITT_OK;
}

// The 7-parameter models (cylinder: point on the axis, direction, radius; cone: apex, direction, opening
// angle): R is the residual functor; finish writes the float coefficients with the direction normalised as
// Eigen::Vector3f::normalize() (fixed size 3: a0 + (a1 + a2), times 1 / norm).
template <class R>
struct Lm7Model {
    static constexpr int N = 7;
    static constexpr int kMaxIt = 200;
    static constexpr double kDiagEps = 1e-30;
    static constexpr int64_t kSmall = R::kSmall;
    using Out = Coef7;
    Coef7 start;
    __device__ void init(double* v) const {
        for (int k = 0; k < 7; ++k) v[k] = start.c[k];
    }
    __device__ double aux(const double* v) const { return R::aux(v); }
    __device__ void residual(const double* v, float px, float py, float pz, double* J, double* f) const {
        R{}(v, px, py, pz, J, f);
    }
    __device__ void finish(const double* xv, Coef7* out) const {
        Coef7 o = {};
        for (int k = 0; k < 3; ++k) o.c[k] = (float)xv[k];
        const float u0 = (float)xv[3], u1 = (float)xv[4], u2 = (float)xv[5];
        const float r = 1.0f / sqrtf(u0 * u0 + (u1 * u1 + u2 * u2));
        o.c[3] = u0 * r;
        o.c[4] = u1 * r;
        o.c[5] = u2 * r;
        o.c[6] = (float)xv[6];
        *out = o;
    }
};
template <class R>
inline int launch_lm7(pitt_ctx* ctx, hipStream_t s, R, const float* x, const float* y, const float* z,
                      const int32_t* inl, int64_t m, const Coef7& init, Coef7* out) {
    return launch_lm(ctx, s, Lm7Model<R>{init}, x, y, z, inl, m, out);
}

// fewer residuals than parameters (m < 7): Eigen's LM returns ImproperInputParameters and leaves the model;
// optimizeModelCoefficients still normalises the direction
template <int = 0>  // a template, so the header can be included by several translation units
__global__ void k_lm7_normalize_dir(Coef7 m, Coef7* out) {
    const float u0 = m.c[3], u1 = m.c[4], u2 = m.c[5];
    const float r = 1.0f / sqrtf(u0 * u0 + (u1 * u1 + u2 * u2));
    m.c[3] = u0 * r;
    m.c[4] = u1 * r;
    m.c[5] = u2 * r;
    *out = m;
}

}  // namespace pitt
