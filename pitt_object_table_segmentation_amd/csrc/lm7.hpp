// lm7.hpp -- the oracle's lm_solve<7> (oracle/pitt_oracle.cpp) on the device: Levenberg-Marquardt in double
// with Marquardt damping (lambda * diag, x10 / x0.1, stop when no damping lowers the cost or the step is
// below 1e-12 relative) over a residual R(v, px, py, pz, J[7], &f) summed over an inlier list, all in one
// 1024-thread block (deterministic sums: per-lane, then a fixed wave and block order).  On exit the
// direction v[3..5] is normalised as PCL's optimizeModelCoefficients does (Eigen::Vector3f::normalize:
// a0 + (a1 + a2), times 1 / norm).  Used by the cylinder (cylinder.hip) and cone (cone.hip) services.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#pragma clang fp contract(off)

namespace pitt {

struct Coef7 {
    float c[7];
    float pad;
};

constexpr int kLmThreads = 1024;
constexpr int kLmSums = 28 + 7 + 1;

template <class R>
__device__ void lm7_sums(R res, const float* X, const float* Y, const float* Z, const int32_t* inl, int64_t m,
                            const double* v, double (*red)[kLmSums], double* out) {
    double acc[kLmSums];
    for (int q = 0; q < kLmSums; ++q) acc[q] = 0;
    for (int64_t k = threadIdx.x; k < m; k += kLmThreads) {
        const int id = inl[k];
        double J[7], f;
        res(v, X[id], Y[id], Z[id], J, &f);
        int t = 0;
        for (int a = 0; a < 7; ++a)
            for (int b = a; b < 7; ++b) acc[t++] += J[a] * J[b];
        for (int a = 0; a < 7; ++a) acc[28 + a] += J[a] * f;
        acc[35] += f * f;
    }
    for (int q = 0; q < kLmSums; ++q) {
        double t = acc[q];
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][q] = t;
    }
    __syncthreads();
    if (threadIdx.x < kLmSums) {
        double t = 0;
        for (int w = 0; w < kLmThreads / 64; ++w) t += red[w][threadIdx.x];
        out[threadIdx.x] = t;
    }
    __syncthreads();
}

// the oracle's lm_solve<7>: Marquardt damping, the damped 7 x 7 system solved by thread 0
template <class R>
__global__ __launch_bounds__(kLmThreads) void k_lm7(R res, const float* __restrict__ X, const float* __restrict__ Y,
                                                          const float* __restrict__ Z, const int32_t* __restrict__ inl,
                                                          int64_t m, Coef7 init, Coef7* __restrict__ out) {
    __shared__ double red[kLmThreads / 64][kLmSums];
    __shared__ double cur[kLmSums], trial[kLmSums];
    __shared__ double xv[7], xn[7];
    __shared__ int state;
    if (threadIdx.x == 0)
        for (int k = 0; k < 7; ++k) xv[k] = init.c[k];
    __syncthreads();
    lm7_sums(res, X, Y, Z, inl, m, xv, red, cur);
    double lambda = 1e-3;
    for (int it = 0; it < 200; ++it) {
        bool moved = false, stop = false;
        for (;;) {
            if (threadIdx.x == 0) {
                state = 0;
                if (!(lambda < 1e10)) state = 3;
                else {
                    double M[7][8];
                    int t = 0;
                    for (int a = 0; a < 7; ++a)
                        for (int b = a; b < 7; ++b) M[a][b] = M[b][a] = cur[t++];
                    for (int a = 0; a < 7; ++a) M[a][a] += lambda * M[a][a] + 1e-30, M[a][7] = -cur[28 + a];
                    for (int col = 0; col < 7 && state == 0; ++col) {
                        int piv = col;
                        for (int r = col + 1; r < 7; ++r)
                            if (fabs(M[r][col]) > fabs(M[piv][col])) piv = r;
                        if (M[piv][col] == 0) {
                            state = 3;
                            break;
                        }
                        if (piv != col)
                            for (int k = 0; k < 8; ++k) {
                                const double tt = M[col][k];
                                M[col][k] = M[piv][k];
                                M[piv][k] = tt;
                            }
                        for (int r = col + 1; r < 7; ++r) {
                            const double f = M[r][col] / M[col][col];
                            for (int k = col; k < 8; ++k) M[r][k] -= f * M[col][k];
                        }
                    }
                    if (state == 0) {
                        double dl[7];
                        for (int r = 6; r >= 0; --r) {
                            double acc = M[r][7];
                            for (int k = r + 1; k < 7; ++k) acc -= M[r][k] * dl[k];
                            dl[r] = acc / M[r][r];
                        }
                        for (int r = 0; r < 7; ++r) xn[r] = xv[r] + dl[r];
                    }
                }
            }
            __syncthreads();
            const int st0 = state;
            __syncthreads();
            if (st0 == 3) {
                stop = true;
                break;
            }
            lm7_sums(res, X, Y, Z, inl, m, xn, red, trial);
            if (threadIdx.x == 0) {
                if (trial[35] < cur[35]) {
                    double step = 0, nx = 0;
                    for (int r = 0; r < 7; ++r) {
                        const double d = xn[r] - xv[r];
                        step += d * d;
                        nx += xn[r] * xn[r];
                        xv[r] = xn[r];
                    }
                    for (int q = 0; q < kLmSums; ++q) cur[q] = trial[q];
                    lambda *= 0.1;
                    state = sqrt(step / (nx + 1e-300)) < 1e-12 ? 3 : 1;
                } else {
                    lambda *= 10;
                    state = 2;
                }
            }
            __syncthreads();
            const int st1 = state;
            __syncthreads();
            if (st1 == 2) continue;
            moved = true;
            stop = st1 == 3;
            break;
        }
        __syncthreads();
        if (!moved || stop) break;
    }
    if (threadIdx.x == 0) {
        Coef7 o = {};
        for (int k = 0; k < 3; ++k) o.c[k] = (float)xv[k];
        // Eigen::Vector3f line_dir(...).normalize(): fixed size 3, a0 + (a1 + a2), times 1 / norm
        const float u0 = (float)xv[3], u1 = (float)xv[4], u2 = (float)xv[5];
        const float r = 1.0f / sqrtf(u0 * u0 + (u1 * u1 + u2 * u2));
        o.c[3] = u0 * r;
        o.c[4] = u1 * r;
        o.c[5] = u2 * r;
        o.c[6] = (float)xv[6];
        *out = o;
    }
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
