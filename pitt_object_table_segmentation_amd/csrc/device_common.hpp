// device_common.hpp -- float-exact building blocks shared by the gfx950 kernels.
//
// Every function here reproduces one PCL 1.7 / Eigen 3.2 float expression bit for bit
// (SURVEY.md Appendix A3, A4, A7, A9).  Compiled with -ffp-contract=off and IEEE division /
// sqrt (hipcc -fhip-fp32-correctly-rounded-divide-sqrt); the pragma below repeats the
// contraction ban so a build flag change cannot silently fuse a mul+add into an FMA.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace pitt {

#ifndef PITT_TILE
#define PITT_TILE 2048
#endif
constexpr int kTile = PITT_TILE;   // points per scoring tile (a divisor of PITT_TILE_POINTS)
constexpr int kBlock = 256;        // threads per tile block
constexpr int kMaxChunk = 512;     // hypotheses per score launch (LDS counters)

// A3: Eigen's 4-lane predux.  ORDER 0 = SSE2 (a0+a2)+(a1+a3), 1 = SSE3 hadd (a0+a1)+(a2+a3),
// 2 = sequential ((a0+a1)+a2)+a3.
template <int ORDER>
__device__ __forceinline__ float red4(float a0, float a1, float a2, float a3) {
    if constexpr (ORDER == 1) return (a0 + a1) + (a2 + a3);
    else if constexpr (ORDER == 2) return ((a0 + a1) + a2) + a3;
    else return (a0 + a2) + (a1 + a3);
}

// SampleConsensusModelPlane point-to-plane value: VectorXf(4).dot(Vector4f(x, y, z, 1)).
template <int ORDER>
__device__ __forceinline__ float plane_dot(float4 c, float x, float y, float z) {
    return red4<ORDER>(c.x * x, c.y * y, c.z * z, c.w);  // c.w * 1.0f == c.w exactly
}

// isSampleGood / the collinearity test of computeModelCoefficients.
__device__ __forceinline__ bool sample_good(float3 p0, float3 p1, float3 p2) {
    float rx = (p1.x - p0.x) / (p2.x - p0.x);
    float ry = (p1.y - p0.y) / (p2.y - p0.y);
    float rz = (p1.z - p0.z) / (p2.z - p0.z);
    return (rx != ry) || (rz != ry);
}

__device__ __forceinline__ float cr_sqrtf(float x) { return __builtin_sqrtf(x); }

// SampleConsensusModelPlane::computeModelCoefficients (after the collinearity test).
template <int ORDER, int DIV>
__device__ __forceinline__ float4 plane_from3(float3 p0, float3 p1, float3 p2) {
    float d1x = p1.x - p0.x, d1y = p1.y - p0.y, d1z = p1.z - p0.z;
    float d2x = p2.x - p0.x, d2y = p2.y - p0.y, d2z = p2.z - p0.z;
    float c0 = d1y * d2z - d1z * d2y;
    float c1 = d1z * d2x - d1x * d2z;
    float c2 = d1x * d2y - d1y * d2x;
    float c3 = 0.0f;
    float nrm = cr_sqrtf(red4<ORDER>(c0 * c0, c1 * c1, c2 * c2, c3 * c3));
    if constexpr (DIV == 0) {  // Eigen 3.2: v /= s  ==> v * (1/s)
        float r = 1.0f / nrm;
        c0 = c0 * r; c1 = c1 * r; c2 = c2 * r; c3 = c3 * r;
    } else {
        c0 = c0 / nrm; c1 = c1 / nrm; c2 = c2 / nrm; c3 = c3 / nrm;
    }
    float d = -1.0f * red4<ORDER>(c0 * p0.x, c1 * p0.y, c2 * p0.z, c3 * 1.0f);
    return make_float4(c0, c1, c2, d);
}

// ---- eigen33 (pcl/common/impl/eigen.hpp), float, CR trig evaluated in double (A7) ----------
__device__ __forceinline__ float std_max(float a, float b) { return (a < b) ? b : a; }

__device__ inline void compute_roots2(float b, float c, float r[3]) {
    r[0] = 0.0f;
    float d = (float)((double)(b * b) - 4.0 * (double)c);
    if (d < 0.0) d = 0.0f;
    float sd = cr_sqrtf(d);
    r[2] = 0.5f * (b + sd);
    r[1] = 0.5f * (b - sd);
}

__device__ inline void compute_roots(const float m[9], float r[3]) {
    const float m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[4], m12 = m[5], m22 = m[8];
    float c0 = m00 * m11 * m22 + 2.0f * m01 * m02 * m12 - m00 * m12 * m12 - m11 * m02 * m02 -
               m22 * m01 * m01;
    float c1 = m00 * m11 - m01 * m01 + m00 * m22 - m02 * m02 + m11 * m22 - m12 * m12;
    float c2 = m00 + m11 + m22;
    if (fabsf(c0) < 1.1920928955078125e-07f) {
        compute_roots2(c2, c1, r);
        return;
    }
    const float s_inv3 = (float)(1.0 / 3.0);
    const float s_sqrt3 = cr_sqrtf(3.0f);
    float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > 0.0f) a_over_3 = 0.0f;
    float half_b = 0.5f * (c0 + c2_over_3 * (2.0f * c2_over_3 * c2_over_3 - c1));
    float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
    if (q > 0.0f) q = 0.0f;
    float rho = cr_sqrtf(-a_over_3);
    float theta = (float)atan2((double)cr_sqrtf(-q), (double)half_b) * s_inv3;
    float cos_theta = (float)cos((double)theta);
    float sin_theta = (float)sin((double)theta);
    r[0] = c2_over_3 + 2.0f * rho * cos_theta;
    r[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
    r[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
    float t;
    if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
    if (r[1] >= r[2]) {
        t = r[1]; r[1] = r[2]; r[2] = t;
        if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
    }
    if (r[0] <= 0) compute_roots2(c2, c1, r);
}

__device__ __forceinline__ float sqnorm3(float a, float b, float c) { return a * a + (b * b + c * c); }

// Smallest eigenpair of a symmetric 3x3 (row-major), as pcl::eigen33(mat, eigenvalue, eigenvector):
// eigenvalue = roots[0] * scale.
__device__ inline void eigen33v(const float mat[9], float* value, float vec[3]) {
    float scale = 0.0f;
#pragma unroll
    for (int i = 0; i < 9; ++i) scale = std_max(scale, fabsf(mat[i]));
    if (scale <= 1.17549435082228750797e-38f) scale = 1.0f;
    float sm[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) sm[i] = mat[i] / scale;
    float r[3];
    compute_roots(sm, r);
    *value = r[0] * scale;
    sm[0] -= r[0];
    sm[4] -= r[0];
    sm[8] -= r[0];
    // rows: a = sm[0..2], b = sm[3..5], c = sm[6..8]
    float v1x = sm[1] * sm[5] - sm[2] * sm[4], v1y = sm[2] * sm[3] - sm[0] * sm[5], v1z = sm[0] * sm[4] - sm[1] * sm[3];
    float v2x = sm[1] * sm[8] - sm[2] * sm[7], v2y = sm[2] * sm[6] - sm[0] * sm[8], v2z = sm[0] * sm[7] - sm[1] * sm[6];
    float v3x = sm[4] * sm[8] - sm[5] * sm[7], v3y = sm[5] * sm[6] - sm[3] * sm[8], v3z = sm[3] * sm[7] - sm[4] * sm[6];
    float l1 = sqnorm3(v1x, v1y, v1z), l2 = sqnorm3(v2x, v2y, v2z), l3 = sqnorm3(v3x, v3y, v3z);
    float ox, oy, oz, l;
    if (l1 >= l2 && l1 >= l3) { ox = v1x; oy = v1y; oz = v1z; l = l1; }
    else if (l2 >= l1 && l2 >= l3) { ox = v2x; oy = v2y; oz = v2z; l = l2; }
    else { ox = v3x; oy = v3y; oz = v3z; l = l3; }
    float s = cr_sqrtf(l);
    vec[0] = ox / s;
    vec[1] = oy / s;
    vec[2] = oz / s;
}

// The eigenvector only (optimizeModelCoefficients).
__device__ inline void eigen33(const float mat[9], float vec[3]) {
    float v;
    eigen33v(mat, &v, vec);
}

// Block-wide exclusive scan of one int per thread (kBlock threads, 4 waves).
__device__ __forceinline__ int block_exscan(int v, int* lds4, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) lds4[w] = inc;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kBlock / 64; ++i) {
        int s = lds4[i];
        pre += (i < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return pre + inc - v;
}

}  // namespace pitt
