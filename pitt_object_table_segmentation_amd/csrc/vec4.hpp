// vec4.hpp -- Eigen::Vector4f arithmetic as PCL 1.7's sample-consensus models compile it (SSE2): element-wise
// float ops, dot / squaredNorm reduced (a0 + a2) + (a1 + a3) (A3), normalize() times 1 / norm (A9),
// normalized() divided by it, cross3 with lane 3 = l3 r3 - l3 r3.  Shared by cylinder.hip and cone.hip;
// restated on the host in oracle/pitt_oracle.cpp (V4).
#pragma once
#include <hip/hip_runtime.h>

#pragma clang fp contract(off)

namespace pitt {

struct CV4 {
    float v[4];
};
__device__ __forceinline__ CV4 cv4(float a, float b, float c, float d = 0.0f) { return CV4{{a, b, c, d}}; }
__device__ __forceinline__ CV4 cadd(CV4 a, CV4 b) {
    return cv4(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2], a.v[3] + b.v[3]);
}
__device__ __forceinline__ CV4 csub(CV4 a, CV4 b) {
    return cv4(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2], a.v[3] - b.v[3]);
}
__device__ __forceinline__ CV4 cmul(float s, CV4 a) { return cv4(s * a.v[0], s * a.v[1], s * a.v[2], s * a.v[3]); }
__device__ __forceinline__ float cdot(CV4 a, CV4 b) {  // SSE2 predux: (a0 + a2) + (a1 + a3)
    return (a.v[0] * b.v[0] + a.v[2] * b.v[2]) + (a.v[1] * b.v[1] + a.v[3] * b.v[3]);
}
__device__ __forceinline__ CV4 ccross3(CV4 l, CV4 r) {
    return cv4(l.v[1] * r.v[2] - l.v[2] * r.v[1], l.v[2] * r.v[0] - l.v[0] * r.v[2], l.v[0] * r.v[1] - l.v[1] * r.v[0],
               l.v[3] * r.v[3] - l.v[3] * r.v[3]);
}
__device__ __forceinline__ CV4 cnormalize(CV4 a) {
    const float r = 1.0f / sqrtf(cdot(a, a));
    return cv4(a.v[0] * r, a.v[1] * r, a.v[2] * r, a.v[3] * r);
}
__device__ __forceinline__ CV4 cnormalized(CV4 a) {
    const float nn = sqrtf(cdot(a, a));
    return cv4(a.v[0] / nn, a.v[1] / nn, a.v[2] / nn, a.v[3] / nn);
}
__device__ __forceinline__ double csqr_pt_line(CV4 pt, CV4 lp, CV4 ld) {
    const CV4 c = ccross3(ld, csub(lp, pt));
    return (double)(cdot(c, c) / cdot(ld, ld));
}

}  // namespace pitt
