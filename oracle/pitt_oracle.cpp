// pitt_oracle.cpp -- CPU restatement of the reference's PCL path.  TEST INFRASTRUCTURE ONLY:
// the parity checker for the HIP path and the CPU baseline of bench.py.  Never shipped.
//
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off, no fast-math: PCL's x86-64 SSE build rounds
// every product and sum separately and keeps denormals).
//
// Reference call sites restated here (paths relative to the reference root):
//   src/segmentation_services/plane_segmentation_srv.cpp:52-67   SACSegmentationFromNormals::segment
//   src/segmentation_services/supports_segmentation_srv.cpp:89-361  support loop + helpers
//   src/segmentation_services/cluster_segmentation_srv.cpp:38-104   EuclideanClusterExtraction
// The PCL 1.7 semantics they call into (external, not in the container) are restated from the
// published PCL 1.7 algorithms, as pinned in SURVEY.md Appendix A1-A8 (+A9 below):
//   sample_consensus/impl/sac_model_plane.hpp  (isSampleGood, computeModelCoefficients,
//       countWithinDistance, selectWithinDistance, optimizeModelCoefficients)
//   sample_consensus/sac_model.h               (drawIndexSample, getSamples, rng seeding)
//   sample_consensus/impl/ransac.hpp           (RandomSampleConsensus::computeModel)
//   segmentation/impl/sac_segmentation.hpp     (segment, initSACModel fall-through A1)
//   common/impl/centroid.hpp                   (computeMeanAndCovarianceMatrix, 9 float accus)
//   common/impl/eigen.hpp                      (eigen33, computeRoots, computeRoots2)
//   segmentation/impl/extract_clusters.hpp     (extractEuclideanClusters, sorted KdTree)
// A9 (Eigen 3.2): `v /= s` on a float vector multiplies by (1/s) (SelfCwiseBinaryOp picks
// scalar_product_op with Scalar(1)/other for non-integer scalars); the binary `v / s` divides.
// Eigen >= 3.3 divides in both.  Selected by div_mode.
#include "pitt_oracle.h"
#include "eigen_lm.hpp"

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <random>
#include <unordered_map>
#include <vector>

namespace {

// ------------------------------------------------------------------------------------------
// A3: the 4-lane reduction of Eigen's vectorised redux (predux) in the PCL binary.
//   SSE2 predux: (a0 + a2) + (a1 + a3); SSE3 hadd: (a0 + a1) + (a2 + a3); scalar: sequential.
// Refinement of the sphere / cylinder / cone models (optimizeModelCoefficients): ORC_LM_PCL restates
// PCL's own Eigen::LevenbergMarquardt<NumericalDiff<Functor>, float> (eigen_lm.hpp: float, forward
// differences, stops at Eigen's sqrt(FLT_EPSILON) tolerances); ORC_LM_OPTIMUM runs a double
// Levenberg-Marquardt to the least-squares optimum of the same residual (what the device computes).
static int g_lm_mode = ORC_LM_PCL;

inline float red4(float a0, float a1, float a2, float a3, int order) {
    switch (order) {
    case ORC_REDUCE_HADD: return (a0 + a1) + (a2 + a3);
    case ORC_REDUCE_SEQ:  return ((a0 + a1) + a2) + a3;
    default:              return (a0 + a2) + (a1 + a3);
    }
}

// VectorXf(4).dot(Vector4f(x, y, z, 1)): products rounded separately (no FMA), reduced by red4.
inline float plane_dot(const float c[4], float x, float y, float z, int order) {
    return red4(c[0] * x, c[1] * y, c[2] * z, c[3] * 1.0f, order);
}

// `fabs(dot) < threshold` with threshold a double: the float is promoted (A4).
inline bool within(float d, double th) { return (double)std::fabs(d) < th; }

struct Cloud {
    const float* x;
    const float* y;
    const float* z;
    int64_t n;
};

// ------------------------------------------------------------------------------------------
// A2: SampleConsensusModel<PointT> sampler.  rng_alg_ = boost::mt19937 seeded 12345 (random_ ==
// false), rnd() = uniform_int<>(0, INT_MAX)(mt) which for a 32-bit engine is mt() >> 1
// (bucket_size 2).  shuffled_indices_ = 0..N-1, rebuilt on every segment() (the model object is
// re-created by initSACModel).
struct Sampler {
    std::mt19937 mt;
    std::vector<int> shuffled;
    explicit Sampler(int64_t n, uint32_t seed) : mt(seed), shuffled((size_t)n) {
        std::iota(shuffled.begin(), shuffled.end(), 0);
    }
    int rnd() { return (int)(mt() >> 1); }
    // drawIndexSample: for i < 3: swap(s[i], s[i + rnd() % (N - i)]); sample = s[0..2].
    void draw(int out[3]) {
        size_t N = shuffled.size();
        for (unsigned i = 0; i < 3; ++i)
            std::swap(shuffled[i], shuffled[i + ((size_t)rnd() % (N - i))]);
        out[0] = shuffled[0];
        out[1] = shuffled[1];
        out[2] = shuffled[2];
    }
};

// SampleConsensusModelPlane::isSampleGood: dy1dy2 = (p1-p0)/(p2-p0) (Array4f, componentwise);
// good iff (dy1dy2[0] != dy1dy2[1]) || (dy1dy2[2] != dy1dy2[1])  (NaN => good).
bool sample_good(const Cloud& c, const int s[3]) {
    float d1x = c.x[s[1]] - c.x[s[0]], d1y = c.y[s[1]] - c.y[s[0]], d1z = c.z[s[1]] - c.z[s[0]];
    float d2x = c.x[s[2]] - c.x[s[0]], d2y = c.y[s[2]] - c.y[s[0]], d2z = c.z[s[2]] - c.z[s[0]];
    float rx = d1x / d2x, ry = d1y / d2y, rz = d1z / d2z;
    return (rx != ry) || (rz != ry);
}

// SampleConsensusModelPlane::computeModelCoefficients.
bool plane_from3(const float p0[3], const float p1[3], const float p2[3], int order, int div_mode,
                 float out[4]) {
    float d1x = p1[0] - p0[0], d1y = p1[1] - p0[1], d1z = p1[2] - p0[2];
    float d2x = p2[0] - p0[0], d2y = p2[1] - p0[1], d2z = p2[2] - p0[2];
    float rx = d1x / d2x, ry = d1y / d2y, rz = d1z / d2z;
    if ((rx == ry) && (rz == ry)) return false;  // collinear
    float c[4];
    c[0] = d1y * d2z - d1z * d2y;
    c[1] = d1z * d2x - d1x * d2z;
    c[2] = d1x * d2y - d1y * d2x;
    c[3] = 0.0f;
    // model_coefficients.normalize(): *this /= norm(); norm() = sqrt(squaredNorm()) with the
    // squaredNorm reduced by predux (dynamic-size VectorXf of size 4).
    float nrm = std::sqrt(red4(c[0] * c[0], c[1] * c[1], c[2] * c[2], c[3] * c[3], order));
    if (div_mode == ORC_DIV_EIGEN32) {
        float r = 1.0f / nrm;
        for (int i = 0; i < 4; ++i) c[i] = c[i] * r;
    } else {
        for (int i = 0; i < 4; ++i) c[i] = c[i] / nrm;
    }
    // model_coefficients[3] = -1 * head<4>().dot(p0) with p0 = (x, y, z, 1) and c[3] == 0.
    c[3] = -1.0f * red4(c[0] * p0[0], c[1] * p0[1], c[2] * p0[2], c[3] * 1.0f, order);
    std::memcpy(out, c, sizeof c);
    return true;
}

bool plane_from_samples(const Cloud& cl, const int s[3], int order, int div_mode, float out[4]) {
    float p0[3] = {cl.x[s[0]], cl.y[s[0]], cl.z[s[0]]};
    float p1[3] = {cl.x[s[1]], cl.y[s[1]], cl.z[s[1]]};
    float p2[3] = {cl.x[s[2]], cl.y[s[2]], cl.z[s[2]]};
    return plane_from3(p0, p1, p2, order, div_mode, out);
}

int64_t count_within(const Cloud& c, const float coef[4], double th, int order) {
    int64_t nr = 0;
    for (int64_t i = 0; i < c.n; ++i)
        if (within(plane_dot(coef, c.x[i], c.y[i], c.z[i], order), th)) ++nr;
    return nr;
}

void select_within(const Cloud& c, const float coef[4], double th, int order,
                   std::vector<int>& out) {
    out.clear();
    for (int64_t i = 0; i < c.n; ++i)
        if (within(plane_dot(coef, c.x[i], c.y[i], c.z[i], order), th)) out.push_back((int)i);
}

// ------------------------------------------------------------------------------------------
// A7: pcl::computeRoots2 / computeRoots / eigen33 (common/impl/eigen.hpp), float Scalar.
float trig_atan2(float y, float x, int mode) {
    return mode == ORC_TRIG_LIBM ? atan2f(y, x) : (float)std::atan2((double)y, (double)x);
}
float trig_cos(float t, int mode) { return mode == ORC_TRIG_LIBM ? cosf(t) : (float)std::cos((double)t); }
float trig_sin(float t, int mode) { return mode == ORC_TRIG_LIBM ? sinf(t) : (float)std::sin((double)t); }

void compute_roots2(float b, float c, float roots[3]) {
    roots[0] = 0.0f;
    float d = (float)((double)(b * b) - 4.0 * (double)c);  // Scalar(b * b - 4.0 * c)
    if (d < 0.0) d = 0.0f;
    float sd = std::sqrt(d);
    roots[2] = 0.5f * (b + sd);
    roots[1] = 0.5f * (b - sd);
}

// m is row-major 3x3 (symmetric).
void compute_roots(const float m[9], float roots[3], int trig) {
    const float m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[4], m12 = m[5], m22 = m[8];
    float c0 = m00 * m11 * m22 + 2.0f * m01 * m02 * m12 - m00 * m12 * m12 - m11 * m02 * m02 -
               m22 * m01 * m01;
    float c1 = m00 * m11 - m01 * m01 + m00 * m22 - m02 * m02 + m11 * m22 - m12 * m12;
    float c2 = m00 + m11 + m22;
    if (std::fabs(c0) < std::numeric_limits<float>::epsilon()) {
        compute_roots2(c2, c1, roots);
        return;
    }
    const float s_inv3 = (float)(1.0 / 3.0);
    const float s_sqrt3 = std::sqrt(3.0f);
    float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > 0.0f) a_over_3 = 0.0f;
    float half_b = 0.5f * (c0 + c2_over_3 * (2.0f * c2_over_3 * c2_over_3 - c1));
    float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
    if (q > 0.0f) q = 0.0f;
    float rho = std::sqrt(-a_over_3);
    float theta = trig_atan2(std::sqrt(-q), half_b, trig) * s_inv3;
    float cos_theta = trig_cos(theta, trig);
    float sin_theta = trig_sin(theta, trig);
    roots[0] = c2_over_3 + 2.0f * rho * cos_theta;
    roots[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
    roots[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
    if (roots[0] >= roots[1]) std::swap(roots[0], roots[1]);
    if (roots[1] >= roots[2]) {
        std::swap(roots[1], roots[2]);
        if (roots[0] >= roots[1]) std::swap(roots[0], roots[1]);
    }
    if (roots[0] <= 0) compute_roots2(c2, c1, roots);
}

// Vector3f squaredNorm: fixed size 3 is not packet-vectorised, so Eigen's unrolled redux is
// a0 + (a1 + a2).
inline float sqnorm3(const float v[3]) { return v[0] * v[0] + (v[1] * v[1] + v[2] * v[2]); }
inline void cross3(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

void eigen33(const float mat[9], int trig, float* eigenvalue, float vec[3]) {
    float scale = 0.0f;
    for (int i = 0; i < 9; ++i) scale = std::max(scale, std::fabs(mat[i]));
    if (scale <= std::numeric_limits<float>::min()) scale = 1.0f;
    float sm[9];
    for (int i = 0; i < 9; ++i) sm[i] = mat[i] / scale;  // binary `mat / scale`: divides
    float roots[3];
    compute_roots(sm, roots, trig);
    *eigenvalue = roots[0] * scale;
    sm[0] -= roots[0];
    sm[4] -= roots[0];
    sm[8] -= roots[0];
    float v1[3], v2[3], v3[3];
    cross3(&sm[0], &sm[3], v1);
    cross3(&sm[0], &sm[6], v2);
    cross3(&sm[3], &sm[6], v3);
    float l1 = sqnorm3(v1), l2 = sqnorm3(v2), l3 = sqnorm3(v3);
    const float* v;
    float l;
    if (l1 >= l2 && l1 >= l3) { v = v1; l = l1; }
    else if (l2 >= l1 && l2 >= l3) { v = v2; l = l2; }
    else { v = v3; l = l3; }
    float s = std::sqrt(l);
    for (int i = 0; i < 3; ++i) vec[i] = v[i] / s;  // binary `vec / sqrt(len)`: divides
}

// SampleConsensusModelPlane::optimizeModelCoefficients (PCL 1.7):
// < 4 inliers => unchanged; else computeMeanAndCovarianceMatrix (9 float accumulators, sequential
// in inlier order, `accu /= n`), eigen33, d = -1 * (e, 0).dot(centroid).
void optimize(const Cloud& c, const int* inl, int64_t n_inl, const float coef[4],
              const orc_sac_params& p, float out[4]) {
    if (n_inl < 4) {
        std::memcpy(out, coef, 4 * sizeof(float));
        return;
    }
    float a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t k = 0; k < n_inl; ++k) {
        const float x = c.x[inl[k]], y = c.y[inl[k]], z = c.z[inl[k]];
        a[0] += x * x;
        a[1] += x * y;
        a[2] += x * z;
        a[3] += y * y;
        a[4] += y * z;
        a[5] += z * z;
        a[6] += x;
        a[7] += y;
        a[8] += z;
    }
    const float fn = (float)n_inl;
    if (p.div_mode == ORC_DIV_EIGEN32) {
        const float r = 1.0f / fn;
        for (int i = 0; i < 9; ++i) a[i] = a[i] * r;
    } else {
        for (int i = 0; i < 9; ++i) a[i] = a[i] / fn;
    }
    float cov[9];
    cov[0] = a[0] - a[6] * a[6];
    cov[1] = a[1] - a[6] * a[7];
    cov[2] = a[2] - a[6] * a[8];
    cov[4] = a[3] - a[7] * a[7];
    cov[5] = a[4] - a[7] * a[8];
    cov[8] = a[5] - a[8] * a[8];
    cov[3] = cov[1];
    cov[6] = cov[2];
    cov[7] = cov[5];
    float ev, e[3];
    eigen33(cov, p.trig_mode, &ev, e);
    float r[4] = {e[0], e[1], e[2], 0.0f};
    r[3] = -1.0f * red4(r[0] * a[6], r[1] * a[7], r[2] * a[8], r[3] * 1.0f, p.reduce_order);
    std::memcpy(out, r, sizeof r);
}

// ------------------------------------------------------------------------------------------
// RandomSampleConsensus::computeModel + SACSegmentation::segment (A5).
struct SegmentOut {
    bool ok = false;
    float coef[4] = {0, 0, 0, 0};
    float best[4] = {0, 0, 0, 0};
    int hypotheses = 0, best_h = -1, rejected = 0;
    int64_t best_count = 0;
    std::vector<int> inliers;
    std::vector<int> counts;
};

SegmentOut segment(const Cloud& c, const orc_sac_params& p) {
    SegmentOut o;
    if (c.n < 3) return o;  // getSamples: "Can not select 3 unique points" => empty model
    Sampler smp(c.n, p.seed);
    int iterations = 0;
    int n_best = -std::numeric_limits<int>::max();
    double k = 1.0;
    const double log_probability = std::log(1.0 - p.probability);
    const double one_over_indices = 1.0 / (double)c.n;
    unsigned skipped = 0;
    const unsigned max_skip = (unsigned)p.max_iterations * 10u;
    bool have_model = false;
    int s[3];
    while (iterations < k && skipped < max_skip) {
        // getSamples: up to max_sample_checks_ (1000) draws until isSampleGood
        bool got = false;
        for (int chk = 0; chk < 1000; ++chk) {
            smp.draw(s);
            if (sample_good(c, s)) { got = true; break; }
            ++o.rejected;
        }
        if (!got) break;  // "No samples could be selected!"
        float coef[4];
        if (!plane_from_samples(c, s, p.reduce_order, p.div_mode, coef)) {
            ++skipped;
            continue;
        }
        int n_in = (int)count_within(c, coef, p.threshold, p.reduce_order);
        o.counts.push_back(n_in);
        if (n_in > n_best) {
            n_best = n_in;
            have_model = true;
            std::memcpy(o.best, coef, sizeof coef);
            o.best_h = iterations;
            double w = (double)n_best * one_over_indices;
            double p_no_outliers = 1.0 - std::pow(w, 3.0);
            p_no_outliers = std::max(std::numeric_limits<double>::epsilon(), p_no_outliers);
            p_no_outliers = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no_outliers);
            k = log_probability / std::log(p_no_outliers);
        }
        ++iterations;
        if (iterations > p.max_iterations) break;
    }
    o.hypotheses = iterations;
    if (!have_model) return o;
    o.best_count = n_best;
    std::vector<int> inl;
    select_within(c, o.best, p.threshold, p.reduce_order, inl);
    if (p.optimize) {
        optimize(c, inl.data(), (int64_t)inl.size(), o.best, p, o.coef);
        select_within(c, o.coef, p.threshold, p.reduce_order, inl);
    } else {
        std::memcpy(o.coef, o.best, sizeof o.coef);
    }
    o.inliers.swap(inl);
    o.ok = true;
    return o;
}

// ------------------------------------------------------------------------------------------
// Support segmentation (supports_segmentation_srv.cpp).
struct SupportOut {
    std::vector<int> idx_map;
    float coef[4];
    std::vector<float> sx, sy, sz;  // support_cloud
    std::vector<float> ox, oy, oz;  // on_support_cloud
};

}  // namespace

struct orc_support_list {
    std::vector<SupportOut> s;
};

struct orc_cluster_list {
    std::vector<std::vector<int>> idx;
    std::vector<std::array<float, 3>> centroid;
};

namespace {

// isHorizontalPlane :161-179 (float, open intervals).
bool is_horizontal(const float c[4], const float axis[3], float var_th) {
    float div = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    float nx = c[0] / div, ny = c[1] / div, nz = c[2] / div;
    float cx = ny * axis[2] - nz * axis[1];
    float cy = nz * axis[0] - nx * axis[2];
    float cz = nx * axis[1] - ny * axis[0];
    float lo = -1 * var_th, hi = var_th;
    return (cx > lo && cx < hi) && (cy > lo && cy < hi) && (cz > lo && cz < hi);
}

// createNewIdxMap :139-157 with valueBelongsToArray :131-136 as a membership bitmask.
std::vector<int> new_idx_map(const std::vector<int>& prev, const std::vector<int>& inl, int level,
                             int64_t n) {
    std::vector<uint8_t> member((size_t)n, 0);
    for (int v : inl) member[(size_t)v] = 1;
    std::vector<int> out(prev.size());
    int cnt = 0;
    for (size_t p = 0; p < prev.size(); ++p) {
        int v = prev[p];
        if (v > level && v < 0) out[p] = v;
        else if (v >= 0 && v < n && member[(size_t)v]) out[p] = level;
        else out[p] = cnt++;
    }
    return out;
}

}  // namespace

extern "C" {

void orc_mt19937(uint32_t seed, int64_t n, uint32_t* out) {
    std::mt19937 mt(seed);
    for (int64_t i = 0; i < n; ++i) out[i] = (uint32_t)mt();
}

void orc_sampler_table(int64_t n, uint32_t seed, int64_t attempts, int32_t* out) {
    Sampler smp(n, seed);
    int s[3];
    for (int64_t a = 0; a < attempts; ++a) {
        smp.draw(s);
        out[3 * a] = s[0];
        out[3 * a + 1] = s[1];
        out[3 * a + 2] = s[2];
    }
}

int orc_plane_coefficients(const float p0[3], const float p1[3], const float p2[3],
                           int32_t reduce_order, int32_t div_mode, float out[4]) {
    return plane_from3(p0, p1, p2, reduce_order, div_mode, out) ? 1 : 0;
}

int64_t orc_count_within(const float* x, const float* y, const float* z, int64_t n,
                         const float coeff[4], double threshold, int32_t reduce_order) {
    Cloud c{x, y, z, n};
    return count_within(c, coeff, threshold, reduce_order);
}

int64_t orc_select_within(const float* x, const float* y, const float* z, int64_t n,
                          const float coeff[4], double threshold, int32_t reduce_order,
                          int32_t* out) {
    Cloud c{x, y, z, n};
    std::vector<int> v;
    select_within(c, coeff, threshold, reduce_order, v);
    if (out) std::memcpy(out, v.data(), v.size() * sizeof(int));
    return (int64_t)v.size();
}

int orc_eigen33(const float cov[9], int32_t trig_mode, int32_t div_mode, float* eigenvalue,
                float vec[3]) {
    (void)div_mode;
    eigen33(cov, trig_mode, eigenvalue, vec);
    return 0;
}

int orc_optimize_plane(const float* x, const float* y, const float* z, const int32_t* inliers,
                       int64_t n_inliers, const float coeff[4], const orc_sac_params* p,
                       float out[4]) {
    Cloud c{x, y, z, 0};
    optimize(c, inliers, n_inliers, coeff, *p, out);
    return 0;
}

int orc_plane_segment(const float* x, const float* y, const float* z, int64_t n,
                      const orc_sac_params* p, int32_t* inliers_out, orc_plane_result* res,
                      int32_t* hyp_counts) {
    Cloud c{x, y, z, n};
    SegmentOut o = segment(c, *p);
    std::memset(res, 0, sizeof *res);
    res->hypotheses = o.hypotheses;
    res->best_hypothesis = o.best_h;
    res->rejected_samples = o.rejected;
    res->best_count = o.best_count;
    std::memcpy(res->best_coefficients, o.best, sizeof o.best);
    if (hyp_counts)
        std::memcpy(hyp_counts, o.counts.data(), o.counts.size() * sizeof(int));
    if (!o.ok) return 1;  // PCL: inliers.indices.clear(); model_coefficients.values.clear()
    res->n_coeff = 4;
    std::memcpy(res->coefficients, o.coef, sizeof o.coef);
    res->n_inliers = (int64_t)o.inliers.size();
    if (inliers_out) std::memcpy(inliers_out, o.inliers.data(), o.inliers.size() * sizeof(int));
    return 0;
}

// findSupports :241-361.
orc_support_list* orc_find_supports(const float* x, const float* y, const float* z, int64_t n,
                                    const orc_support_params* sp) {
    orc_support_list* L = new orc_support_list;
    orc_sac_params p;
    p.threshold = (double)sp->ransac_distance_threshold;
    p.max_iterations = sp->ransac_max_iterations;
    p.probability = 0.99;
    p.seed = 12345u;
    p.optimize = 1;
    p.reduce_order = sp->reduce_order;
    p.trig_mode = sp->trig_mode;
    p.div_mode = sp->div_mode;

    std::vector<float> ix(x, x + n), iy(y, y + n), iz(z, z + n);  // iterativeCloud
    std::vector<int> prev_map;
    int level = -2, cnt = 0;
    const float nf = (float)n;
    while (true) {
        Cloud ic{ix.data(), iy.data(), iz.data(), (int64_t)ix.size()};
        SegmentOut o = segment(ic, p);
        const std::vector<int>& inl = o.inliers;
        if (inl.empty()) break;
        if ((float)ix.size() < nf * sp->min_iterative_cloud_percentage) break;
        if ((float)inl.size() < nf * sp->min_iterative_plane_percentage) break;

        std::vector<int> inliers_idx;
        if (!cnt) {
            inliers_idx.resize((size_t)n);
            std::iota(inliers_idx.begin(), inliers_idx.end(), 0);
        } else {
            inliers_idx = prev_map;
        }
        // removePlaneInliner :114-127: positive extract (inlier order), then negative in place.
        SupportOut so;
        so.sx.reserve(inl.size());
        for (int i : inl) {
            so.sx.push_back(ix[i]);
            so.sy.push_back(iy[i]);
            so.sz.push_back(iz[i]);
        }
        {
            std::vector<uint8_t> rm(ix.size(), 0);
            for (int i : inl) rm[(size_t)i] = 1;
            size_t w = 0;
            for (size_t r = 0; r < ix.size(); ++r)
                if (!rm[r]) { ix[w] = ix[r]; iy[w] = iy[r]; iz[w] = iz[r]; ++w; }
            ix.resize(w); iy.resize(w); iz.resize(w);
        }
        if (is_horizontal(o.coef, sp->horizontal_axis, sp->horizontal_variance_threshold)) {
            std::vector<int> nm = new_idx_map(inliers_idx, inl, level, n);
            // getPointOnPlane :187-238 (double bbox with the `else if`, double z sum).
            const double inf = std::numeric_limits<double>::infinity();
            double xMax = -inf, yMax = -inf, zMed = 0, xMin = inf, yMin = inf;
            for (size_t i = 0; i < so.sx.size(); ++i) {
                if (so.sx[i] > xMax) xMax = so.sx[i];
                else if (so.sx[i] < xMin) xMin = so.sx[i];
                if (so.sy[i] > yMax) yMax = so.sy[i];
                else if (so.sy[i] < yMin) yMin = so.sy[i];
                zMed += so.sz[i];
            }
            xMax -= sp->edge_remove_offset[0];
            xMin += sp->edge_remove_offset[0];
            yMax -= sp->edge_remove_offset[1];
            yMin += sp->edge_remove_offset[1];
            zMed = zMed / (double)so.sx.size() + sp->edge_remove_offset[2];
            for (int64_t i = 0; i < n; ++i) {
                if (nm[(size_t)i] == level) continue;  // removingIdx membership
                if (x[i] > xMin && x[i] < xMax && z[i] > zMed && y[i] > yMin && y[i] < yMax) {
                    so.ox.push_back(x[i]);
                    so.oy.push_back(y[i]);
                    so.oz.push_back(z[i]);
                }
            }
            std::memcpy(so.coef, o.coef, sizeof so.coef);
            so.idx_map = nm;
            prev_map.swap(nm);
            L->s.push_back(std::move(so));
        } else {
            prev_map = new_idx_map(inliers_idx, inl, -1, n);
        }
        ++cnt;
        --level;
    }
    return L;
}

int32_t orc_support_count(const orc_support_list* L) { return (int32_t)L->s.size(); }

int orc_support_get(const orc_support_list* L, int32_t s, int32_t* idx_map, float coeff[4],
                    int64_t* n_support, int64_t* n_on_support) {
    if (s < 0 || s >= (int32_t)L->s.size()) return -1;
    const SupportOut& so = L->s[(size_t)s];
    if (idx_map) std::memcpy(idx_map, so.idx_map.data(), so.idx_map.size() * sizeof(int));
    if (coeff) std::memcpy(coeff, so.coef, sizeof so.coef);
    if (n_support) *n_support = (int64_t)so.sx.size();
    if (n_on_support) *n_on_support = (int64_t)so.ox.size();
    return 0;
}

int orc_support_cloud(const orc_support_list* L, int32_t s, int32_t which, float* x, float* y,
                      float* z) {
    if (s < 0 || s >= (int32_t)L->s.size()) return -1;
    const SupportOut& so = L->s[(size_t)s];
    const std::vector<float>& a = which ? so.ox : so.sx;
    const std::vector<float>& b = which ? so.oy : so.sy;
    const std::vector<float>& c = which ? so.oz : so.sz;
    std::memcpy(x, a.data(), a.size() * sizeof(float));
    std::memcpy(y, b.data(), b.size() * sizeof(float));
    std::memcpy(z, c.data(), c.size() * sizeof(float));
    return 0;
}

void orc_support_free(orc_support_list* L) { delete L; }

// clusterize :38-108 + extractEuclideanClusters (A8).
orc_cluster_list* orc_euclidean_clusters(const float* x, const float* y, const float* z, int64_t n,
                                         double tolerance, double min_rate, double max_rate,
                                         int32_t min_input_size) {
    orc_cluster_list* L = new orc_cluster_list;
    if (n < (int64_t)min_input_size) return L;  // :54
    const unsigned min_pts = (unsigned)(int)std::round((double)n * min_rate);  // :64
    const unsigned max_pts = (unsigned)(int)std::round((double)n * max_rate);  // :65
    // extract(): tolerance -> float; KdTreeFLANN::radiusSearch: r2 = (float)((double)tol^2).
    const float tol_f = (float)tolerance;
    const float r2 = (float)((double)tol_f * (double)tol_f);
    // Uniform grid (cell slightly above the radius) for candidate generation; the predicate is
    // FLANN L2_Simple: ((dx*dx + dy*dy) + dz*dz) < r2 in float.
    double cell = (double)tol_f * 1.01;
    double mnx = 1e300, mny = 1e300, mnz = 1e300;
    auto finite = [&](int64_t i) { return std::isfinite(x[i]) && std::isfinite(y[i]) && std::isfinite(z[i]); };
    for (int64_t i = 0; i < n; ++i) {
        if (!finite(i)) continue;
        mnx = std::min(mnx, (double)x[i]);
        mny = std::min(mny, (double)y[i]);
        mnz = std::min(mnz, (double)z[i]);
    }
    auto key = [&](int64_t gx, int64_t gy, int64_t gz) {
        return (uint64_t)((gx & 0x1FFFFF) | ((gy & 0x1FFFFF) << 21) | ((gz & 0x1FFFFF) << 42));
    };
    std::unordered_map<uint64_t, std::vector<int>> grid;
    std::vector<int64_t> gxs((size_t)n), gys((size_t)n), gzs((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        if (!finite(i)) continue;  // no radius neighbours (NaN distances): a singleton
        gxs[i] = (int64_t)std::floor(((double)x[i] - mnx) / cell);
        gys[i] = (int64_t)std::floor(((double)y[i] - mny) / cell);
        gzs[i] = (int64_t)std::floor(((double)z[i] - mnz) / cell);
        grid[key(gxs[i], gys[i], gzs[i])].push_back((int)i);
    }
    std::vector<uint8_t> processed((size_t)n, 0);
    std::vector<std::pair<float, int>> nn;
    std::vector<std::vector<int>> clusters;
    for (int64_t i = 0; i < n; ++i) {
        if (processed[i]) continue;
        std::vector<int> q;
        size_t sq = 0;
        q.push_back((int)i);
        processed[i] = 1;
        while (sq < q.size()) {
            const int qi = q[sq];
            nn.clear();
            if (!finite(qi)) { ++sq; continue; }
            for (int dx = -1; dx <= 1; ++dx)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dz = -1; dz <= 1; ++dz) {
                        auto it = grid.find(key(gxs[qi] + dx, gys[qi] + dy, gzs[qi] + dz));
                        if (it == grid.end()) continue;
                        for (int j : it->second) {
                            float ex = x[qi] - x[j], ey = y[qi] - y[j], ez = z[qi] - z[j];
                            float d = ex * ex + ey * ey + ez * ez;
                            if (d < r2) nn.emplace_back(d, j);
                        }
                    }
            std::sort(nn.begin(), nn.end());  // sorted results (search::KdTree sorted_ = true)
            for (size_t j = 1; j < nn.size(); ++j) {  // nn_start_idx = 1
                const int id = nn[j].second;
                if (processed[id]) continue;
                q.push_back(id);
                processed[id] = 1;
            }
            ++sq;
        }
        if (q.size() >= min_pts && q.size() <= max_pts) {
            std::sort(q.begin(), q.end());
            q.erase(std::unique(q.begin(), q.end()), q.end());
            clusters.push_back(std::move(q));
        }
    }
    // EuclideanClusterExtraction::extract: std::sort(rbegin, rend, size <)
    std::sort(clusters.rbegin(), clusters.rend(),
              [](const std::vector<int>& a, const std::vector<int>& b) { return a.size() < b.size(); });
    for (auto& c : clusters) {
        float sx = 0, sy = 0, sz = 0;
        int cnt = 1;  // Q7: the handler starts its counter at 1
        for (int id : c) {
            sx += x[id];
            sy += y[id];
            sz += z[id];
            cnt++;
        }
        L->centroid.push_back({sx / cnt, sy / cnt, sz / cnt});
        L->idx.push_back(std::move(c));
    }
    return L;
}

int32_t orc_cluster_count(const orc_cluster_list* L) { return (int32_t)L->idx.size(); }
int64_t orc_cluster_size(const orc_cluster_list* L, int32_t c) {
    return (c < 0 || c >= (int32_t)L->idx.size()) ? -1 : (int64_t)L->idx[(size_t)c].size();
}
int orc_cluster_get(const orc_cluster_list* L, int32_t c, int32_t* idx, float centroid[3]) {
    if (c < 0 || c >= (int32_t)L->idx.size()) return -1;
    const auto& v = L->idx[(size_t)c];
    if (idx) std::memcpy(idx, v.data(), v.size() * sizeof(int));
    if (centroid) std::memcpy(centroid, L->centroid[(size_t)c].data(), 3 * sizeof(float));
    return 0;
}
void orc_cluster_free(orc_cluster_list* L) { delete L; }

// --- preprocessing in front of findSupports ---------------------------------
// srv_manager.h:163-167 getServiceFloatParameter: a request value >= 0 is used, anything else
// (the -1 sentinel, NaN) selects the default.
float orc_service_float_param(float input, float default_value) { return input >= 0.0f ? input : default_value; }

// deep_filter_srv.cpp:37-44 deepFiltering: points with z == z (not NaN) split at z > th into
// "further", else "closer", each in input order.  Either output may be NULL (counted only).
int orc_deep_filter(const float* x, const float* y, const float* z, int64_t n, float th, float* cx, float* cy,
                    float* cz, int64_t* n_closer, float* fx, float* fy, float* fz, int64_t* n_further) {
    int64_t nc = 0, nf = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!(z[i] == z[i])) continue;
        if (z[i] > th) {
            if (fx) { fx[nf] = x[i]; fy[nf] = y[i]; fz[nf] = z[i]; }
            ++nf;
        } else {
            if (cx) { cx[nc] = x[i]; cy[nc] = y[i]; cz[nc] = z[i]; }
            ++nc;
        }
    }
    if (n_closer) *n_closer = nc;
    if (n_further) *n_further = nf;
    return 0;
}

// fromROSMsg of the XYZ fields as called by PCManager::cloudForRosMsg (pc_manager.cpp:94-104):
// point r * width + c is read at byte r * row_step + c * point_step (little-endian host).
int orc_unpack_pointcloud2(const uint8_t* data, int32_t width, int32_t height, int32_t point_step, int64_t row_step,
                           int32_t off_x, int32_t off_y, int32_t off_z, float* x, float* y, float* z) {
    for (int64_t r = 0; r < height; ++r)
        for (int64_t c = 0; c < width; ++c) {
            const uint8_t* p = data + r * row_step + c * point_step;
            const int64_t i = r * width + c;
            std::memcpy(&x[i], p + off_x, 4);
            std::memcpy(&y[i], p + off_y, 4);
            std::memcpy(&z[i], p + off_z, 4);
        }
    return 0;
}

// pcl::transformPointCloud(cloud, out, Eigen::Matrix4f) as called at obj_segmentation.cpp:248
// (PCL 1.7 common/impl/transforms.hpp, absent here): the Matrix4f becomes an Affine3f and every
// point is  out.k = m(k,0) * x + m(k,1) * y + m(k,2) * z + m(k,3)  evaluated left to right in
// float, no FMA (the x86 build).  A non-dense cloud (is_dense == false) copies every point first
// and transforms only the points whose x, y and z are all finite.  m: row-major 4x4.
int orc_transform_cloud(const float* x, const float* y, const float* z, int64_t n, const float m[16], int32_t dense,
                        float* ox, float* oy, float* oz) {
    for (int64_t i = 0; i < n; ++i) {
        const float px = x[i], py = y[i], pz = z[i];
        if (!dense && !(std::isfinite(px) && std::isfinite(py) && std::isfinite(pz))) {
            ox[i] = px;
            oy[i] = py;
            oz[i] = pz;
            continue;
        }
        ox[i] = m[0] * px + m[1] * py + m[2] * pz + m[3];
        oy[i] = m[4] * px + m[5] * py + m[6] * pz + m[7];
        oz[i] = m[8] * px + m[9] * py + m[10] * pz + m[11];
    }
    return 0;
}

// pcl::VoxelGrid<PointXYZ>::applyFilter (PCL 1.7 filters/impl/voxel_grid.hpp, absent here) as used by
// PCManager::downSampling (pc_manager.cpp:61-67, leaf 0.01 m from :19; called at
// obj_segmentation.cpp:238).  Defaults: no filter field, downsample_all_data_ = true (x, y, z are the
// PointXYZ fields), min_points_per_voxel_ = 0.
//   * getMinMax3D over the finite points (Array4f min/max in float);
//   * dx = (int64)((max - min) * inv) + 1 per axis, inv = 1.0f / leaf; dx*dy*dz > INT32_MAX: the
//     filter warns and outputs the input cloud unchanged (return 1);
//   * min_b = (int)floor(min * inv); div_b = max_b - min_b + 1; divb_mul = (1, div_b0, div_b0*div_b1);
//   * per finite point (in input order): ijk = (int)(floor(p * inv) - (float)min_b),
//     idx = ijk0 + ijk1 * divb_mul1 + ijk2 * divb_mul2;
//   * std::sort of (idx, point index) pairs by idx only -- NOT stable: the order inside a voxel is
//     libstdc++'s introsort permutation (this build's libstdc++; assumption A10).  sort_mode 1 uses
//     std::stable_sort instead (ascending point index inside a voxel);
//   * per voxel, ascending idx: centroid = first point, += the others in sorted order (float),
//     then `centroid /= n` -- Eigen 3.2 multiplies by 1.0f / n (A9).
// Non-finite points never enter (the is_dense == false path; a dense cloud has none).
struct VoxPair {
    uint32_t idx, cloud_point_index;
    bool operator<(const VoxPair& o) const { return idx < o.idx; }
};

int orc_voxel_grid(const float* x, const float* y, const float* z, int64_t n, float lx, float ly, float lz,
                   int32_t sort_mode, float* ox, float* oy, float* oz, int64_t* n_out) {
    const float inv[3] = {1.0f / lx, 1.0f / ly, 1.0f / lz};
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    const float* c[3] = {x, y, z};
    int64_t finite = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!(std::isfinite(x[i]) && std::isfinite(y[i]) && std::isfinite(z[i]))) continue;
        ++finite;
        for (int k = 0; k < 3; ++k) {
            mn[k] = c[k][i] < mn[k] ? c[k][i] : mn[k];  // Eigen cwiseMin: std::min(a, b)
            mx[k] = mx[k] < c[k][i] ? c[k][i] : mx[k];
        }
    }
    *n_out = 0;
    if (finite == 0) return 0;
    int64_t d[3];
    for (int k = 0; k < 3; ++k) d[k] = (int64_t)((mx[k] - mn[k]) * inv[k]) + 1;
    if (d[0] * d[1] * d[2] > (int64_t)INT32_MAX) {
        for (int64_t i = 0; i < n; ++i) {
            ox[i] = x[i];
            oy[i] = y[i];
            oz[i] = z[i];
        }
        *n_out = n;
        return 1;
    }
    int min_b[3], max_b[3], div_b[3];
    for (int k = 0; k < 3; ++k) {
        min_b[k] = (int)std::floor(mn[k] * inv[k]);
        max_b[k] = (int)std::floor(mx[k] * inv[k]);
        div_b[k] = max_b[k] - min_b[k] + 1;
    }
    const int mul[3] = {1, div_b[0], div_b[0] * div_b[1]};
    std::vector<VoxPair> v;
    v.reserve((size_t)finite);
    for (int64_t i = 0; i < n; ++i) {
        if (!(std::isfinite(x[i]) && std::isfinite(y[i]) && std::isfinite(z[i]))) continue;
        int idx = 0;
        for (int k = 0; k < 3; ++k) idx += (int)(std::floor(c[k][i] * inv[k]) - (float)min_b[k]) * mul[k];
        v.push_back({(uint32_t)idx, (uint32_t)i});
    }
    if (sort_mode == 1) std::stable_sort(v.begin(), v.end());
    else std::sort(v.begin(), v.end());
    int64_t out = 0;
    for (size_t a = 0; a < v.size();) {
        size_t b = a + 1;
        while (b < v.size() && v[b].idx == v[a].idx) ++b;
        float s[3] = {x[v[a].cloud_point_index], y[v[a].cloud_point_index], z[v[a].cloud_point_index]};
        for (size_t j = a + 1; j < b; ++j) {
            s[0] += x[v[j].cloud_point_index];
            s[1] += y[v[j].cloud_point_index];
            s[2] += z[v[j].cloud_point_index];
        }
        const float r = 1.0f / (float)(b - a);
        ox[out] = s[0] * r;
        oy[out] = s[1] * r;
        oz[out] = s[2] * r;
        ++out;
        a = b;
    }
    *n_out = out;
    return 0;
}

// pcl::NormalEstimation<PointXYZ, Normal>::compute with a search::KdTree and setKSearch(k), as
// PCManager::estimateNormal (pc_manager.cpp:68-78, k = 50 from :18; called at obj_segmentation.cpp:253
// and ransac_segmentation.cpp:233).  PCL 1.7 features/impl/normal_3d.hpp + feature.h:
//   * neighbours: KdTreeFLANN::nearestKSearch(point, k) -- exact (eps 0), k clamped to the number of
//     indexed (finite) points, results ascending by FLANN's L2_Simple float distance
//     ((dx*dx + dy*dy) + dz*dz, dx = query - point); equal distances in ascending point index here
//     (FLANN keeps its traversal order: assumption A11, exact ties only between duplicate points);
//   * computePointNormal: < 3 neighbours -> NaN; else computeMeanAndCovarianceMatrix over the
//     neighbours in that order (the nine float accumulators, `accu /= n` as x * (1/n), A6/A9), then
//     solvePlaneParameters: eigen33 -> (nx, ny, nz), curvature = |l_min / (c00 + c11 + c22)| (0 when
//     the trace is 0);
//   * flipNormalTowardsViewpoint: (vp - p) . n = ((vx*nx + vy*ny) + vz*nz) < 0 -> negate;
//   * a non-finite query point (is_dense == false) gets NaN normal and curvature.
// Exact kNN by rings of a uniform grid (the ring is grown until the k-th distance is certainly
// below the distance of every point outside it).
int orc_normal_estimation(const float* x, const float* y, const float* z, int64_t n, int32_t k, const float vp[3],
                          float* nx, float* ny, float* nz, float* curv, int32_t* nn_out, int32_t* nn_cnt) {
    const float qnan = std::numeric_limits<float>::quiet_NaN();
    auto fin = [&](int64_t i) { return std::isfinite(x[i]) && std::isfinite(y[i]) && std::isfinite(z[i]); };
    std::vector<int32_t> pts;
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    for (int64_t i = 0; i < n; ++i) {
        if (!fin(i)) continue;
        pts.push_back((int32_t)i);
        const double p[3] = {x[i], y[i], z[i]};
        for (int a = 0; a < 3; ++a) {
            mn[a] = std::min(mn[a], p[a]);
            mx[a] = std::max(mx[a], p[a]);
        }
    }
    const int64_t nf = (int64_t)pts.size();
    const int kk = (int)std::min<int64_t>(k, nf);
    double h = 0.05;
    if (nf > 0) {  // ~16 points per occupied cell on a surface-like cloud
        double ext = std::max(mx[0] - mn[0], std::max(mx[1] - mn[1], mx[2] - mn[2]));
        h = std::max(ext / 64.0, 1e-6);
        for (int it = 0; it < 2; ++it) {
            std::unordered_map<uint64_t, int> occ;
            for (int32_t i : pts) {
                const int64_t c[3] = {(int64_t)((x[i] - mn[0]) / h), (int64_t)((y[i] - mn[1]) / h),
                                      (int64_t)((z[i] - mn[2]) / h)};
                ++occ[(uint64_t)c[0] | ((uint64_t)c[1] << 21) | ((uint64_t)c[2] << 42)];
            }
            const double per = (double)nf / (double)occ.size();
            h = std::max(h * std::sqrt(16.0 / per), 1e-6);
        }
    }
    int64_t dim[3];
    for (int a = 0; a < 3; ++a) dim[a] = nf ? (int64_t)((mx[a] - mn[a]) / h) + 1 : 1;
    std::unordered_map<uint64_t, std::vector<int32_t>> grid;
    auto key = [](int64_t a, int64_t b, int64_t c) { return (uint64_t)a | ((uint64_t)b << 21) | ((uint64_t)c << 42); };
    std::vector<int64_t> cell((size_t)n * 3, 0);
    for (int32_t i : pts) {
        cell[3 * i] = (int64_t)((x[i] - mn[0]) / h);
        cell[3 * i + 1] = (int64_t)((y[i] - mn[1]) / h);
        cell[3 * i + 2] = (int64_t)((z[i] - mn[2]) / h);
        grid[key(cell[3 * i], cell[3 * i + 1], cell[3 * i + 2])].push_back(i);
    }
    const int64_t rmax = std::max(dim[0], std::max(dim[1], dim[2]));
    std::vector<std::pair<float, int32_t>> cand;
    for (int64_t q = 0; q < n; ++q) {
        if (nn_cnt) nn_cnt[q] = 0;
        if (!fin(q) || kk < 3) {  // no normal: no neighbour list is summed (count 0)
            nx[q] = ny[q] = nz[q] = curv[q] = qnan;
            continue;
        }
        for (int64_t r = 1;; ++r) {
            cand.clear();
            for (int64_t a = cell[3 * q] - r; a <= cell[3 * q] + r; ++a)
                for (int64_t b = cell[3 * q + 1] - r; b <= cell[3 * q + 1] + r; ++b)
                    for (int64_t c = cell[3 * q + 2] - r; c <= cell[3 * q + 2] + r; ++c) {
                        if (a < 0 || b < 0 || c < 0 || a >= dim[0] || b >= dim[1] || c >= dim[2]) continue;
                        auto it = grid.find(key(a, b, c));
                        if (it == grid.end()) continue;
                        for (int32_t j : it->second) {
                            const float dx = x[q] - x[j], dy = y[q] - y[j], dz = z[q] - z[j];
                            cand.emplace_back(dx * dx + dy * dy + dz * dz, j);
                        }
                    }
            if ((int)cand.size() < kk && r < rmax) continue;
            std::partial_sort(cand.begin(), cand.begin() + kk, cand.end());
            const double lim = (double)r * h;
            if (r >= rmax || (double)cand[(size_t)kk - 1].first <= lim * lim * (1.0 - 1e-5)) break;
        }
        float a9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int t = 0; t < kk; ++t) {
            const int32_t j = cand[(size_t)t].second;
            if (nn_out) nn_out[(size_t)q * k + t] = j;
            const float px = x[j], py = y[j], pz = z[j];
            a9[0] += px * px;
            a9[1] += px * py;
            a9[2] += px * pz;
            a9[3] += py * py;
            a9[4] += py * pz;
            a9[5] += pz * pz;
            a9[6] += px;
            a9[7] += py;
            a9[8] += pz;
        }
        if (nn_cnt) nn_cnt[q] = kk;
        const float rcp = 1.0f / (float)kk;
        for (int t = 0; t < 9; ++t) a9[t] = a9[t] * rcp;
        float cov[9];
        cov[0] = a9[0] - a9[6] * a9[6];
        cov[1] = a9[1] - a9[6] * a9[7];
        cov[2] = a9[2] - a9[6] * a9[8];
        cov[4] = a9[3] - a9[7] * a9[7];
        cov[5] = a9[4] - a9[7] * a9[8];
        cov[8] = a9[5] - a9[8] * a9[8];
        cov[3] = cov[1];
        cov[6] = cov[2];
        cov[7] = cov[5];
        float ev, e[3];
        eigen33(cov, ORC_TRIG_CR, &ev, e);
        const float tr = cov[0] + cov[4] + cov[8];
        curv[q] = tr != 0.0f ? std::fabs(ev / tr) : 0.0f;
        const float vx = vp[0] - x[q], vy = vp[1] - y[q], vz = vp[2] - z[q];
        const float ct = vx * e[0] + vy * e[1] + vz * e[2];
        if (ct < 0) {
            e[0] *= -1.0f;
            e[1] *= -1.0f;
            e[2] *= -1.0f;
        }
        nx[q] = e[0];
        ny[q] = e[1];
        nz[q] = e[2];
    }
    return 0;
}

}  // extern "C"

// The permutation std::sort gives (key, value) pairs compared by key (VoxelGrid's index_vector), twice:
// orc_std_sort_pairs runs this image's libstdc++ std::sort; orc_introsort_pairs restates libstdc++'s
// algorithm (introsort loop with median-of-3 to first and the unguarded Hoare partition, heapsort
// when the depth limit runs out, final insertion sort) with a settable depth limit (< 0: the
// library's 2 floor(log2 n)), so the tests can check the restatement against the library and the
// device emulation against the restatement -- including the heapsort fallback.
namespace {
struct KV {
    uint32_t k, v;
};
inline bool kv_less(const KV& a, const KV& b) { return a.k < b.k; }

void is_push_heap(KV* a, long hole, long top, KV value) {
    long parent = (hole - 1) / 2;
    while (hole > top && kv_less(a[parent], value)) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = value;
}
void is_adjust_heap(KV* a, long hole, long len, KV value) {
    const long top = hole;
    long second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (kv_less(a[second], a[second - 1])) second--;
        a[hole] = a[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a[hole] = a[second - 1];
        hole = second - 1;
    }
    is_push_heap(a, hole, top, value);
}
void is_heap_sort(KV* a, long len) {
    if (len >= 2)
        for (long parent = (len - 2) / 2;; --parent) {
            is_adjust_heap(a, parent, len, a[parent]);
            if (parent == 0) break;
        }
    for (long last = len; last > 1;) {
        --last;
        KV value = a[last];
        a[last] = a[0];
        is_adjust_heap(a, 0, last, value);
    }
}
void is_loop(KV* a, long first, long last, int depth) {
    while (last - first > 16) {
        if (depth == 0) {
            is_heap_sort(a + first, last - first);
            return;
        }
        --depth;
        const long mid = first + (last - first) / 2, x = first + 1, y = mid, z = last - 1;
        long m;
        if (kv_less(a[x], a[y])) m = kv_less(a[y], a[z]) ? y : kv_less(a[x], a[z]) ? z : x;
        else m = kv_less(a[x], a[z]) ? x : kv_less(a[y], a[z]) ? z : y;
        std::swap(a[first], a[m]);
        long lo = first + 1, hi = last;
        while (true) {
            while (kv_less(a[lo], a[first])) ++lo;
            --hi;
            while (kv_less(a[first], a[hi])) --hi;
            if (!(lo < hi)) break;
            std::swap(a[lo], a[hi]);
            ++lo;
        }
        is_loop(a, lo, last, depth);
        last = lo;
    }
}
void is_insertion(KV* a, long n) {  // __insertion_sort: stable for equal keys
    for (long i = 1; i < n; ++i) {
        KV v = a[i];
        long j = i;
        while (j > 0 && kv_less(v, a[j - 1])) {
            a[j] = a[j - 1];
            --j;
        }
        a[j] = v;
    }
}
}  // namespace

extern "C" {
void orc_std_sort_pairs(uint32_t* key, uint32_t* val, int64_t n) {
    std::vector<KV> a((size_t)n);
    for (int64_t i = 0; i < n; ++i) a[(size_t)i] = {key[i], val[i]};
    std::sort(a.begin(), a.end(), kv_less);
    for (int64_t i = 0; i < n; ++i) key[i] = a[(size_t)i].k, val[i] = a[(size_t)i].v;
}

void orc_partial_sort_pairs(uint32_t* key, uint32_t* val, int64_t n) {  // the library's heapsort path
    std::vector<KV> a((size_t)n);
    for (int64_t i = 0; i < n; ++i) a[(size_t)i] = {key[i], val[i]};
    std::partial_sort(a.begin(), a.end(), a.end(), kv_less);
    for (int64_t i = 0; i < n; ++i) key[i] = a[(size_t)i].k, val[i] = a[(size_t)i].v;
}

void orc_introsort_pairs(uint32_t* key, uint32_t* val, int64_t n, int32_t depth_limit) {
    std::vector<KV> a((size_t)n);
    for (int64_t i = 0; i < n; ++i) a[(size_t)i] = {key[i], val[i]};
    if (n > 1) {
        int lg = 0;
        while (((int64_t)2 << lg) <= n) ++lg;
        is_loop(a.data(), 0, (long)n, depth_limit >= 0 ? depth_limit : 2 * lg);
        is_insertion(a.data(), (long)n);
    }
    for (int64_t i = 0; i < n; ++i) key[i] = a[(size_t)i].k, val[i] = a[(size_t)i].v;
}

// cylinder_segmentation_srv.cpp:53-79 (getNormalizeAxesDirectionVector, getPointOnAxes,
// getVectorBetweenPoints) and :129-178; cone_segmentation_srv.cpp:129-178 differs only in the centroid.
// Every operation is a float operation in source order (x86-64 SSE, no FMA); sqrt of a float is the
// correctly rounded float sqrt (std::sqrt(float), or the double sqrt rounded to float: the same value).
void orc_axis_height(const float* x, const float* y, const float* z, int64_t n, const float coef[6], int32_t mode,
                     float* px, float* py, float* pz, float* height, int32_t* idx1, int32_t* idx2,
                     float centroid[3]) {
    const float norm = std::sqrt(coef[3] * coef[3] + coef[4] * coef[4] + coef[5] * coef[5]);
    const float dx = coef[3] / norm, dy = coef[4] / norm, dz = coef[5] / norm;
    const float a1x = coef[0] + dx * -1.0f, a1y = coef[1] + dy * -1.0f, a1z = coef[2] + dz * -1.0f;
    const float a2x = coef[0] + dx * 1.0f, a2y = coef[1] + dy * 1.0f, a2z = coef[2] + dz * 1.0f;
    const float ux = a2x - a1x, uy = a2y - a1y, uz = a2z - a1z;
    const float gdiv = ux * ux + uy * uy + uz * uz;
    std::vector<float> qx((size_t)n), qy((size_t)n), qz((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        const float vx = x[i] - a1x, vy = y[i] - a1y, vz = z[i] - a1z;
        const float g = (vx * ux + vy * uy + vz * uz) / gdiv;
        qx[(size_t)i] = a1x + g * ux;
        qy[(size_t)i] = a1y + g * uy;
        qz[(size_t)i] = a1z + g * uz;
    }
    float h = -1.0f;
    int32_t b1 = -1, b2 = -1;
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t j = 0; j < i; ++j) {  // the reference's j loop, i > j
            const float ex = qx[(size_t)i] - qx[(size_t)j], ey = qy[(size_t)i] - qy[(size_t)j],
                        ez = qz[(size_t)i] - qz[(size_t)j];
            const float d = std::sqrt(ex * ex + ey * ey + ez * ez);
            if (d > h) {
                h = d;
                b1 = (int32_t)i;
                b2 = (int32_t)j;
            }
        }
    }
    *height = h;
    *idx1 = b1;
    *idx2 = b2;
    if (mode == 0) {  // cylinder: the midpoint of the pair (no pair: the reference reads points[-1])
        const float nan = std::numeric_limits<float>::quiet_NaN();
        centroid[0] = b1 < 0 ? nan : (qx[(size_t)b1] + qx[(size_t)b2]) / 2;
        centroid[1] = b1 < 0 ? nan : (qy[(size_t)b1] + qy[(size_t)b2]) / 2;
        centroid[2] = b1 < 0 ? nan : (qz[(size_t)b1] + qz[(size_t)b2]) / 2;
    } else {  // cone: apex + 3/4 of the height along the axis
        centroid[0] = coef[0] + 3.0f / 4.0f * h * dx;
        centroid[1] = coef[1] + 3.0f / 4.0f * h * dy;
        centroid[2] = coef[2] + 3.0f / 4.0f * h * dz;
    }
    if (px)
        for (int64_t i = 0; i < n; ++i) px[i] = qx[(size_t)i], py[i] = qy[(size_t)i], pz[i] = qz[(size_t)i];
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// Sphere (PCL 1.7 sample_consensus/impl/sac_model_sphere.hpp; the RANSAC loop as segment() above).
namespace {
// Eigen 3.2 determinant_impl<4>: Costabel's 30-multiplication expansion, terms left to right.
inline float det4_helper(const float m[16], int j, int k, int a, int b) {
    return (m[j * 4 + 0] * m[k * 4 + 1] - m[k * 4 + 0] * m[j * 4 + 1]) *
           (m[a * 4 + 2] * m[b * 4 + 3] - m[b * 4 + 2] * m[a * 4 + 3]);
}
inline float det4(const float m[16]) {
    return det4_helper(m, 0, 1, 2, 3) - det4_helper(m, 0, 2, 1, 3) + det4_helper(m, 0, 3, 1, 2) +
           det4_helper(m, 1, 2, 0, 3) - det4_helper(m, 1, 3, 0, 2) + det4_helper(m, 2, 3, 0, 1);
}

// computeModelCoefficients: Cramer's rule on the 4 x 4 system, temp's columns permuted in place.
bool sphere_from4(const float px[4], const float py[4], const float pz[4], float c[4]) {
    float t[16];
    for (int i = 0; i < 4; ++i) t[i * 4 + 0] = px[i], t[i * 4 + 1] = py[i], t[i * 4 + 2] = pz[i], t[i * 4 + 3] = 1;
    const float m11 = det4(t);
    if (m11 == 0) return false;  // the points don't define a sphere
    for (int i = 0; i < 4; ++i) t[i * 4 + 0] = px[i] * px[i] + py[i] * py[i] + pz[i] * pz[i];
    const float m12 = det4(t);
    for (int i = 0; i < 4; ++i) t[i * 4 + 1] = t[i * 4 + 0], t[i * 4 + 0] = px[i];
    const float m13 = det4(t);
    for (int i = 0; i < 4; ++i) t[i * 4 + 2] = t[i * 4 + 1], t[i * 4 + 1] = py[i];
    const float m14 = det4(t);
    for (int i = 0; i < 4; ++i)
        t[i * 4 + 0] = t[i * 4 + 2], t[i * 4 + 1] = px[i], t[i * 4 + 2] = py[i], t[i * 4 + 3] = pz[i];
    const float m15 = det4(t);
    c[0] = 0.5f * m12 / m11;
    c[1] = 0.5f * m13 / m11;
    c[2] = 0.5f * m14 / m11;
    c[3] = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2] - m15 / m11);
    return true;
}

// isModelValid: the radius limits (set by setRadiusLimits; -DBL_MAX / DBL_MAX = unset)
bool sphere_valid(const float c[4], double rmin, double rmax) {
    if (rmin != -DBL_MAX && c[3] < rmin) return false;
    if (rmax != DBL_MAX && c[3] > rmax) return false;
    return true;
}

// |sqrtf((x - c0)^2 + (y - c1)^2 + (z - c2)^2) - c3| < threshold (float promoted to double, A4)
inline bool sphere_in(const Cloud& c, int64_t i, const float m[4], double th) {
    const float dx = c.x[i] - m[0], dy = c.y[i] - m[1], dz = c.z[i] - m[2];
    return std::fabs(std::sqrt(dx * dx + dy * dy + dz * dz) - m[3]) < th;
}

// Levenberg-Marquardt in double over the inliers' residuals ||p - c|| - r (the same iteration the
// library's host loop runs on device sums, pitt_sphere_segment).
elm::Result pcl_lm_sphere(const float* x, const float* y, const float* z, const int32_t* inl, int64_t m, float c[4]);

void sphere_refine(const Cloud& c, const std::vector<int>& inl, const float in[4], float out[4]) {
    if (g_lm_mode == ORC_LM_PCL) {
        for (int k = 0; k < 4; ++k) out[k] = in[k];
        pcl_lm_sphere(c.x, c.y, c.z, inl.data(), (int64_t)inl.size(), out);
        return;
    }
    double x[4] = {in[0], in[1], in[2], in[3]};
    auto sums = [&](const double* v, double* jtj, double* jtr, double* cost) {
        for (int i = 0; i < 10; ++i) jtj[i] = 0;
        for (int i = 0; i < 4; ++i) jtr[i] = 0;
        *cost = 0;
        for (int id : inl) {
            const double dx = (double)c.x[id] - v[0], dy = (double)c.y[id] - v[1], dz = (double)c.z[id] - v[2];
            const double d = std::sqrt(dx * dx + dy * dy + dz * dz);
            const double r = d - v[3];
            const double j[4] = {d > 0 ? -dx / d : 0.0, d > 0 ? -dy / d : 0.0, d > 0 ? -dz / d : 0.0, -1.0};
            int q = 0;
            for (int a = 0; a < 4; ++a)
                for (int b = a; b < 4; ++b) jtj[q++] += j[a] * j[b];
            for (int a = 0; a < 4; ++a) jtr[a] += j[a] * r;
            *cost += r * r;
        }
    };
    double jtj[10], jtr[4], cost;
    sums(x, jtj, jtr, &cost);
    double lambda = 1e-3;
    for (int it = 0; it < 100; ++it) {
        bool moved = false;
        double step = 0;
        while (lambda < 1e10) {
            double A[4][5];
            int q = 0;
            for (int a = 0; a < 4; ++a)
                for (int b = a; b < 4; ++b) A[a][b] = A[b][a] = jtj[q++];
            for (int a = 0; a < 4; ++a) A[a][a] += lambda * A[a][a], A[a][4] = -jtr[a];
            // Gaussian elimination with partial pivoting on the 4 x 4 system
            bool ok = true;
            for (int col = 0; col < 4 && ok; ++col) {
                int piv = col;
                for (int r = col + 1; r < 4; ++r)
                    if (std::fabs(A[r][col]) > std::fabs(A[piv][col])) piv = r;
                if (A[piv][col] == 0) { ok = false; break; }
                if (piv != col)
                    for (int k = 0; k < 5; ++k) std::swap(A[col][k], A[piv][k]);
                for (int r = col + 1; r < 4; ++r) {
                    const double f = A[r][col] / A[col][col];
                    for (int k = col; k < 5; ++k) A[r][k] -= f * A[col][k];
                }
            }
            if (!ok) break;
            double dlt[4];
            for (int r = 3; r >= 0; --r) {
                double acc = A[r][4];
                for (int k = r + 1; k < 4; ++k) acc -= A[r][k] * dlt[k];
                dlt[r] = acc / A[r][r];
            }
            double xn[4], jn[10], rn[4], cn;
            for (int a = 0; a < 4; ++a) xn[a] = x[a] + dlt[a];
            sums(xn, jn, rn, &cn);
            if (cn < cost) {
                step = 0;
                double nx = 0;
                for (int a = 0; a < 4; ++a) step += dlt[a] * dlt[a], nx += xn[a] * xn[a];
                step = std::sqrt(step / (nx + 1e-300));
                for (int a = 0; a < 4; ++a) x[a] = xn[a];
                std::memcpy(jtj, jn, sizeof jtj);
                std::memcpy(jtr, rn, sizeof jtr);
                cost = cn;
                lambda *= 0.1;
                moved = true;
                break;
            }
            // rejected: a step already below 1e-10 relative cannot change the float result -- stop
            // (instead of raising the damping to 1e10 through the summation noise)
            double rs = 0, rx = 0;
            for (int a = 0; a < 4; ++a) rs += dlt[a] * dlt[a], rx += xn[a] * xn[a];
            if (std::sqrt(rs / (rx + 1e-300)) < 1e-10) break;
            lambda *= 10;
        }
        if (!moved || step < 1e-10) break;
    }
    for (int a = 0; a < 4; ++a) out[a] = (float)x[a];
}
}  // namespace

extern "C" {
int orc_sphere_from4(const float xyz[12], float coef[4]) {
    const float px[4] = {xyz[0], xyz[3], xyz[6], xyz[9]}, py[4] = {xyz[1], xyz[4], xyz[7], xyz[10]},
                pz[4] = {xyz[2], xyz[5], xyz[8], xyz[11]};
    return sphere_from4(px, py, pz, coef) ? 1 : 0;
}

int orc_sphere_segment(const float* x, const float* y, const float* z, int64_t n, const orc_sphere_params* p,
                       int32_t* inliers, int64_t* n_inliers, float coef[4], float best_out[4], int32_t* hypotheses,
                       int32_t* counts, int32_t counts_cap, int32_t* n_counts) {
    Cloud c{x, y, z, n};
    *n_inliers = 0;
    *hypotheses = 0;
    if (n_counts) *n_counts = 0;
    if (n < 4) return 0;  // getSamples: "Can not select 4 unique points"
    std::mt19937 mt(p->seed);
    std::vector<int> sh((size_t)n);
    std::iota(sh.begin(), sh.end(), 0);
    int iterations = 0, n_best = -std::numeric_limits<int>::max();
    double k = 1.0;
    const double log_probability = std::log(1.0 - p->probability);
    const double one_over_indices = 1.0 / (double)n;
    unsigned skipped = 0;
    const unsigned max_skip = (unsigned)p->max_iterations * 10u;
    bool have = false;
    float best[4] = {0, 0, 0, 0};
    int nc = 0;
    while (iterations < k && skipped < max_skip) {
        // getSamples: SampleConsensusModelSphere::isSampleGood accepts every sample
        for (unsigned i = 0; i < 4; ++i)
            std::swap(sh[i], sh[i + ((size_t)(mt() >> 1) % ((size_t)n - i))]);
        const float px[4] = {x[sh[0]], x[sh[1]], x[sh[2]], x[sh[3]]}, py[4] = {y[sh[0]], y[sh[1]], y[sh[2]], y[sh[3]]},
                    pz[4] = {z[sh[0]], z[sh[1]], z[sh[2]], z[sh[3]]};
        float m[4];
        if (!sphere_from4(px, py, pz, m)) {
            ++skipped;
            continue;
        }
        int n_in = 0;
        if (sphere_valid(m, p->radius_min, p->radius_max))  // countWithinDistance: 0 for an invalid model
            for (int64_t i = 0; i < n; ++i) n_in += sphere_in(c, i, m, p->threshold);
        if (counts && nc < counts_cap) counts[nc] = n_in;
        ++nc;
        if (n_in > n_best) {
            n_best = n_in;
            have = true;
            std::memcpy(best, m, sizeof m);
            const double w = (double)n_best * one_over_indices;
            double p_no = 1.0 - std::pow(w, 4.0);
            p_no = std::max(std::numeric_limits<double>::epsilon(), p_no);
            p_no = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no);
            k = log_probability / std::log(p_no);
        }
        ++iterations;
        if (iterations > p->max_iterations) break;
    }
    *hypotheses = iterations;
    if (n_counts) *n_counts = nc;
    if (!have) return 0;
    std::memcpy(best_out, best, sizeof best);
    std::vector<int> inl;
    auto select = [&](const float* m) {
        inl.clear();
        if (!sphere_valid(m, p->radius_min, p->radius_max)) return;  // selectWithinDistance: none
        for (int64_t i = 0; i < n; ++i)
            if (sphere_in(c, i, m, p->threshold)) inl.push_back((int)i);
    };
    select(best);
    float out[4];
    std::memcpy(out, best, sizeof out);
    if (p->optimize && inl.size() > 4) {  // optimizeModelCoefficients needs more than 4 inliers
        sphere_refine(c, inl, best, out);
        select(out);
    } else if (p->optimize) {
        select(out);
    }
    std::memcpy(coef, out, sizeof out);
    for (size_t i = 0; i < inl.size(); ++i) inliers[i] = inl[i];
    *n_inliers = (int64_t)inl.size();
    return 1;
}
}  // extern "C"

// ------------------------------------------------------------------------------------------
// Cylinder (PCL 1.7 sample_consensus/impl/sac_model_cylinder.hpp, common/distances.h, common.hpp).
// Eigen::Vector4f arithmetic: element-wise float ops, dot / squaredNorm reduced in SSE2 order (A3),
// normalize() multiplies by 1 / norm (A9), normalized() divides by it.
namespace {
struct V4 {
    float v[4];
};
inline V4 v4(float a, float b, float c, float d = 0.0f) { return V4{{a, b, c, d}}; }
inline V4 add(V4 a, V4 b) { return v4(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2], a.v[3] + b.v[3]); }
inline V4 sub(V4 a, V4 b) { return v4(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2], a.v[3] - b.v[3]); }
inline V4 mul(float s, V4 a) { return v4(s * a.v[0], s * a.v[1], s * a.v[2], s * a.v[3]); }
inline float dot(V4 a, V4 b) { return red4(a.v[0] * b.v[0], a.v[1] * b.v[1], a.v[2] * b.v[2], a.v[3] * b.v[3], 0); }
inline V4 cross3(V4 l, V4 r) {  // Eigen's SSE cross3: lane 3 = l3 r3 - l3 r3
    return v4(l.v[1] * r.v[2] - l.v[2] * r.v[1], l.v[2] * r.v[0] - l.v[0] * r.v[2], l.v[0] * r.v[1] - l.v[1] * r.v[0],
              l.v[3] * r.v[3] - l.v[3] * r.v[3]);
}
inline V4 normalize(V4 a) {  // *this /= norm(): times 1 / norm (A9)
    const float r = 1.0f / std::sqrt(dot(a, a));
    return v4(a.v[0] * r, a.v[1] * r, a.v[2] * r, a.v[3] * r);
}
inline V4 normalized(V4 a) {  // *this / norm()
    const float nn = std::sqrt(dot(a, a));
    return v4(a.v[0] / nn, a.v[1] / nn, a.v[2] / nn, a.v[3] / nn);
}
// sqrPointToLineDistance: |line_dir x (line_pt - pt)|^2 / |line_dir|^2 (float quotient, as double)
inline double sqr_pt_line(V4 pt, V4 lp, V4 ld) {
    const V4 c = cross3(ld, sub(lp, pt));
    return (double)(dot(c, c) / dot(ld, ld));
}
// getAngle3D: acos of the clamped dot of the normalized vectors (double)
inline double angle3d(V4 a, V4 b) {
    double rad = dot(normalized(a), normalized(b));
    if (rad < -1.0) rad = -1.0;
    else if (rad > 1.0) rad = 1.0;
    return std::acos(rad);
}

bool cyl_from2(const float* x, const float* y, const float* z, const float* nx, const float* ny, const float* nz,
               const int s[2], double rmin, double rmax, float c[7]) {
    const int a = s[0], b = s[1];
    const float eps = std::numeric_limits<float>::epsilon();
    if (std::fabs(x[a] - x[b]) <= eps && std::fabs(y[a] - y[b]) <= eps && std::fabs(z[a] - z[b]) <= eps) return false;
    const V4 p1 = v4(x[a], y[a], z[a]), p2 = v4(x[b], y[b], z[b]);
    const V4 n1 = v4(nx[a], ny[a], nz[a]), n2 = v4(nx[b], ny[b], nz[b]);
    const V4 w = sub(add(n1, p1), p2);
    const float A = dot(n1, n1), B = dot(n1, n2), C = dot(n2, n2), D = dot(n1, w), E = dot(n2, w);
    const float den = A * C - B * B;
    float sc, tc;
    if (den < 1e-8) {
        sc = 0.0f;
        tc = (B > C ? D / B : E / C);
    } else {
        sc = (B * E - C * D) / den;
        tc = (A * E - B * D) / den;
    }
    const V4 lp = add(add(p1, n1), mul(sc, n1));
    const V4 ld = normalize(sub(add(p2, mul(tc, n2)), lp));
    for (int k = 0; k < 3; ++k) c[k] = lp.v[k], c[3 + k] = ld.v[k];
    c[6] = (float)std::sqrt(sqr_pt_line(p1, lp, ld));
    if (c[6] > rmax || c[6] < rmin) return false;
    return true;
}

bool cyl_valid(const float c[7], double rmin, double rmax) {
    if (rmin != -DBL_MAX && c[6] < rmin) return false;
    if (rmax != DBL_MAX && c[6] > rmax) return false;
    return true;
}

inline double angle3d_e(V4 a, V4 b, int eigen33);

inline bool cyl_in(const float* x, const float* y, const float* z, const float* nx, const float* ny, const float* nz,
                   int64_t i, const float c[7], double w, double th, int eigen33) {
    const V4 lp = v4(c[0], c[1], c[2]), ld = v4(c[3], c[4], c[5]);
    const float ptdotdir = dot(lp, ld), dirdotdir = 1.0f / dot(ld, ld);
    const V4 pt = v4(x[i], y[i], z[i]), nn = v4(nx[i], ny[i], nz[i]);
    const double d_euclid = std::fabs(std::sqrt(sqr_pt_line(pt, lp, ld)) - (double)c[6]);
    const float k = (dot(pt, ld) - ptdotdir) * dirdotdir;
    const V4 proj = add(lp, mul(k, ld));
    const V4 dir = normalize(sub(pt, proj));
    double d_normal = std::fabs(angle3d_e(nn, dir, eigen33));
    d_normal = std::min(d_normal, M_PI - d_normal);
    return std::fabs(w * d_normal + (1 - w) * d_euclid) < th;
}

// f = |u x (c - p)|^2 / |u|^2 - r^2 and its gradient in (c, u, r)
inline void cyl_residual(const double* v, float px, float py, float pz, double J[7], double* f) {
    const double vx = v[0] - px, vy = v[1] - py, vz = v[2] - pz;  // c - p
    const double ux = v[3], uy = v[4], uz = v[5];
    const double wx = uy * vz - uz * vy, wy = uz * vx - ux * vz, wz = ux * vy - uy * vx;  // u x v
    const double s = ux * ux + uy * uy + uz * uz, w2 = wx * wx + wy * wy + wz * wz;
    *f = w2 / s - v[6] * v[6];
    // d|w|^2/dv = 2 (w x u); d|w|^2/du = 2 (v x w)
    J[0] = 2.0 * (wy * uz - wz * uy) / s;
    J[1] = 2.0 * (wz * ux - wx * uz) / s;
    J[2] = 2.0 * (wx * uy - wy * ux) / s;
    J[3] = 2.0 * (vy * wz - vz * wy) / s - 2.0 * w2 * ux / (s * s);
    J[4] = 2.0 * (vz * wx - vx * wz) / s - 2.0 * w2 * uy / (s * s);
    J[5] = 2.0 * (vx * wy - vy * wx) / s - 2.0 * w2 * uz / (s * s);
    J[6] = -2.0 * v[6];
}

// Levenberg-Marquardt (Marquardt damping lambda * diag, x10 / x0.1) over N parameters; sums(v, jtj
// (upper triangle, row major), jtr, cost).  Stops when no damping lowers the cost, or an accepted or
// rejected step is below 1e-10 relative (below the float coefficients' resolution; past it the damping
// would only climb through the summation noise).
template <int N, class Sums>
void lm_solve(double* x, Sums sums) {
    double jtj[N * (N + 1) / 2], jtr[N], cost;
    sums(x, jtj, jtr, &cost);
    double lambda = 1e-3;
    for (int it = 0; it < 200; ++it) {
        bool moved = false;
        double step = 0;
        while (lambda < 1e10) {
            double M[N][N + 1];
            int t = 0;
            for (int a = 0; a < N; ++a)
                for (int b = a; b < N; ++b) M[a][b] = M[b][a] = jtj[t++];
            for (int a = 0; a < N; ++a) M[a][a] += lambda * M[a][a] + 1e-30, M[a][N] = -jtr[a];
            bool ok = true;
            for (int col = 0; col < N && ok; ++col) {
                int piv = col;
                for (int r = col + 1; r < N; ++r)
                    if (std::fabs(M[r][col]) > std::fabs(M[piv][col])) piv = r;
                if (M[piv][col] == 0) { ok = false; break; }
                if (piv != col)
                    for (int k = 0; k <= N; ++k) std::swap(M[col][k], M[piv][k]);
                for (int r = col + 1; r < N; ++r) {
                    const double f = M[r][col] / M[col][col];
                    for (int k = col; k <= N; ++k) M[r][k] -= f * M[col][k];
                }
            }
            if (!ok) break;
            double dl[N];
            for (int r = N - 1; r >= 0; --r) {
                double acc = M[r][N];
                for (int k = r + 1; k < N; ++k) acc -= M[r][k] * dl[k];
                dl[r] = acc / M[r][r];
            }
            double xn[N], jn[N * (N + 1) / 2], rn[N], cn;
            for (int a = 0; a < N; ++a) xn[a] = x[a] + dl[a];
            sums(xn, jn, rn, &cn);
            if (cn < cost) {
                double nx = 0;
                for (int a = 0; a < N; ++a) step += dl[a] * dl[a], nx += xn[a] * xn[a];
                step = std::sqrt(step / (nx + 1e-300));
                for (int a = 0; a < N; ++a) x[a] = xn[a];
                std::memcpy(jtj, jn, sizeof jtj);
                std::memcpy(jtr, rn, sizeof jtr);
                cost = cn;
                lambda *= 0.1;
                moved = true;
                break;
            }
            // rejected: a step already below 1e-10 relative cannot change the float result -- stop
            double rs = 0, rx = 0;
            for (int a = 0; a < N; ++a) rs += dl[a] * dl[a], rx += xn[a] * xn[a];
            if (std::sqrt(rs / (rx + 1e-300)) < 1e-10) break;
            lambda *= 10;
        }
        if (!moved || step < 1e-10) break;
    }
}

// Levenberg-Marquardt in double on f_i = |u x (c - p_i)|^2 / |u|^2 - r^2 (OptimizationFunctor's
// residual), parameters (c, u, r); then u normalised.
elm::Result pcl_lm_cylinder(const float* x, const float* y, const float* z, const int32_t* inl, int64_t m,
                            float c[7]);

void cyl_refine(const float* x, const float* y, const float* z, const std::vector<int>& inl, const float in[7],
                float out[7]) {
    double q[7];
    for (int k = 0; k < 7; ++k) q[k] = in[k];
    if (g_lm_mode == ORC_LM_PCL) {
        float c[7];
        for (int k = 0; k < 7; ++k) c[k] = in[k];
        if (!inl.empty()) pcl_lm_cylinder(x, y, z, inl.data(), (int64_t)inl.size(), c);
        for (int k = 0; k < 7; ++k) q[k] = c[k];
    }
    auto sums = [&](const double* v, double* jtj /*28*/, double* jtr /*7*/, double* cost) {
        for (int k = 0; k < 28; ++k) jtj[k] = 0;
        for (int k = 0; k < 7; ++k) jtr[k] = 0;
        *cost = 0;
        for (int id : inl) {
            double J[7], f;
            cyl_residual(v, x[id], y[id], z[id], J, &f);
            int t = 0;
            for (int a = 0; a < 7; ++a)
                for (int b = a; b < 7; ++b) jtj[t++] += J[a] * J[b];
            for (int a = 0; a < 7; ++a) jtr[a] += J[a] * f;
            *cost += f * f;
        }
    };
    if (g_lm_mode != ORC_LM_PCL && inl.size() >= 7) lm_solve<7>(q, sums);  // Eigen's LM refuses m < n
    const double nu = std::sqrt(q[3] * q[3] + q[4] * q[4] + q[5] * q[5]);
    for (int k = 0; k < 3; ++k) out[k] = (float)q[k];
    // Eigen::Vector3f line_dir(...).normalize() on the float coefficients
    // Vector3f: fixed size 3, not vectorised: a0 + (a1 + a2)
    const float u0 = (float)q[3], u1 = (float)q[4], u2 = (float)q[5];
    const float r = 1.0f / std::sqrt(u0 * u0 + (u1 * u1 + u2 * u2));
    out[3] = u0 * r;
    out[4] = u1 * r;
    out[5] = u2 * r;
    out[6] = (float)q[6];
    (void)nu;
}
}  // namespace

extern "C" int orc_cylinder_segment(const float* x, const float* y, const float* z, const float* nx, const float* ny,
                                    const float* nz, int64_t n, const orc_cylinder_params* p, int32_t* inliers,
                                    int64_t* n_inliers, float coef[7], float best_out[7], int32_t* hypotheses) {
    *n_inliers = 0;
    *hypotheses = 0;
    if (n < 2) return 0;  // getSamples: "Can not select 2 unique points"
    std::mt19937 mt(p->seed);
    std::vector<int> sh((size_t)n);
    std::iota(sh.begin(), sh.end(), 0);
    int iterations = 0, n_best = -std::numeric_limits<int>::max();
    double k = 1.0;
    const double log_probability = std::log(1.0 - p->probability);
    const double one_over_indices = 1.0 / (double)n;
    unsigned skipped = 0;
    const unsigned max_skip = (unsigned)p->max_iterations * 10u;
    bool have = false;
    float best[7] = {0, 0, 0, 0, 0, 0, 0};
    while (iterations < k && skipped < max_skip) {
        for (unsigned i = 0; i < 2; ++i) std::swap(sh[i], sh[i + ((size_t)(mt() >> 1) % ((size_t)n - i))]);
        const int smp[2] = {sh[0], sh[1]};
        float m[7];
        if (!cyl_from2(x, y, z, nx, ny, nz, smp, p->radius_min, p->radius_max, m)) {
            ++skipped;
            continue;
        }
        int n_in = 0;
        if (cyl_valid(m, p->radius_min, p->radius_max))
            for (int64_t i = 0; i < n; ++i) n_in += cyl_in(x, y, z, nx, ny, nz, i, m, p->normal_distance_weight, p->threshold, p->eigen33);
        if (n_in > n_best) {
            n_best = n_in;
            have = true;
            std::memcpy(best, m, sizeof m);
            const double w = (double)n_best * one_over_indices;
            double p_no = 1.0 - std::pow(w, 2.0);
            p_no = std::max(std::numeric_limits<double>::epsilon(), p_no);
            p_no = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no);
            k = log_probability / std::log(p_no);
        }
        ++iterations;
        if (iterations > p->max_iterations) break;
    }
    *hypotheses = iterations;
    if (!have) return 0;
    std::memcpy(best_out, best, sizeof best);
    std::vector<int> inl;
    auto select = [&](const float* m) {
        inl.clear();
        if (!cyl_valid(m, p->radius_min, p->radius_max)) return;
        for (int64_t i = 0; i < n; ++i)
            if (cyl_in(x, y, z, nx, ny, nz, i, m, p->normal_distance_weight, p->threshold, p->eigen33)) inl.push_back((int)i);
    };
    select(best);
    float out[7];
    std::memcpy(out, best, sizeof out);
    if (p->optimize && !inl.empty()) {  // optimizeModelCoefficients: any inliers
        cyl_refine(x, y, z, inl, best, out);
        select(out);
    }
    std::memcpy(coef, out, sizeof out);
    for (size_t i = 0; i < inl.size(); ++i) inliers[i] = inl[i];
    *n_inliers = (int64_t)inl.size();
    return 1;
}

// ------------------------------------------------------------------------------------------
// Cone (PCL 1.7 sample_consensus/impl/sac_model_cone.hpp; SACSegmentationFromNormals::initSACModel sets
// the opening-angle limits and the eps angle, not the radius limits).  Vector4f arithmetic as for the
// cylinder.  A7: acosf / sinf / cosf taken as correctly rounded (float)f((double)x); tan(angle) in
// double.
namespace {
inline float acosf_cr(float a) { return (float)std::acos((double)a); }
inline float sinf_cr(float a) { return (float)std::sin((double)a); }
inline float cosf_cr(float a) { return (float)std::cos((double)a); }

// getAngle3D with Eigen's normalized(): 3.2 divides by the norm (0 / 0 = NaN); >= 3.3 keeps a zero vector
inline V4 normalized_e(V4 a, int eigen33) {
    if (eigen33 && !(dot(a, a) > 0.0f)) return a;
    return normalized(a);
}
inline double angle3d_e(V4 a, V4 b, int eigen33) {
    double rad = dot(normalized_e(a, eigen33), normalized_e(b, eigen33));
    if (rad < -1.0) rad = -1.0;
    else if (rad > 1.0) rad = 1.0;
    return std::acos(rad);
}

bool cone_from3(const V4 p[3], const V4 nn[3], double amin, double amax, float c[7]) {
    const V4 o12 = cross3(nn[0], nn[1]), o23 = cross3(nn[1], nn[2]), o31 = cross3(nn[2], nn[0]);
    const float den = dot(nn[0], o23);
    const float d1 = dot(p[0], nn[0]), d2 = dot(p[1], nn[1]), d3 = dot(p[2], nn[2]);
    const V4 num = add(add(mul(d1, o23), mul(d2, o31)), mul(d3, o12));
    const V4 apex = v4(num.v[0] / den, num.v[1] / den, num.v[2] / den, num.v[3] / den);
    V4 ap[3], np[3];
    for (int k = 0; k < 3; ++k) {
        ap[k] = sub(p[k], apex);
        const V4 u = normalized(ap[k]);  // ap / ap.norm()
        np[k] = add(apex, u);
    }
    const V4 axis = normalize(cross3(sub(np[1], np[0]), sub(np[2], np[0])));
    float acc = 0.0f;
    for (int k = 0; k < 3; ++k) acc = acc + acosf_cr(dot(normalize(ap[k]), axis));
    const float ang = acc / 3.0f;
    for (int k = 0; k < 3; ++k) c[k] = apex.v[k], c[3 + k] = axis.v[k];
    c[6] = ang;
    if (c[6] != -DBL_MAX && c[6] < amin) return false;
    if (c[6] != DBL_MAX && c[6] > amax) return false;
    return true;
}

bool cone_valid(const float c[7], const orc_cone_params* p) {
    if (p->eps_angle > 0.0) {
        const V4 coeff = v4(c[3], c[4], c[5]), ax = v4(p->axis[0], p->axis[1], p->axis[2]);
        double d = std::fabs(angle3d_e(ax, coeff, p->eigen33));
        d = std::min(d, M_PI - d);
        if (d > p->eps_angle) return false;
    }
    if (c[6] != -DBL_MAX && c[6] < p->min_angle) return false;
    if (c[6] != DBL_MAX && c[6] > p->max_angle) return false;
    return true;
}

inline bool cone_in(const float* x, const float* y, const float* z, const float* nx, const float* ny, const float* nz,
                    int64_t i, const float c[7], const orc_cone_params* p) {
    const V4 apex = v4(c[0], c[1], c[2]), ad = v4(c[3], c[4], c[5]);
    const float ang = c[6];
    const float apexdotdir = dot(apex, ad), dirdotdir = 1.0f / dot(ad, ad);
    const V4 pt = v4(x[i], y[i], z[i]), nn = v4(nx[i], ny[i], nz[i]);
    const float k = (dot(pt, ad) - apexdotdir) * dirdotdir;
    const V4 proj = add(apex, mul(k, ad));
    const V4 dir = normalize(sub(pt, proj));
    V4 h = sub(apex, proj);
    const double radius = std::tan((double)ang) * (double)std::sqrt(dot(h, h));
    h = normalize(h);
    const V4 cn = add(mul(sinf_cr(ang), h), mul(cosf_cr(ang), dir));
    const double d_euclid = std::fabs(std::sqrt(sqr_pt_line(pt, apex, ad)) - radius);
    double d_normal = std::fabs(angle3d_e(nn, cn, p->eigen33));
    d_normal = std::min(d_normal, M_PI - d_normal);
    const double w = p->normal_distance_weight;
    return std::fabs(w * d_normal + (1 - w) * d_euclid) < p->threshold;
}

// f = |v|^2 - (1 + tan^2 a) (u.v)^2 / |u|^2 with v = apex - p: the functor's sqrPointToLineDistance -
// (tan(a) |apex - proj|)^2 (Lagrange's identity), and its gradient in (apex, u, a)
inline void cone_residual(const double* q, float px, float py, float pz, double J[7], double* f) {
    const double vx = q[0] - px, vy = q[1] - py, vz = q[2] - pz;
    const double ux = q[3], uy = q[4], uz = q[5];
    const double s = ux * ux + uy * uy + uz * uz, g = ux * vx + uy * vy + uz * vz;
    const double t = std::tan(q[6]), K = 1.0 + t * t;
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

// optimizeModelCoefficients: Eigen's LM refuses fewer residuals than parameters (m < n:
// ImproperInputParameters, the coefficients unchanged); the direction is normalised either way.
elm::Result pcl_lm_cone(const float* x, const float* y, const float* z, const int32_t* inl, int64_t m, float c[7]);

void cone_refine(const float* x, const float* y, const float* z, const std::vector<int>& inl, const float in[7],
                 float out[7]) {
    double q[7];
    for (int k = 0; k < 7; ++k) q[k] = in[k];
    if (g_lm_mode == ORC_LM_PCL) {
        float c[7];
        for (int k = 0; k < 7; ++k) c[k] = in[k];
        if (!inl.empty()) pcl_lm_cone(x, y, z, inl.data(), (int64_t)inl.size(), c);
        for (int k = 0; k < 7; ++k) q[k] = c[k];
    } else if (inl.size() >= 7) {
        auto sums = [&](const double* v, double* jtj, double* jtr, double* cost) {
            for (int k = 0; k < 28; ++k) jtj[k] = 0;
            for (int k = 0; k < 7; ++k) jtr[k] = 0;
            *cost = 0;
            for (int id : inl) {
                double J[7], f;
                cone_residual(v, x[id], y[id], z[id], J, &f);
                int t = 0;
                for (int a = 0; a < 7; ++a)
                    for (int b = a; b < 7; ++b) jtj[t++] += J[a] * J[b];
                for (int a = 0; a < 7; ++a) jtr[a] += J[a] * f;
                *cost += f * f;
            }
        };
        lm_solve<7>(q, sums);
    }
    for (int k = 0; k < 3; ++k) out[k] = (float)q[k];
    const float u0 = (float)q[3], u1 = (float)q[4], u2 = (float)q[5];
    const float r = 1.0f / std::sqrt(u0 * u0 + (u1 * u1 + u2 * u2));
    out[3] = u0 * r;
    out[4] = u1 * r;
    out[5] = u2 * r;
    out[6] = (float)q[6];
}
}  // namespace

extern "C" int orc_cone_from3(const float xyz[9], const float nrm[9], double min_angle, double max_angle,
                              float coef[7]) {
    V4 p[3], nn[3];
    for (int k = 0; k < 3; ++k) {
        p[k] = v4(xyz[3 * k], xyz[3 * k + 1], xyz[3 * k + 2]);
        nn[k] = v4(nrm[3 * k], nrm[3 * k + 1], nrm[3 * k + 2]);
    }
    return cone_from3(p, nn, min_angle, max_angle, coef) ? 1 : 0;
}

extern "C" int orc_cone_segment(const float* x, const float* y, const float* z, const float* nx, const float* ny,
                                const float* nz, int64_t n, const orc_cone_params* p, int32_t* inliers,
                                int64_t* n_inliers, float coef[7], float best_out[7], int32_t* hypotheses) {
    *n_inliers = 0;
    *hypotheses = 0;
    if (n < 3) return 0;  // getSamples: "Can not select 3 unique points"
    std::mt19937 mt(p->seed);
    std::vector<int> sh((size_t)n);
    std::iota(sh.begin(), sh.end(), 0);
    int iterations = 0, n_best = -std::numeric_limits<int>::max();
    double k = 1.0;
    const double log_probability = std::log(1.0 - p->probability);
    const double one_over_indices = 1.0 / (double)n;
    unsigned skipped = 0;
    const unsigned max_skip = (unsigned)p->max_iterations * 10u;
    bool have = false;
    float best[7] = {0, 0, 0, 0, 0, 0, 0};
    while (iterations < k && skipped < max_skip) {
        for (unsigned i = 0; i < 3; ++i) std::swap(sh[i], sh[i + ((size_t)(mt() >> 1) % ((size_t)n - i))]);
        V4 ps[3], ns[3];
        for (int q = 0; q < 3; ++q) {
            const int id = sh[q];
            ps[q] = v4(x[id], y[id], z[id]);
            ns[q] = v4(nx[id], ny[id], nz[id]);
        }
        float m[7];
        if (!cone_from3(ps, ns, p->min_angle, p->max_angle, m)) {
            ++skipped;
            continue;
        }
        int n_in = 0;
        if (cone_valid(m, p))
            for (int64_t i = 0; i < n; ++i) n_in += cone_in(x, y, z, nx, ny, nz, i, m, p);
        if (n_in > n_best) {
            n_best = n_in;
            have = true;
            std::memcpy(best, m, sizeof m);
            const double w = (double)n_best * one_over_indices;
            double p_no = 1.0 - std::pow(w, 3.0);
            p_no = std::max(std::numeric_limits<double>::epsilon(), p_no);
            p_no = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no);
            k = log_probability / std::log(p_no);
        }
        ++iterations;
        if (iterations > p->max_iterations) break;
    }
    *hypotheses = iterations;
    if (!have) return 0;
    std::memcpy(best_out, best, sizeof best);
    std::vector<int> inl;
    auto select = [&](const float* m) {
        inl.clear();
        if (!cone_valid(m, p)) return;
        for (int64_t i = 0; i < n; ++i)
            if (cone_in(x, y, z, nx, ny, nz, i, m, p)) inl.push_back((int)i);
    };
    select(best);
    float out[7];
    std::memcpy(out, best, sizeof out);
    if (p->optimize && !inl.empty()) {  // optimizeModelCoefficients: "Inliers vector empty" returns unchanged
        cone_refine(x, y, z, inl, best, out);
        select(out);
    }
    std::memcpy(coef, out, sizeof out);
    for (size_t i = 0; i < inl.size(); ++i) inliers[i] = inl[i];
    *n_inliers = (int64_t)inl.size();
    return 1;
}

// ------------------------------------------------------------------------------------------
// PCL 1.7's optimizeModelCoefficients through Eigen's float Levenberg-Marquardt (eigen_lm.hpp), with
// each model's OptimizationFunctor (sac_model_sphere.h, sac_model_cylinder.h, sac_model_cone.h):
//   sphere    fvec[i] = sqrtf(cen_t.dot(cen_t)) - x[3], cen_t = (p - x[0..2], 0) (Vector4f dot, A3)
//   cylinder  fvec[i] = (float)(sqrPointToLineDistance(pt, line_pt, line_dir) - x[6] * x[6])
//   cone      fvec[i] = (float)(sqrPointToLineDistance(pt, apex, dir) - r * r),
//             r = tanf(x[6]) * |apex - proj(pt)| (A7: tanf as correctly rounded)
namespace {
inline float tanf_cr(float a) { return (float)std::tan((double)a); }

elm::Result pcl_lm_sphere(const float* x, const float* y, const float* z, const int32_t* inl, int64_t m, float c[4]) {
    std::vector<float> v(c, c + 4);
    auto f = [&](const float* q, float* fv) {
        for (int64_t i = 0; i < m; ++i) {
            const int32_t id = inl[i];
            const float cx = x[id] - q[0], cy = y[id] - q[1], cz = z[id] - q[2];
            fv[i] = std::sqrt(red4(cx * cx, cy * cy, cz * cz, 0.0f * 0.0f, ORC_REDUCE_SSE2)) - q[3];
        }
    };
    const elm::Result r = elm::minimize(f, m, v);
    for (int k = 0; k < 4; ++k) c[k] = v[(size_t)k];
    return r;
}

elm::Result pcl_lm_cylinder(const float* x, const float* y, const float* z, const int32_t* inl, int64_t m,
                            float c[7]) {
    std::vector<float> v(c, c + 7);
    auto f = [&](const float* q, float* fv) {
        const V4 lp = v4(q[0], q[1], q[2], 0.0f), ld = v4(q[3], q[4], q[5], 0.0f);
        for (int64_t i = 0; i < m; ++i) {
            const int32_t id = inl[i];
            const V4 pt = v4(x[id], y[id], z[id], 0.0f);
            fv[i] = (float)(sqr_pt_line(pt, lp, ld) - (double)(q[6] * q[6]));
        }
    };
    const elm::Result r = elm::minimize(f, m, v);
    for (int k = 0; k < 7; ++k) c[k] = v[(size_t)k];
    return r;
}

elm::Result pcl_lm_cone(const float* x, const float* y, const float* z, const int32_t* inl, int64_t m, float c[7]) {
    std::vector<float> v(c, c + 7);
    auto f = [&](const float* q, float* fv) {
        const V4 apex = v4(q[0], q[1], q[2], 0.0f), ad = v4(q[3], q[4], q[5], 0.0f);
        const float apexdotdir = dot(apex, ad), dirdotdir = 1.0f / dot(ad, ad);
        const float ta = tanf_cr(q[6]);
        for (int64_t i = 0; i < m; ++i) {
            const int32_t id = inl[i];
            const V4 pt = v4(x[id], y[id], z[id], 0.0f);
            const float k = (dot(pt, ad) - apexdotdir) * dirdotdir;
            const V4 proj = add(apex, mul(k, ad));
            const V4 h = sub(apex, proj);
            const float rad = ta * std::sqrt(dot(h, h));
            fv[i] = (float)(sqr_pt_line(pt, apex, ad) - (double)(rad * rad));
        }
    };
    const elm::Result r = elm::minimize(f, m, v);
    for (int k = 0; k < 7; ++k) c[k] = v[(size_t)k];
    return r;
}
}  // namespace

extern "C" {
void orc_set_lm_mode(int32_t mode) { g_lm_mode = mode == ORC_LM_OPTIMUM ? ORC_LM_OPTIMUM : ORC_LM_PCL; }
int32_t orc_get_lm_mode(void) { return g_lm_mode; }

int orc_lm_refine(int32_t model, const float* x, const float* y, const float* z, const int32_t* inl, int64_t m,
                  const float* in, float* out, int32_t mode, int32_t* status, int32_t* nfev) {
    const int saved = g_lm_mode;
    g_lm_mode = mode == ORC_LM_OPTIMUM ? ORC_LM_OPTIMUM : ORC_LM_PCL;
    std::vector<int> v(inl, inl + m);
    int st = -3, nf = 0;
    if (g_lm_mode == ORC_LM_PCL) {
        const int np = model == ORC_MODEL_SPHERE ? 4 : 7;
        for (int k = 0; k < np; ++k) out[k] = in[k];
        elm::Result r;
        if (model == ORC_MODEL_SPHERE) {
            if (m > 4) r = pcl_lm_sphere(x, y, z, inl, m, out);
        } else if (m > 0) {
            r = model == ORC_MODEL_CYLINDER ? pcl_lm_cylinder(x, y, z, inl, m, out) : pcl_lm_cone(x, y, z, inl, m, out);
        }
        if (model == ORC_MODEL_SPHERE ? m > 4 : m > 0) st = r.status, nf = r.nfev;
        if (model != ORC_MODEL_SPHERE) {  // line_dir.normalize() (Vector3f: a0 + (a1 + a2), times 1 / norm)
            const float rr = 1.0f / std::sqrt(out[3] * out[3] + (out[4] * out[4] + out[5] * out[5]));
            out[3] *= rr;
            out[4] *= rr;
            out[5] *= rr;
        }
    } else {
        Cloud c{x, y, z, 0};
        if (model == ORC_MODEL_SPHERE) {
            for (int k = 0; k < 4; ++k) out[k] = in[k];
            if (m > 4) sphere_refine(c, v, in, out);
        } else if (model == ORC_MODEL_CYLINDER) {
            cyl_refine(x, y, z, v, in, out);
        } else {
            cone_refine(x, y, z, v, in, out);
        }
    }
    g_lm_mode = saved;
    if (status) *status = st;
    if (nfev) *nfev = nf;
    return 1;
}
}  // extern "C"

// ---- independent pin of the LM restatement: the same driver instantiated in double ---------------
// (elm::Impl<double>) on double residuals, for comparison with MINPACK's lmdif (scipy's leastsq):
//   sphere    sqrt((dx dx + dy dy) + dz dz) - r,     d = p - c
//   cylinder  |u x (c - p)|^2 / |u|^2 - r^2           (x, y, z components in that order)
//   cone      |u x (a - p)|^2 / |u|^2 - (tan(t) |a - proj(p)|)^2
extern "C" int orc_elm_fit64(int32_t model, const float* x, const float* y, const float* z, const int32_t* inl,
                             int64_t m, const double* in, double* out, int32_t* status, int32_t* njac,
                             int32_t* trials) {
    const int np = model == ORC_MODEL_SPHERE ? 4 : 7;
    std::vector<double> v(in, in + np);
    auto cross_sq = [](double ux, double uy, double uz, double vx, double vy, double vz) {
        const double wx = uy * vz - uz * vy, wy = uz * vx - ux * vz, wz = ux * vy - uy * vx;
        return (wx * wx + wy * wy) + wz * wz;
    };
    auto f = [&](const double* q, double* fv) {
        for (int64_t i = 0; i < m; ++i) {
            const int32_t id = inl[i];
            const double px = x[id], py = y[id], pz = z[id];
            if (model == ORC_MODEL_SPHERE) {
                const double dx = px - q[0], dy = py - q[1], dz = pz - q[2];
                fv[i] = std::sqrt((dx * dx + dy * dy) + dz * dz) - q[3];
            } else {
                const double su = (q[3] * q[3] + q[4] * q[4]) + q[5] * q[5];
                const double d2 = cross_sq(q[3], q[4], q[5], q[0] - px, q[1] - py, q[2] - pz) / su;
                if (model == ORC_MODEL_CYLINDER) {
                    fv[i] = d2 - q[6] * q[6];
                } else {
                    const double k = (((px - q[0]) * q[3] + (py - q[1]) * q[4]) + (pz - q[2]) * q[5]) / su;
                    const double hx = k * q[3], hy = k * q[4], hz = k * q[5];
                    const double r = std::tan(q[6]) * std::sqrt((hx * hx + hy * hy) + hz * hz);
                    fv[i] = d2 - r * r;
                }
            }
        }
    };
    const elm::Result r = elm::minimize(f, m, v);
    for (int k = 0; k < np; ++k) out[k] = v[(size_t)k];
    if (status) *status = r.status;
    if (njac) *njac = r.njac;
    if (trials) *trials = r.trials;
    return 1;
}
