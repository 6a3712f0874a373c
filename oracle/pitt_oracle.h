/*
 * pitt_oracle.h -- CPU restatement of the reference's PCL path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker for the MI355X path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  It is never linked into, or called by, the
 * product library (pitt_object_table_segmentation_amd/csrc).
 *
 * Pinning status: PARTIALLY PINNED.  The reference ships no tests, no fixtures and no golden
 * vectors, and its arithmetic lives in PCL 1.7 which is absent here (s8c).
 * What is pinned: the mt19937 stream (C++ standard KAT, 10000th draw of the default seed =
 * 4123659995) and the reference's rnd() draws for seed 12345; analytic plane / cluster /
 * support known-answer cases (tests/test_oracle_kat.py).  What is NOT pinnable here: the
 * float reduction order of PCL's Eigen build (A3), Eigen 3.2 division forms (A9) and the
 * host libm trig used by eigen33 (A7).  Each of these is a switch below.
 */
#ifndef PITT_ORACLE_H
#define PITT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A3: 4-lane Eigen reduction order of dot()/squaredNorm() in the PCL binary. */
enum { ORC_REDUCE_SSE2 = 0, ORC_REDUCE_HADD = 1, ORC_REDUCE_SEQ = 2 };
/* A7: trig used inside eigen33: CR = float result of the double-evaluated function;
 *     LIBM = the host's atan2f/cosf/sinf (what PCL called on its platform). */
enum { ORC_TRIG_CR = 0, ORC_TRIG_LIBM = 1 };
/* Refinement of the sphere / cylinder / cone models (optimizeModelCoefficients):
 * ORC_LM_PCL      PCL's Eigen::LevenbergMarquardt<NumericalDiff<Functor>, float> restated (eigen_lm.hpp):
 *                 float, forward differences, Eigen's sqrt(FLT_EPSILON) stopping tolerances (default);
 * ORC_LM_OPTIMUM  a double Levenberg-Marquardt to the least-squares optimum of the same residual. */
enum { ORC_LM_PCL = 0, ORC_LM_OPTIMUM = 1 };
enum { ORC_MODEL_SPHERE = 0, ORC_MODEL_CYLINDER = 1, ORC_MODEL_CONE = 2 };
/* A9: Eigen 3.2 compound `v /= s` multiplies by (1/s); Eigen >= 3.3 divides. */
enum { ORC_DIV_EIGEN32 = 0, ORC_DIV_TRUE = 1 };

typedef struct {
    double   threshold;       /* SACSegmentation::setDistanceThreshold (double) */
    int32_t  max_iterations;  /* setMaxIterations */
    double   probability;     /* RandomSampleConsensus probability_ (PCL default 0.99) */
    uint32_t seed;            /* SampleConsensusModel rng seed (12345 when random_ == false) */
    int32_t  optimize;        /* setOptimizeCoefficients */
    int32_t  reduce_order;    /* ORC_REDUCE_* */
    int32_t  trig_mode;       /* ORC_TRIG_* */
    int32_t  div_mode;        /* ORC_DIV_* */
} orc_sac_params;

typedef struct {
    float    coefficients[4];      /* final (refined if optimize) coefficients */
    int32_t  n_coeff;              /* 4, or 0 when no model (PCL clears the vector) */
    int32_t  hypotheses;           /* T: hypotheses PCL evaluated (countWithinDistance calls) */
    int64_t  n_inliers;            /* final inlier count */
    int32_t  best_hypothesis;      /* index of the winning hypothesis */
    int32_t  rejected_samples;     /* isSampleGood rejections */
    int64_t  best_count;           /* countWithinDistance of the winning hypothesis */
    float    best_coefficients[4]; /* unrefined winning coefficients */
} orc_plane_result;

/* --- RNG / sampler (A2) --- */
void    orc_mt19937(uint32_t seed, int64_t n, uint32_t* out);
/* attempts*3 indices of SampleConsensusModel::drawIndexSample for a cloud of n points */
void    orc_sampler_table(int64_t n, uint32_t seed, int64_t attempts, int32_t* out);

/* --- plane model primitives (SampleConsensusModelPlane) --- */
int     orc_plane_coefficients(const float p0[3], const float p1[3], const float p2[3],
                               int32_t reduce_order, int32_t div_mode, float out[4]);
int64_t orc_count_within(const float* x, const float* y, const float* z, int64_t n,
                         const float coeff[4], double threshold, int32_t reduce_order);
int64_t orc_select_within(const float* x, const float* y, const float* z, int64_t n,
                          const float coeff[4], double threshold, int32_t reduce_order,
                          int32_t* out);
int     orc_eigen33(const float cov[9], int32_t trig_mode, int32_t div_mode,
                    float* eigenvalue, float vec[3]);
int     orc_optimize_plane(const float* x, const float* y, const float* z,
                           const int32_t* inliers, int64_t n_inliers, const float coeff[4],
                           const orc_sac_params* p, float out[4]);

/* --- SACSegmentation::segment (plane, RANSAC) --- */
int     orc_plane_segment(const float* x, const float* y, const float* z, int64_t n,
                          const orc_sac_params* p, int32_t* inliers_out /* cap n */,
                          orc_plane_result* res, int32_t* hyp_counts /* optional, cap max_it+1 */);

/* --- support segmentation service (supports_segmentation_srv.cpp:241-361) --- */
typedef struct {
    float   min_iterative_cloud_percentage;  /* 0.03 */
    float   min_iterative_plane_percentage;  /* 0.03 */
    float   horizontal_variance_threshold;   /* 0.09 */
    float   ransac_distance_threshold;       /* 0.02f */
    int32_t ransac_max_iterations;           /* 10 */
    float   horizontal_axis[3];              /* 0,0,-1 */
    float   edge_remove_offset[3];           /* 0.02,0.02,0.005 */
    int32_t reduce_order, trig_mode, div_mode;
} orc_support_params;

typedef struct orc_support_list orc_support_list;
orc_support_list* orc_find_supports(const float* x, const float* y, const float* z, int64_t n,
                                    const orc_support_params* p);
int32_t orc_support_count(const orc_support_list*);
/* copies support s: inliers (idx map, n ints), coefficients[4], sizes of the two clouds */
int     orc_support_get(const orc_support_list*, int32_t s, int32_t* idx_map /* cap n */,
                        float coeff[4], int64_t* n_support, int64_t* n_on_support);
int     orc_support_cloud(const orc_support_list*, int32_t s, int32_t which /*0 support,1 on*/,
                          float* x, float* y, float* z);
void    orc_support_free(orc_support_list*);

/* --- Euclidean cluster extraction (cluster_segmentation_srv.cpp:38-108) --- */
typedef struct orc_cluster_list orc_cluster_list;
orc_cluster_list* orc_euclidean_clusters(const float* x, const float* y, const float* z, int64_t n,
                                         double tolerance, double min_rate, double max_rate,
                                         int32_t min_input_size);
int32_t orc_cluster_count(const orc_cluster_list*);
int64_t orc_cluster_size(const orc_cluster_list*, int32_t c);
int     orc_cluster_get(const orc_cluster_list*, int32_t c, int32_t* idx, float centroid[3]);
void    orc_cluster_free(orc_cluster_list*);

/* --- preprocessing (deep_filter_srv.cpp:27-44, obj_segmentation.cpp:248) --- */
float   orc_service_float_param(float input, float default_value);
int     orc_deep_filter(const float* x, const float* y, const float* z, int64_t n, float th,
                        float* cx, float* cy, float* cz, int64_t* n_closer,
                        float* fx, float* fy, float* fz, int64_t* n_further);
int     orc_unpack_pointcloud2(const uint8_t* data, int32_t width, int32_t height, int32_t point_step,
                               int64_t row_step, int32_t off_x, int32_t off_y, int32_t off_z,
                               float* x, float* y, float* z);
int     orc_transform_cloud(const float* x, const float* y, const float* z, int64_t n, const float m[16],
                            int32_t dense, float* ox, float* oy, float* oz);
// VoxelGrid<PointXYZ>::applyFilter (pc_manager.cpp:61-67); sort_mode 0 = std::sort (PCL), 1 = stable.
// Returns 1 when the grid would overflow int32 (the output is then the input, n_out = n).
int     orc_voxel_grid(const float* x, const float* y, const float* z, int64_t n, float lx, float ly, float lz,
                       int32_t sort_mode, float* ox, float* oy, float* oz, int64_t* n_out);
// NormalEstimation<PointXYZ, Normal> with KdTree + setKSearch(k) (pc_manager.cpp:68-78), viewpoint vp.
// nn_out (n x k, optional) / nn_cnt (n, optional): the neighbours in summation order.
int     orc_normal_estimation(const float* x, const float* y, const float* z, int64_t n, int32_t k,
                              const float vp[3], float* nx, float* ny, float* nz, float* curv,
                              int32_t* nn_out, int32_t* nn_cnt);
// std::sort of (key, value) pairs by key: the library's, and a restatement with a settable depth limit
void    orc_std_sort_pairs(uint32_t* key, uint32_t* val, int64_t n);
void    orc_partial_sort_pairs(uint32_t* key, uint32_t* val, int64_t n);
void    orc_introsort_pairs(uint32_t* key, uint32_t* val, int64_t n, int32_t depth_limit);
// The sphere service (sphere_segmentation_srv.cpp:57-73): SACSegmentationFromNormals with SACMODEL_SPHERE
// falls through to the plain SampleConsensusModelSphere (normals unused), RANSAC, radius limits,
// optimize.  RANSAC bit-exact restatement; the refinement is a double Levenberg-Marquardt to the
// least-squares optimum (PCL: Eigen's float LM with numerical differences -- matched within tolerance).
typedef struct {
    double  threshold;
    int32_t max_iterations;
    int32_t optimize;
    double  probability;
    double  radius_min, radius_max;
    uint32_t seed;
    int32_t pad;
} orc_sphere_params;
// returns 1 with a model, 0 without; inliers (cap n) ascending; counts (cap counts_cap) per hypothesis
int     orc_sphere_segment(const float* x, const float* y, const float* z, int64_t n, const orc_sphere_params* p,
                           int32_t* inliers, int64_t* n_inliers, float coef[4], float best[4],
                           int32_t* hypotheses, int32_t* counts, int32_t counts_cap, int32_t* n_counts);
// SampleConsensusModelSphere::computeModelCoefficients on 4 points (xyz[4][3]); returns 0 when m11 == 0
int     orc_sphere_from4(const float xyz[12], float coef[4]);
// The cylinder service's seg.segment (cylinder_segmentation_srv.cpp:110-126): SampleConsensusModelCylinder
// with normals (2-point samples, the normal-weighted distance), radius limits, optimize (Levenberg-
// Marquardt on sqrPointToLineDistance - r^2, restated in double; PCL: Eigen's float LM).
typedef struct {
    double  threshold;
    int32_t max_iterations;
    int32_t optimize;
    double  probability;
    double  radius_min, radius_max;
    double  normal_distance_weight;
    uint32_t seed;
    int32_t eigen33;  // getAngle3D's normalized(): 0 = Eigen 3.2, 1 = Eigen >= 3.3 (as orc_cone_params)
} orc_cylinder_params;
int     orc_cylinder_segment(const float* x, const float* y, const float* z, const float* nx, const float* ny,
                             const float* nz, int64_t n, const orc_cylinder_params* p, int32_t* inliers,
                             int64_t* n_inliers, float coef[7], float best[7], int32_t* hypotheses);
// The cone service's seg.segment (cone_segmentation_srv.cpp:111-127): SampleConsensusModelCone with
// normals (3-point samples: the apex as the intersection of the three tangent planes, the axis as the
// normal of the plane through the unit apex-to-sample offsets, the opening angle as the mean of their
// angles to it), the opening-angle limits, isModelValid's eps angle against axis[3] (the service sets
// none: the zero vector), the normal-weighted distance, optimize (Levenberg-Marquardt in double on
// OptimizationFunctor's residual sqrPointToLineDistance - (tan(angle) |apex - proj|)^2; PCL: Eigen's
// float LM).  eigen33: 0 = Eigen 3.2's normalized() (a zero vector gives NaN, so the eps check against
// a zero axis never rejects); 1 = Eigen >= 3.3 (a zero vector stays zero: the angle is pi/2).
typedef struct {
    double  threshold;
    int32_t max_iterations;
    int32_t optimize;
    double  probability;
    double  normal_distance_weight;
    double  min_angle, max_angle;  // radians
    double  eps_angle;
    float   axis[3];
    int32_t eigen33;
    uint32_t seed;
    int32_t pad;
} orc_cone_params;
int     orc_cone_segment(const float* x, const float* y, const float* z, const float* nx, const float* ny,
                         const float* nz, int64_t n, const orc_cone_params* p, int32_t* inliers,
                         int64_t* n_inliers, float coef[7], float best[7], int32_t* hypotheses);
// SampleConsensusModelCone::computeModelCoefficients on 3 points + normals; returns 0 outside the angle limits
int     orc_cone_from3(const float xyz[9], const float nrm[9], double min_angle, double max_angle, float coef[7]);
// The axis "height" post-processing of the cylinder / cone services (cylinder_segmentation_srv.cpp:129-189,
// cone_segmentation_srv.cpp:129-189): every point projected on the axis of coef[0..5], the pair (i > j)
// of projected points farthest apart (first maximum in loop order), and the centroid (mode 0 cylinder:
// the pair's midpoint; mode 1 cone: apex + 3/4 height along the axis).  px/py/pz optional.
void    orc_axis_height(const float* x, const float* y, const float* z, int64_t n, const float coef[6],
                        int32_t mode, float* px, float* py, float* pz, float* height, int32_t* idx1,
                        int32_t* idx2, float centroid[3]);

/* Process-wide refinement mode of orc_{sphere,cylinder,cone}_segment (ORC_LM_*). */
void    orc_set_lm_mode(int32_t mode);
int32_t orc_get_lm_mode(void);
/* optimizeModelCoefficients alone: model ORC_MODEL_*, the inliers' indices inl[m] into x/y/z, the
 * coefficients in[4 or 7] -> out (cylinder / cone: the direction normalised afterwards, as PCL).
 * *status: Eigen's LevenbergMarquardtSpace::Status (ORC_LM_PCL; -3 when PCL skips the LM for too few
 * inliers), *nfev: functor evaluations.  Returns 1. */
int     orc_lm_refine(int32_t model, const float* x, const float* y, const float* z, const int32_t* inl, int64_t m,
                      const float* in, float* out, int32_t mode, int32_t* status, int32_t* nfev);
/* The LM restatement instantiated in double on double residuals (its pin against MINPACK's lmdif). */
int     orc_elm_fit64(int32_t model, const float* x, const float* y, const float* z, const int32_t* inl, int64_t m,
                      const double* in, double* out, int32_t* status, int32_t* njac, int32_t* trials);

#ifdef __cplusplus
}
#endif
#endif
