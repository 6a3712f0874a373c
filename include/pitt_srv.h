/*
 * pitt_srv.h -- C ABI over the C++ service mirror (pitt_srv.hpp), for FFI callers and tests.
 *
 * Each handler call runs the reference handler's semantics end to end (parameter resolution,
 * PCL-equivalent arithmetic on the MI355X, post-processing quirks) and keeps the response inside
 * the pitt_srv object until the next call; getters copy it out.
 *   pitt_srv_ransac_plane     <-> ransacPlaneDetaction  plane_segmentation_srv.cpp:27
 *   pitt_srv_find_supports    <-> findSupports          supports_segmentation_srv.cpp:241
 *   pitt_srv_clusterize       <-> clusterize            cluster_segmentation_srv.cpp:38
 *   pitt_srv_segment_objects  <-> depthAcquisition's support->cluster portion, obj_segmentation.cpp:261-312
 *   pitt_srv_segment_objects_dev <-> the same with the world cloud in HBM (adapters/ros/obj_segmentation_node.cpp)
 *   pitt_srv_ransac_sphere    <-> ransacSphereDetection sphere_segmentation_srv.cpp:29
 *   pitt_srv_ransac_cylinder  <-> ransacCylinderDetaction cylinder_segmentation_srv.cpp:82
 *   pitt_srv_ransac_cone      <-> ransacConeDetaction     cone_segmentation_srv.cpp:83
 *   pitt_srv_call_ransac_plane <-> callRansacPlaneSegmentation  ransac_segmentation.cpp:175-199
 *   pitt_srv_arbitrate        <-> clustersAcquisition's arbitration  ransac_segmentation.cpp:265-302
 *   pitt_srv_classify_clusters <-> clustersAcquisition's loop over a frame's clusters (normals, the four
 *                               services, the arbitration)            ransac_segmentation.cpp:230-302
 * Clouds are PCL PointXYZ arrays (x, y, z, pad: 16-byte stride), host memory.
 * Handler calls return 1 when the handler returns true, 0 when false, < 0 on an ABI error.
 */
#ifndef PITT_SRV_H
#define PITT_SRV_H
#include <stdint.h>

#include "pitt_seg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pitt_srv pitt_srv;

pitt_srv* pitt_srv_create(pitt_ctx* ctx);
void pitt_srv_destroy(pitt_srv* srv);

/* parameter server (roscpp typed-read rules, see pitt_srv.hpp) */
int pitt_srv_param_set_int(pitt_srv* srv, const char* name, int32_t v);
int pitt_srv_param_set_double(pitt_srv* srv, const char* name, double v);
int pitt_srv_param_set_list(pitt_srv* srv, const char* name, const double* v, int32_t n);
int pitt_srv_param_erase(pitt_srv* srv, const char* name);

/* SupportSegmentation request scalars; negative / wrong-length fields mean "service default" */
typedef struct {
    float   min_iterative_cloud_percentual_size;
    float   min_iterative_plane_percentual_size;
    float   variance_threshold_for_horizontal;
    float   ransac_distance_point_in_shape_threshold;
    float   ransac_model_normal_distance_weigth;
    int32_t ransac_max_iteration_threshold;
    int32_t n_horizontal_axis;
    float   horizontal_axis[8];
    int32_t n_edge_remove_offset;
    float   edge_remove_offset[8];
} pitt_srv_support_request;

int pitt_srv_ransac_plane(pitt_srv* srv, const float* xyz16, int64_t n, int64_t n_normals,
                          int32_t* inliers_out /* cap n */, int64_t* n_inliers,
                          float* coefficients_out /* cap 4 */, int32_t* n_coefficients,
                          float centroid_out[3]);

/* The sphere service: inliers (index 0 dropped, Q1), coefficients (centre, radius; none without a
 * model), centroid_out = the centre when there are coefficients. */
int pitt_srv_ransac_sphere(pitt_srv* srv, const float* xyz16, int64_t n, int64_t n_normals,
                           int32_t* inliers_out /* cap n */, int64_t* n_inliers,
                           float* coefficients_out /* cap 4 */, int32_t* n_coefficients, float centroid_out[3]);

/* The cylinder service: normals3 = (nx, ny, nz) per point (needed when n_normals == n); inliers (index 0
 * dropped, Q1); coefficients = the 7 model values (none without a model) followed by the axis height
 * (-1 without inliers); centroid_out = the midpoint of the farthest projected pair (0 without inliers). */
int pitt_srv_ransac_cylinder(pitt_srv* srv, const float* xyz16, int64_t n, const float* normals3, int64_t n_normals,
                             int32_t* inliers_out /* cap n */, int64_t* n_inliers,
                             float* coefficients_out /* cap 8 */, int32_t* n_coefficients, float centroid_out[3]);

/* The cone service: as the cylinder's; coefficients = apex, axis direction, opening angle (none without
 * a model) followed by the axis height (-1 without inliers); centroid_out = apex + 3/4 height along the
 * unit axis (0 without inliers). */
int pitt_srv_ransac_cone(pitt_srv* srv, const float* xyz16, int64_t n, const float* normals3, int64_t n_normals,
                         int32_t* inliers_out /* cap n */, int64_t* n_inliers, float* coefficients_out /* cap 8 */,
                         int32_t* n_coefficients, float centroid_out[3]);

/* callRansacPlaneSegmentation, ransac_segmentation.cpp:175-199: the plane service, accepted (1) only
 * when its response holds more than 0 inliers (Q2: the min-inliers parameter is read but unused);
 * 0 leaves *n_inliers = *n_coefficients = 0. */
int pitt_srv_call_ransac_plane(pitt_srv* srv, const float* xyz16, int64_t n, int64_t n_normals,
                               int32_t* inliers_out /* cap n */, int64_t* n_inliers,
                               float* coefficients_out /* cap 4 */, int32_t* n_coefficients);

/* The primitive arbitration of clustersAcquisition, ransac_segmentation.cpp:265-302, over the four
 * services' inlier counts: returns the reference's tag (0 unknown, 1 plane, 2 sphere, 3 cone,
 * 4 cylinder; :42-46) or PITT_E_INVALID for a negative count. */
int pitt_srv_arbitrate(int64_t sphere_inliers, int64_t cylinder_inliers, int64_t cone_inliers,
                       int64_t plane_inliers);

/* clustersAcquisition's loop (ransac_segmentation.cpp:230-302) over n_clusters clusters of one SoA
 * (device or host x/y/z; cluster c = [offsets[c], offsets[c] + counts[c]), host arrays): the four
 * services with the parameters their handlers read, one pass for all clusters (pitt_classify_clusters).
 * out: host [n_clusters].  Returns the pitt status. */
int pitt_srv_classify_clusters(pitt_srv* srv, const float* x, const float* y, const float* z,
                               const int64_t* offsets, const int64_t* counts, int32_t n_clusters,
                               pitt_cluster_shape* out);

/* used_out: the response's used_* fields in declaration order:
 * cloud%, plane%, max var, min var, max iter, distance th, normal weight, axis[3], offset[3] */
int pitt_srv_find_supports(pitt_srv* srv, const float* xyz16, int64_t n, int64_t n_normals,
                           const pitt_srv_support_request* req, int32_t* n_supports, float used_out[13]);
int pitt_srv_support_get(pitt_srv* srv, int32_t s, int32_t* idx_map /* cap n */, float coef[4],
                         int64_t* n_support, int64_t* n_on_support);
int pitt_srv_support_cloud(pitt_srv* srv, int32_t s, int32_t which /* 0 support, 1 on-support */,
                           float* xyz16_out);

int pitt_srv_clusterize(pitt_srv* srv, const float* xyz16, int64_t n, int32_t* n_clusters);
int pitt_srv_cluster_get(pitt_srv* srv, int32_t c, int32_t* inliers /* cap size */, int64_t* size,
                         float centroid[3], float* xyz16_out /* optional, cap size */);

int pitt_srv_segment_objects(pitt_srv* srv, const float* xyz16, int64_t n, int64_t n_normals,
                             int32_t* n_outputs);
int pitt_srv_output_size(pitt_srv* srv, int32_t o, int32_t* n_clusters);
int pitt_srv_output_cluster(pitt_srv* srv, int32_t o, int32_t c, int32_t* inliers, int64_t* size,
                            float centroid[3]);

/* depthAcquisition's support -> cluster portion (obj_segmentation.cpp:261-312) with the world cloud in HBM:
 * x/y/z device SoA (the output of pitt_transform_cloud).  The support request is built from the
 * parameter server as callSupportFilter builds it (:164-177, -1 when a parameter is unset) and resolved
 * as findSupports resolves it (supports_segmentation_srv.cpp:70-86); the cluster parameters are read
 * as clusterize reads them (cluster_segmentation_srv.cpp:44-50, Q6); then pitt_segment_objects_dev.
 * The normals callSupportFilter sends are not needed: the support service's SACMODEL_PLANE never reads
 * them, and the node's normals always match the cloud's size (A1).  Returns the pitt status; *out is
 * valid until the next call on the context. */
int pitt_srv_segment_objects_dev(pitt_srv* srv, const float* x, const float* y, const float* z, int64_t n,
                                 pitt_scene* out);
/* The two parameter sets pitt_srv_segment_objects_dev would use now (either pointer may be NULL). */
int pitt_srv_resolved_params(pitt_srv* srv, pitt_support_params* sp, pitt_cluster_params* cp);

#ifdef __cplusplus
}
#endif
#endif /* PITT_SRV_H */
