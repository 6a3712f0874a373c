// pitt_srv.cpp -- the service mirror: the reference's handler logic above the C ABI.
// Reference paths cited per function.  No arithmetic of the path lives here; it is parameter
// resolution, message assembly and the reference's post-processing (Q1, Q2, Q3, Q6, Q7).
#include "../../include/pitt_srv.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pitt_srv.h"

namespace pitt {

// ---- ParamServer: roscpp param.cpp getImpl typed reads ---------------------------------------
bool ParamServer::get(const std::string& k, double& out) const {
    auto it = m_.find(k);
    if (it == m_.end()) return false;
    if (it->second.kind == INT) { out = (double)it->second.i; return true; }
    if (it->second.kind == DOUBLE) { out = it->second.d; return true; }
    return false;
}
bool ParamServer::get(const std::string& k, float& out) const {
    double d;
    if (!get(k, d)) return false;
    out = (float)d;
    return true;
}
bool ParamServer::get(const std::string& k, int& out) const {
    auto it = m_.find(k);
    if (it == m_.end()) return false;
    if (it->second.kind == INT) { out = (int)it->second.i; return true; }
    if (it->second.kind == DOUBLE) {  // roscpp rounds a double read as int
        double d = it->second.d;
        d = std::fmod(d, 1.0) < 0.5 ? std::floor(d) : std::ceil(d);
        out = (int)d;
        return true;
    }
    return false;
}
bool ParamServer::get(const std::string& k, std::vector<float>& out) const {
    auto it = m_.find(k);
    if (it == m_.end() || it->second.kind != LIST) return false;
    out.assign(it->second.list.begin(), it->second.list.end());
    return true;
}

// The parameter reads of the four primitive handlers (each service reads its own on every call).
// plane_segmentation_srv.cpp:27-74 (the normal weight, eps and opening angles do not reach
// SACMODEL_PLANE, A1)
pitt_sac_params SegmentationServices::planeParams() {
    int maxIterations;
    double normalDistanceWeight, distanceThreshold, epsAngleTh, minOpeningAngle, maxOpeningAngle;
    params_.param(srvm::PARAM_NAME_PLANE_NORMAL_DISTANCE_WEIGHT, normalDistanceWeight, 0.001);
    params_.param(srvm::PARAM_NAME_PLANE_DISTANCE_TH, distanceThreshold, 0.007);
    params_.param(srvm::PARAM_NAME_PLANE_MAX_ITERATION_LIMIT, maxIterations, 1000);
    params_.param(srvm::PARAM_NAME_PLANE_EPS_ANGLE_TH, epsAngleTh, 0.0);
    params_.param(srvm::PARAM_NAME_PLANE_MIN_OPENING_ANGLE_DEGREE, minOpeningAngle, 0.0);
    params_.param(srvm::PARAM_NAME_PLANE_MAX_OPENING_ANGLE_DEGREE, maxOpeningAngle, 10.0);
    (void)normalDistanceWeight; (void)epsAngleTh; (void)minOpeningAngle; (void)maxOpeningAngle;  // unused by SACMODEL_PLANE (A1)

    pitt_sac_params p;
    pitt_sac_params_default(&p);
    p.threshold = distanceThreshold;
    p.max_iterations = maxIterations;
    return p;
}

// cylinder_segmentation_srv.cpp:82-126
pitt_cylinder_params SegmentationServices::cylinderParams() {
    int maxIterations;
    double normalDistanceWeight, distanceThreshold, minRadiusLimit, maxRadiusLimit, epsAngleTh, minOpeningAngle,
        maxOpeningAngle;
    params_.param(srvm::PARAM_NAME_CYLINDER_NORMAL_DISTANCE_WEIGHT, normalDistanceWeight, 0.001);
    params_.param(srvm::PARAM_NAME_CYLINDER_DISTANCE_TH, distanceThreshold, 0.008);
    params_.param(srvm::PARAM_NAME_CYLINDER_MAX_ITERATION_LIMIT, maxIterations, 1000);
    params_.param(srvm::PARAM_NAME_CYLINDER_MIN_RADIUS_LIMIT, minRadiusLimit, 0.005);
    params_.param(srvm::PARAM_NAME_CYLINDER_MAX_RADIUS_LIMIT, maxRadiusLimit, 0.500);
    params_.param(srvm::PARAM_NAME_CYLINDER_EPS_ANGLE_TH, epsAngleTh, 0.0001);
    params_.param(srvm::PARAM_NAME_CYLINDER_MIN_OPENING_ANGLE_DEGREE, minOpeningAngle, 50.0);
    params_.param(srvm::PARAM_NAME_CYLINDER_MAX_OPENING_ANGLE_DEGREE, maxOpeningAngle, 180.0);
    (void)epsAngleTh; (void)minOpeningAngle; (void)maxOpeningAngle;

    pitt_cylinder_params p;
    p.threshold = distanceThreshold;
    p.max_iterations = maxIterations;
    p.optimize = 1;
    p.probability = 0.99;
    p.radius_min = minRadiusLimit;
    p.radius_max = maxRadiusLimit;
    p.normal_distance_weight = normalDistanceWeight;
    p.seed = 12345u;
    p.eigen33 = 0;  // Eigen 3.2 (the reference's ROS Indigo toolchain)
    return p;
}

// cone_segmentation_srv.cpp:83-127
pitt_cone_params SegmentationServices::coneParams() {
    int maxIterations;
    double normalDistanceWeight, distanceThreshold, minRadiusLimit, maxRadiusLimit, epsAngleTh, minOpeningAngle,
        maxOpeningAngle;
    params_.param(srvm::PARAM_NAME_CONE_NORMAL_DISTANCE_WEIGHT, normalDistanceWeight, 0.0006);
    params_.param(srvm::PARAM_NAME_CONE_DISTANCE_TH, distanceThreshold, 0.0055);
    params_.param(srvm::PARAM_NAME_CONE_MAX_ITERATION_LIMIT, maxIterations, 1000);
    params_.param(srvm::PARAM_NAME_CONE_MIN_RADIUS_LIMIT, minRadiusLimit, 0.001);
    params_.param(srvm::PARAM_NAME_CONE_MAX_RADIUS_LIMIT, maxRadiusLimit, 0.500);
    params_.param(srvm::PARAM_NAME_CONE_EPS_ANGLE_TH, epsAngleTh, 0.4);
    params_.param(srvm::PARAM_NAME_CONE_MIN_OPENING_ANGLE_DEGREE, minOpeningAngle, 10.0);
    params_.param(srvm::PARAM_NAME_CONE_MAX_OPENING_ANGLE_DEGREE, maxOpeningAngle, 170.0);
    (void)minRadiusLimit; (void)maxRadiusLimit;

    pitt_cone_params p;
    p.threshold = distanceThreshold;
    p.max_iterations = maxIterations;
    p.optimize = 1;
    p.probability = 0.99;
    p.normal_distance_weight = normalDistanceWeight;
    p.min_angle = minOpeningAngle / 180.0 * M_PI;
    p.max_angle = maxOpeningAngle / 180.0 * M_PI;
    p.eps_angle = epsAngleTh;
    p.axis[0] = p.axis[1] = p.axis[2] = 0.0f;
    p.seed = 12345u;
    p.pad = 0;
    p.eigen33 = 0;  // Eigen 3.2 (the reference's ROS Indigo toolchain)
    return p;
}

// sphere_segmentation_srv.cpp:29-73
pitt_sphere_params SegmentationServices::sphereParams() {
    int maxIterations;
    double normalDistanceWeight, distanceThreshold, minRadiusLimit, maxRadiusLimit, epsAngleTh, minOpeningAngle,
        maxOpeningAngle;
    params_.param(srvm::PARAM_NAME_SPHERE_NORMAL_DISTANCE_WEIGHT, normalDistanceWeight, 0.001);
    params_.param(srvm::PARAM_NAME_SPHERE_DISTANCE_TH, distanceThreshold, 0.007);
    params_.param(srvm::PARAM_NAME_SPHERE_MAX_ITERATION_LIMIT, maxIterations, 1000);
    params_.param(srvm::PARAM_NAME_SPHERE_MIN_RADIUS_LIMIT, minRadiusLimit, 0.005);
    params_.param(srvm::PARAM_NAME_SPHERE_MAX_RADIUS_LIMIT, maxRadiusLimit, 0.500);
    params_.param(srvm::PARAM_NAME_SPHERE_EPS_ANGLE_TH, epsAngleTh, 0.0);
    params_.param(srvm::PARAM_NAME_SPHERE_MIN_OPENING_ANGLE_DEGREE, minOpeningAngle, 100.0);
    params_.param(srvm::PARAM_NAME_SPHERE_MAX_OPENING_ANGLE_DEGREE, maxOpeningAngle, 180.0);
    (void)normalDistanceWeight; (void)epsAngleTh; (void)minOpeningAngle; (void)maxOpeningAngle;

    pitt_sphere_params p;
    p.threshold = distanceThreshold;
    p.max_iterations = maxIterations;
    p.optimize = 1;
    p.probability = 0.99;
    p.radius_min = minRadiusLimit;
    p.radius_max = maxRadiusLimit;
    p.seed = 12345u;
    p.pad = 0;
    return p;
}

// plane_segmentation_srv.cpp:27-74
bool SegmentationServices::ransacPlaneDetaction(pitt_msgs::PrimitiveSegmentation::Request& req,
                                                pitt_msgs::PrimitiveSegmentation::Response& res) {
    const pitt_sac_params p = planeParams();
    std::vector<int32_t> inl(req.cloud.size());
    int64_t n_inl = 0;
    float coef[4] = {0, 0, 0, 0};
    int32_t n_coef = 0;
    status_ = PITT_OK;
    // SACSegmentationFromNormals::initSACModel: the normals must match the cloud, else PCL clears
    // the outputs (A1).
    if (req.normals.size() == req.cloud.size()) {
        status_ = pitt_plane_segment(ctx_, req.cloud.data.data(), (int64_t)req.cloud.size(), 16, &p, inl.data(),
                                     &n_inl, coef, &n_coef);
        if (status_ < 0) { n_inl = 0; n_coef = 0; }
    }
    // PCManager::inlierToVectorMsg (pc_manager.cpp:105-111): drops index 0 (Q1)
    res.inliers.clear();
    for (int64_t i = 0; i < n_inl; ++i)
        if (inl[(size_t)i] != 0) res.inliers.push_back(inl[(size_t)i]);
    // coefficientToVectorMsg (:112-117)
    res.coefficients.assign(coef, coef + n_coef);
    return true;
}

// cylinder_segmentation_srv.cpp:82-216.  The eps angle and opening angles are read but do not constrain
// SACMODEL_CYLINDER here (no axis is set, :123); after the fit, the cloud's projection on the axis gives
// the height (pushed after the 7 coefficients) and the centroid (:129-200).
bool SegmentationServices::ransacCylinderDetaction(pitt_msgs::PrimitiveSegmentation::Request& req,
                                                   pitt_msgs::PrimitiveSegmentation::Response& res) {
    const pitt_cylinder_params p = cylinderParams();
    const size_t n = req.cloud.size();
    std::vector<int32_t> inl(n + 1);
    int64_t n_inl = 0;
    float coef[7] = {0, 0, 0, 0, 0, 0, 0};
    int32_t n_coef = 0;
    status_ = PITT_OK;
    if (req.normals.size() == n) {  // initSACModel: normals must match the cloud
        if (req.normals.data.size() != 3 * n) {
            status_ = PITT_E_INVALID;  // the normal vectors themselves are needed here
            return false;
        }
        status_ = pitt_cylinder_segment_host(ctx_, req.cloud.data.data(), req.normals.data.data(), (int64_t)n, &p,
                                             inl.data(), &n_inl, coef, nullptr);
        if (status_ == PITT_OK) n_coef = 7;
        if (status_ != PITT_OK) n_inl = 0;
        if (status_ == PITT_NO_MODEL) status_ = PITT_OK;
        if (status_ < 0) return false;
    }
    float height = -1.0f, centroid[3] = {0, 0, 0};  // the reference leaves the centroid unset without inliers
    if (n_inl > 0) {
        int32_t i1 = -1, i2 = -1;
        status_ = pitt_axis_height_host(ctx_, req.cloud.data.data(), (int64_t)n, coef, PITT_AXIS_CYLINDER, &height,
                                        &i1, &i2, centroid);
        if (status_ < 0) return false;
    }
    res.inliers.clear();  // inlierToVectorMsg drops index 0 (Q1)
    for (int64_t i = 0; i < n_inl; ++i)
        if (inl[(size_t)i] != 0) res.inliers.push_back(inl[(size_t)i]);
    res.coefficients.assign(coef, coef + n_coef);
    res.coefficients.push_back(height);  // :195
    res.x_centroid = centroid[0];
    res.y_centroid = centroid[1];
    res.z_centroid = centroid[2];
    return true;
}

// cone_segmentation_srv.cpp:83-216.  The radius limits are read and set (:121) but SACMODEL_CONE does not
// use them; the opening angles (degrees, converted at :124) and the eps angle (:125, against no axis)
// constrain the model.  After the fit, the cloud's projection on the axis gives the height (pushed after
// the 7 coefficients) and the centroid, apex + 3/4 height along the unit axis (:129-200).
bool SegmentationServices::ransacConeDetaction(pitt_msgs::PrimitiveSegmentation::Request& req,
                                                   pitt_msgs::PrimitiveSegmentation::Response& res) {
    const pitt_cone_params p = coneParams();
    const size_t n = req.cloud.size();
    std::vector<int32_t> inl(n + 1);
    int64_t n_inl = 0;
    float coef[7] = {0, 0, 0, 0, 0, 0, 0};
    int32_t n_coef = 0;
    status_ = PITT_OK;
    if (req.normals.size() == n) {  // initSACModel: normals must match the cloud
        if (req.normals.data.size() != 3 * n) {
            status_ = PITT_E_INVALID;  // the normal vectors themselves are needed here
            return false;
        }
        status_ = pitt_cone_segment_host(ctx_, req.cloud.data.data(), req.normals.data.data(), (int64_t)n, &p,
                                         inl.data(), &n_inl, coef, nullptr);
        if (status_ == PITT_OK) n_coef = 7;
        if (status_ != PITT_OK) n_inl = 0;
        if (status_ == PITT_NO_MODEL) status_ = PITT_OK;
        if (status_ < 0) return false;
    }
    float height = -1.0f, centroid[3] = {0, 0, 0};  // the reference leaves the centroid unset without inliers
    if (n_inl > 0) {
        int32_t i1 = -1, i2 = -1;
        status_ = pitt_axis_height_host(ctx_, req.cloud.data.data(), (int64_t)n, coef, PITT_AXIS_CONE, &height,
                                        &i1, &i2, centroid);
        if (status_ < 0) return false;
    }
    res.inliers.clear();  // inlierToVectorMsg drops index 0 (Q1)
    for (int64_t i = 0; i < n_inl; ++i)
        if (inl[(size_t)i] != 0) res.inliers.push_back(inl[(size_t)i]);
    res.coefficients.assign(coef, coef + n_coef);
    res.coefficients.push_back(height);  // :195
    res.x_centroid = centroid[0];
    res.y_centroid = centroid[1];
    res.z_centroid = centroid[2];
    return true;
}

// sphere_segmentation_srv.cpp:29-96.  SACSegmentationFromNormals with SACMODEL_SPHERE falls through to
// the plain sphere model: the normal weight, eps angle and opening angles are read but unused.
bool SegmentationServices::ransacSphereDetection(pitt_msgs::PrimitiveSegmentation::Request& req,
                                                 pitt_msgs::PrimitiveSegmentation::Response& res) {
    const pitt_sphere_params p = sphereParams();
    std::vector<int32_t> inl(req.cloud.size() + 1);
    int64_t n_inl = 0;
    float coef[4] = {0, 0, 0, 0};
    int32_t n_coef = 0;
    status_ = PITT_OK;
    if (req.normals.size() == req.cloud.size()) {  // initSACModel: normals must match the cloud
        status_ = pitt_sphere_segment_host(ctx_, req.cloud.data.data(), (int64_t)req.cloud.size(), &p, inl.data(),
                                           &n_inl, coef, nullptr);
        if (status_ == PITT_OK) n_coef = 4;
        if (status_ != PITT_OK) n_inl = 0;  // no model: PCL clears both outputs
        if (status_ == PITT_NO_MODEL) status_ = PITT_OK;
    }
    res.inliers.clear();  // inlierToVectorMsg drops index 0 (Q1)
    for (int64_t i = 0; i < n_inl; ++i)
        if (inl[(size_t)i] != 0) res.inliers.push_back(inl[(size_t)i]);
    res.coefficients.assign(coef, coef + n_coef);
    if (n_coef > 0) {  // :79-83, the centre
        res.x_centroid = coef[0];
        res.y_centroid = coef[1];
        res.z_centroid = coef[2];
    }
    return true;
}

// initializeInputParameters, supports_segmentation_srv.cpp:70-86: a request field < 0 (or a vector
// that is not 3 long) selects the service default.
pitt_support_params SegmentationServices::resolveSupport(const pitt_msgs::SupportSegmentation::Request& req) {
    static const float kAxis[3] = {0.0f, 0.0f, -1.0f};
    static const float kOffset[3] = {0.02f, 0.02f, 0.005f};
    pitt_support_params sp;
    pitt_support_params_default(&sp);
    sp.min_iterative_cloud_percentage = srvm::getServiceFloatParameter(req.min_iterative_cloud_percentual_size, 0.030f);
    sp.min_iterative_plane_percentage = srvm::getServiceFloatParameter(req.min_iterative_plane_percentual_size, 0.030f);
    sp.horizontal_variance_threshold = srvm::getServiceFloatParameter(req.variance_threshold_for_horizontal, 0.09f);
    sp.ransac_distance_threshold = srvm::getServiceFloatParameter(req.ransac_distance_point_in_shape_threshold, 0.02f);
    sp.ransac_max_iterations = srvm::getServiceIntParameter(req.ransac_max_iteration_threshold, 10);
    const std::vector<float> axis = srvm::getService3DArrayParameter(req.horizontal_axis, kAxis);
    const std::vector<float> off = srvm::getService3DArrayParameter(req.support_edge_remove_offset, kOffset);
    for (int i = 0; i < 3; ++i) {
        sp.horizontal_axis[i] = axis[(size_t)i];
        sp.edge_remove_offset[i] = off[(size_t)i];
    }
    return sp;
}

// supports_segmentation_srv.cpp:241-361 (+ initializeInputParameters :70-86)
bool SegmentationServices::findSupports(pitt_msgs::SupportSegmentation::Request& req,
                                        pitt_msgs::SupportSegmentation::Response& res) {
    return findSupports(req.input_cloud.data.data(), req.input_cloud.size(), req.input_norm.size(), req, res);
}

namespace {
// f(i0, i1) over [0, n) in up to 8 host threads (chunks of at least 2^17): the response of a
// 1.2M-point scene is ~25 MB of copies, ~5 ms on one core
template <class F>
void host_parallel(int64_t n, F f) {
    const int64_t kMin = 1 << 17;
    const int nt = (int)std::min<int64_t>(8, std::max<int64_t>(1, n / kMin));
    if (nt <= 1) {
        f((int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve((size_t)nt - 1);
    for (int t = 1; t < nt; ++t) th.emplace_back(f, n * t / nt, n * (t + 1) / nt);
    f((int64_t)0, n / nt);
    for (std::thread& x : th) x.join();
}

// SoA planes (n apart) -> a PointXYZ message cloud (x, y, z, 1), sized once
void planes_to_cloud(const float* p, int64_t n, pitt_msgs::PointCloud& c) {
    c.data.resize((size_t)n * 4);
    float* d = c.data.data();
    host_parallel(n, [=](int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            d[4 * i] = p[i];
            d[4 * i + 1] = p[n + i];
            d[4 * i + 2] = p[2 * n + i];
            d[4 * i + 3] = 1.0f;
        }
    });
}

void copy_ints(const int32_t* src, int64_t n, std::vector<int32_t>& dst) {
    dst.resize((size_t)n);
    int32_t* d = dst.data();
    host_parallel(n, [=](int64_t i0, int64_t i1) { std::memcpy(d + i0, src + i0, (size_t)(i1 - i0) * 4); });
}
}  // namespace

bool SegmentationServices::findSupports(const float* xyz16, size_t n, size_t n_normals,
                                        const pitt_msgs::SupportSegmentation::Request& req,
                                        pitt_msgs::SupportSegmentation::Response& res) {
    const pitt_support_params sp = resolveSupport(req);
    const float ndw = srvm::getServiceFloatParameter(req.ransac_model_normal_distance_weigth, 0.9f);

    status_ = PITT_OK;
    size_t found = 0;
    // The first RANSAC call runs with the request's normals: a size mismatch fails it (A1) and the
    // loop exits before any support is found.  Later rounds re-estimate normals of matching size.
    if (n_normals == n) {
        // the request's PointXYZ bytes go up as they lie (one copy, deinterleaved on the device)
        pitt_support_list L;
        status_ = pitt_find_supports_aos(ctx_, xyz16, (int64_t)n, 16, &sp, &L);
        if (status_ == PITT_OK) {
            // a response used again keeps its supports' buffers: assign / resize refill them in place
            // (a config-5 response is ~25 MB; fresh vectors would fault every page in again)
            found = (size_t)L.n_supports;
            if (res.supports_description.size() < found) res.supports_description.resize(found);
            for (size_t s = 0; s < found; ++s) {
                const pitt_support& su = L.supports[s];
                pitt_msgs::Support& m = res.supports_description[s];
                copy_ints(su.idx_map, su.n_points, m.inliers);
                planes_to_cloud(su.support_xyz, su.n_support, m.support_cloud);
                planes_to_cloud(su.on_support_xyz, su.n_on_support, m.on_support_cloud);
                m.support_coefficient_a = su.coefficients[0];
                m.support_coefficient_b = su.coefficients[1];
                m.support_coefficient_c = su.coefficients[2];
                m.support_coefficient_d = su.coefficients[3];
            }
        }
    }
    res.supports_description.resize(found);
    res.used_min_iterative_cloud_percentual_size = sp.min_iterative_cloud_percentage;
    res.used_min_iterative_plane_percentual_size = sp.min_iterative_plane_percentage;
    res.used_max_variance_threshold_for_horizontal = sp.horizontal_variance_threshold;
    res.used_min_variance_threshold_for_horizontal = -1 * sp.horizontal_variance_threshold;
    res.used_ransac_max_iteration_threshold = sp.ransac_max_iterations;
    res.used_ransac_distance_point_in_shape_threshold = sp.ransac_distance_threshold;
    res.used_ransac_model_normal_distance_weigth = ndw;
    res.used_horizontal_axis.assign(sp.horizontal_axis, sp.horizontal_axis + 3);
    res.used_support_edge_remove_offset.assign(sp.edge_remove_offset, sp.edge_remove_offset + 3);
    return true;
}

// cluster_segmentation_srv.cpp:38-108
bool SegmentationServices::clusterize(pitt_msgs::ClusterSegmentation::Request& req,
                                      pitt_msgs::ClusterSegmentation::Response& res) {
    return clusterize(req.cloud.data.data(), req.cloud.size(), res);
}

bool SegmentationServices::clusterize(const float* xyz16, size_t n, pitt_msgs::ClusterSegmentation::Response& res) {
    const pitt_cluster_params cp = clusterParams();
    status_ = PITT_OK;
    size_t found = 0;
    if (n >= (size_t)(int64_t)cp.min_input_size) {
        const int mn = (int)std::round((double)n * cp.min_rate);
        const int mx = (int)std::round((double)n * cp.max_rate);
        pitt_cluster_list L;
        status_ = pitt_euclidean_clusters_aos(ctx_, xyz16, (int64_t)n, 16, cp.tolerance, mn, mx, &L);
        if (status_ == PITT_OK) {
            found = (size_t)L.n_clusters;  // buffers of a response used again are refilled in place
            if (res.cluster_objs.size() < found) res.cluster_objs.resize(found);
            for (int c = 0; c < L.n_clusters; ++c) {
                const pitt_cluster& cl = L.clusters[c];
                pitt_msgs::InliersCluster& m = res.cluster_objs[(size_t)c];
                m.shape_id.clear();  // as a fresh message
                copy_ints(cl.indices, cl.size, m.inliers);
                m.cloud.data.resize((size_t)cl.size * 4);  // the members' points in index order (:85-95)
                float* dst = m.cloud.data.data();
                const int32_t* idx = cl.indices;
                host_parallel(cl.size, [=](int64_t k0, int64_t k1) {
                    for (int64_t k = k0; k < k1; ++k) {
                        const float* p = xyz16 + 4 * (size_t)idx[k];
                        float* d = dst + 4 * k;
                        d[0] = p[0];
                        d[1] = p[1];
                        d[2] = p[2];
                        d[3] = 1.0f;
                    }
                });
                const int cnt = (int)cl.size + 1;  // Q7: the counter starts at 1
                m.x_centroid = cl.sum_xyz[0] / cnt;
                m.y_centroid = cl.sum_xyz[1] / cnt;
                m.z_centroid = cl.sum_xyz[2] / cnt;
            }
        }
    }
    res.cluster_objs.resize(found);
    return true;
}

// ransac_segmentation.cpp:175-199
bool SegmentationServices::callRansacPlaneSegmentation(const pitt_msgs::PointCloud& cloud,
                                                       const pitt_msgs::NormalCloud& norm,
                                                       pitt_msgs::PrimitiveSegmentation& out) {
    pitt_msgs::PrimitiveSegmentation srv;
    srv.request.cloud = cloud;
    srv.request.normals = norm;
    if (ransacPlaneDetaction(srv.request, srv.response)) {
        const int minInliers = 0;  // Q2: the /pitt/srv/plane_segmentation/min_inliers param is read but unused
        if (srv.response.inliers.size() > (size_t)minInliers) {
            out = srv;
            return true;
        }
    }
    return false;
}

// clustersAcquisition's per-cluster loop (ransac_segmentation.cpp:230-302) for all clusters at once:
// the four services with the parameters their handlers read, normals with k = 50 (pc_manager.cpp:18).
int SegmentationServices::classifyClusters(const float* x, const float* y, const float* z, const int64_t* offsets,
                                           const int64_t* counts, int32_t n, pitt_cluster_shape* out) {
    pitt_classify_params prm;
    pitt_classify_params_default(&prm);
    prm.plane = planeParams();
    prm.sphere = sphereParams();
    prm.cylinder = cylinderParams();
    prm.cone = coneParams();
    prm.cone_over_cylinder = DEFAULT_CONE_OVER_CYLINDER_PRIORITY;
    status_ = pitt_classify_clusters(ctx_, x, y, z, offsets, counts, n, &prm, out);
    return status_;
}

// ransac_segmentation.cpp:265-302.  size_t counts as the reference's; the cone rule compares
// (float)coneInl against (float)cylinderInl * 0.9f (size_t * float is float arithmetic).
int SegmentationServices::arbitratePrimitive(size_t sphereInl, size_t cylinderInl, size_t coneInl, size_t planeInl) {
    if (!planeInl && !sphereInl && !cylinderInl && !coneInl) return TXT_UNKNOWN_SHAPE_TAG;
    if (coneInl >= planeInl && coneInl >= sphereInl &&
        (float)coneInl >= (float)cylinderInl * DEFAULT_CONE_OVER_CYLINDER_PRIORITY)
        return TXT_CONE_SHAPE_TAG;
    if (cylinderInl >= planeInl && cylinderInl >= coneInl && cylinderInl >= sphereInl) return TXT_CYLINDER_SHAPE_TAG;
    if (planeInl >= coneInl && planeInl >= sphereInl && planeInl >= cylinderInl) return TXT_PLANE_SHAPE_TAG;
    if (sphereInl >= planeInl && sphereInl >= coneInl && sphereInl >= cylinderInl) return TXT_SPHERE_SHAPE_TAG;
    return TXT_UNKNOWN_SHAPE_TAG;
}

// callSupportFilter's request fields, obj_segmentation.cpp:164-177 (-1 / {-1} when a parameter is unset)
pitt_msgs::SupportSegmentation::Request SegmentationServices::supportRequest() {
    pitt_msgs::SupportSegmentation srv;
    params_.param(srvm::PARAM_NAME_MIN_ITERATIVE_CLOUD_PERCENTAGE, srv.request.min_iterative_cloud_percentual_size,
                  srvm::DEFAULT_SERVICE_PARAMETER_REQUEST_F);
    params_.param(srvm::PARAM_NAME_MIN_ITERATIVE_SUPPORT_PERCENTAGE, srv.request.min_iterative_plane_percentual_size,
                  srvm::DEFAULT_SERVICE_PARAMETER_REQUEST_F);
    params_.param(srvm::PARAM_NAME_HORIZONTAL_VARIANCE_THRESHOLD, srv.request.variance_threshold_for_horizontal,
                  srvm::DEFAULT_SERVICE_PARAMETER_REQUEST_F);
    params_.param(srvm::PARAM_NAME_RANSAC_IN_SHAPE_DISTANCE_POINT_THRESHOLD,
                  srv.request.ransac_distance_point_in_shape_threshold, srvm::DEFAULT_SERVICE_PARAMETER_REQUEST_F);
    params_.param(srvm::PARAM_NAME_RANSAC_MODEL_NORMAL_DISTANCE_WEIGHT, srv.request.ransac_model_normal_distance_weigth,
                  srvm::DEFAULT_SERVICE_PARAMETER_REQUEST_F);
    params_.param(srvm::PARAM_NAME_RANSAC_MAX_ITERATION_THRESHOLD, srv.request.ransac_max_iteration_threshold,
                  srvm::DEFAULT_SERVICE_PARAMETER_REQUEST);
    params_.param(srvm::PARAM_NAME_HORIZONTAL_AXIS, srv.request.horizontal_axis, std::vector<float>(1, -1.0f));
    params_.param(srvm::PARAM_NAME_SUPPORT_EDGE_REMOVE_OFFSET, srv.request.support_edge_remove_offset,
                  std::vector<float>(1, -1.0f));
    return srv.request;
}

pitt_support_params SegmentationServices::supportParams() { return resolveSupport(supportRequest()); }

pitt_cluster_params SegmentationServices::clusterParams() {
    pitt_cluster_params cp;
    pitt_cluster_params_default(&cp);
    int minInputSize = 30;
    params_.param(srvm::PARAM_NAME_CLUSTER_TOLERANCE, cp.tolerance, 0.03);
    params_.param(srvm::PARAM_NAME_CLUSTER_MIN_RATE, cp.min_rate, 0.01);
    params_.param(srvm::PARAM_NAME_CLUSTER_MAX_RATE, cp.max_rate, 0.99);
    params_.param(srvm::PARAM_NAME_CLUSTER_TOLERANCE, minInputSize, 30);  // Q6: the tolerance name
    cp.min_input_size = minInputSize;
    return cp;
}

int SegmentationServices::segmentObjectsDev(const float* x, const float* y, const float* z, int64_t n,
                                            pitt_scene* out) {
    const pitt_support_params sp = supportParams();
    const pitt_cluster_params cp = clusterParams();
    status_ = pitt_segment_objects_dev(ctx_, x, y, z, n, &sp, &cp, out);
    return status_;
}

// obj_segmentation.cpp:143-207 (callSupportFilter) and :261-312 (support -> cluster glue)
std::vector<pitt_msgs::ClustersOutput> SegmentationServices::segmentObjects(const pitt_msgs::PointCloud& world_cloud,
                                                                            const pitt_msgs::NormalCloud& normals) {
    pitt_msgs::SupportSegmentation srv;
    srv.request = supportRequest();
    srv.request.input_cloud = world_cloud;
    srv.request.input_norm = normals;
    std::vector<pitt_msgs::ClustersOutput> outs;
    if (!findSupports(srv.request, srv.response)) return outs;
    for (pitt_msgs::Support& s : srv.response.supports_description) {
        pitt_msgs::ClusterSegmentation cs;
        cs.request.cloud = s.on_support_cloud;
        clusterize(cs.request, cs.response);
        if (!cs.response.cluster_objs.empty()) {
            pitt_msgs::ClustersOutput o;
            o.cluster_objs = cs.response.cluster_objs;
            outs.push_back(std::move(o));
        }
    }
    return outs;
}

}  // namespace pitt

// ---- C ABI (pitt_srv.h) -----------------------------------------------------------------------
struct pitt_srv {
    pitt::SegmentationServices svc;
    pitt_msgs::SupportSegmentation::Response supports;
    pitt_msgs::ClusterSegmentation::Response clusters;
    std::vector<pitt_msgs::ClustersOutput> outputs;
    explicit pitt_srv(pitt_ctx* c) : svc(c) {}
};

namespace {
pitt_msgs::PointCloud cloud_from(const float* xyz16, int64_t n) {
    pitt_msgs::PointCloud c;
    if (n > 0) c.data.assign(xyz16, xyz16 + 4 * n);
    return c;
}
}  // namespace

extern "C" {

pitt_srv* pitt_srv_create(pitt_ctx* ctx) { return ctx ? new pitt_srv(ctx) : nullptr; }
void pitt_srv_destroy(pitt_srv* s) { delete s; }

int pitt_srv_param_set_int(pitt_srv* s, const char* k, int32_t v) {
    if (!s || !k) return PITT_E_INVALID;
    s->svc.params().set(k, (int)v);
    return PITT_OK;
}
int pitt_srv_param_set_double(pitt_srv* s, const char* k, double v) {
    if (!s || !k) return PITT_E_INVALID;
    s->svc.params().set(k, v);
    return PITT_OK;
}
int pitt_srv_param_set_list(pitt_srv* s, const char* k, const double* v, int32_t n) {
    if (!s || !k || (n > 0 && !v) || n < 0) return PITT_E_INVALID;
    s->svc.params().set(k, std::vector<double>(v, v + n));
    return PITT_OK;
}
int pitt_srv_param_erase(pitt_srv* s, const char* k) {
    if (!s || !k) return PITT_E_INVALID;
    s->svc.params().erase(k);
    return PITT_OK;
}

int pitt_srv_ransac_plane(pitt_srv* s, const float* xyz16, int64_t n, int64_t n_normals, int32_t* inliers_out,
                          int64_t* n_inliers, float* coefficients_out, int32_t* n_coefficients, float centroid_out[3]) {
    if (!s || (n > 0 && !xyz16) || n < 0 || !n_inliers || !n_coefficients) return PITT_E_INVALID;
    pitt_msgs::PrimitiveSegmentation srv;
    srv.request.cloud = cloud_from(xyz16, n);
    srv.request.normals.n = (size_t)n_normals;
    bool ok = s->svc.ransacPlaneDetaction(srv.request, srv.response);
    if (s->svc.last_status() < 0) return s->svc.last_status();
    *n_inliers = (int64_t)srv.response.inliers.size();
    *n_coefficients = (int32_t)srv.response.coefficients.size();
    if (inliers_out && !srv.response.inliers.empty())
        std::memcpy(inliers_out, srv.response.inliers.data(), srv.response.inliers.size() * 4);
    if (coefficients_out && !srv.response.coefficients.empty())
        std::memcpy(coefficients_out, srv.response.coefficients.data(), srv.response.coefficients.size() * 4);
    if (centroid_out) {
        centroid_out[0] = srv.response.x_centroid;
        centroid_out[1] = srv.response.y_centroid;
        centroid_out[2] = srv.response.z_centroid;
    }
    return ok ? 1 : 0;
}

int pitt_srv_ransac_sphere(pitt_srv* s, const float* xyz16, int64_t n, int64_t n_normals, int32_t* inliers_out,
                           int64_t* n_inliers, float* coefficients_out, int32_t* n_coefficients, float centroid_out[3]) {
    if (!s || (n > 0 && !xyz16) || n < 0 || !n_inliers || !n_coefficients) return PITT_E_INVALID;
    pitt_msgs::PrimitiveSegmentation srv;
    srv.request.cloud = cloud_from(xyz16, n);
    srv.request.normals.n = (size_t)n_normals;
    bool ok = s->svc.ransacSphereDetection(srv.request, srv.response);
    if (s->svc.last_status() < 0) return s->svc.last_status();
    *n_inliers = (int64_t)srv.response.inliers.size();
    *n_coefficients = (int32_t)srv.response.coefficients.size();
    if (inliers_out && !srv.response.inliers.empty())
        std::memcpy(inliers_out, srv.response.inliers.data(), srv.response.inliers.size() * 4);
    if (coefficients_out && !srv.response.coefficients.empty())
        std::memcpy(coefficients_out, srv.response.coefficients.data(), srv.response.coefficients.size() * 4);
    if (centroid_out) {
        centroid_out[0] = srv.response.x_centroid;
        centroid_out[1] = srv.response.y_centroid;
        centroid_out[2] = srv.response.z_centroid;
    }
    return ok ? 1 : 0;
}

int pitt_srv_ransac_cylinder(pitt_srv* s, const float* xyz16, int64_t n, const float* normals3, int64_t n_normals,
                             int32_t* inliers_out, int64_t* n_inliers, float* coefficients_out, int32_t* n_coefficients,
                             float centroid_out[3]) {
    if (!s || (n > 0 && !xyz16) || n < 0 || !n_inliers || !n_coefficients) return PITT_E_INVALID;
    if (n_normals == n && n > 0 && !normals3) return PITT_E_INVALID;
    pitt_msgs::PrimitiveSegmentation srv;
    srv.request.cloud = cloud_from(xyz16, n);
    srv.request.normals.n = (size_t)n_normals;
    if (normals3 && n_normals == n) srv.request.normals.data.assign(normals3, normals3 + 3 * n);
    bool ok = s->svc.ransacCylinderDetaction(srv.request, srv.response);
    if (s->svc.last_status() < 0) return s->svc.last_status();
    *n_inliers = (int64_t)srv.response.inliers.size();
    *n_coefficients = (int32_t)srv.response.coefficients.size();
    if (inliers_out && !srv.response.inliers.empty())
        std::memcpy(inliers_out, srv.response.inliers.data(), srv.response.inliers.size() * 4);
    if (coefficients_out && !srv.response.coefficients.empty())
        std::memcpy(coefficients_out, srv.response.coefficients.data(), srv.response.coefficients.size() * 4);
    if (centroid_out) {
        centroid_out[0] = srv.response.x_centroid;
        centroid_out[1] = srv.response.y_centroid;
        centroid_out[2] = srv.response.z_centroid;
    }
    return ok ? 1 : 0;
}

int pitt_srv_ransac_cone(pitt_srv* s, const float* xyz16, int64_t n, const float* normals3, int64_t n_normals,
                         int32_t* inliers_out, int64_t* n_inliers, float* coefficients_out, int32_t* n_coefficients,
                         float centroid_out[3]) {
    if (!s || (n > 0 && !xyz16) || n < 0 || !n_inliers || !n_coefficients) return PITT_E_INVALID;
    if (n_normals == n && n > 0 && !normals3) return PITT_E_INVALID;
    pitt_msgs::PrimitiveSegmentation srv;
    srv.request.cloud = cloud_from(xyz16, n);
    srv.request.normals.n = (size_t)n_normals;
    if (normals3 && n_normals == n) srv.request.normals.data.assign(normals3, normals3 + 3 * n);
    bool ok = s->svc.ransacConeDetaction(srv.request, srv.response);
    if (s->svc.last_status() < 0) return s->svc.last_status();
    *n_inliers = (int64_t)srv.response.inliers.size();
    *n_coefficients = (int32_t)srv.response.coefficients.size();
    if (inliers_out && !srv.response.inliers.empty())
        std::memcpy(inliers_out, srv.response.inliers.data(), srv.response.inliers.size() * 4);
    if (coefficients_out && !srv.response.coefficients.empty())
        std::memcpy(coefficients_out, srv.response.coefficients.data(), srv.response.coefficients.size() * 4);
    if (centroid_out) {
        centroid_out[0] = srv.response.x_centroid;
        centroid_out[1] = srv.response.y_centroid;
        centroid_out[2] = srv.response.z_centroid;
    }
    return ok ? 1 : 0;
}

int pitt_srv_call_ransac_plane(pitt_srv* s, const float* xyz16, int64_t n, int64_t n_normals, int32_t* inliers_out,
                               int64_t* n_inliers, float* coefficients_out, int32_t* n_coefficients) {
    if (!s || (n > 0 && !xyz16) || n < 0 || !n_inliers || !n_coefficients) return PITT_E_INVALID;
    pitt_msgs::NormalCloud nc;
    nc.n = (size_t)n_normals;
    pitt_msgs::PrimitiveSegmentation out;
    const bool ok = s->svc.callRansacPlaneSegmentation(cloud_from(xyz16, n), nc, out);
    if (s->svc.last_status() < 0) return s->svc.last_status();
    *n_inliers = ok ? (int64_t)out.response.inliers.size() : 0;
    *n_coefficients = ok ? (int32_t)out.response.coefficients.size() : 0;
    if (ok && inliers_out && !out.response.inliers.empty())
        std::memcpy(inliers_out, out.response.inliers.data(), out.response.inliers.size() * 4);
    if (ok && coefficients_out && !out.response.coefficients.empty())
        std::memcpy(coefficients_out, out.response.coefficients.data(), out.response.coefficients.size() * 4);
    return ok ? 1 : 0;
}

int pitt_srv_classify_clusters(pitt_srv* s, const float* x, const float* y, const float* z, const int64_t* offsets,
                               const int64_t* counts, int32_t n_clusters, pitt_cluster_shape* out) {
    if (!s) return PITT_E_INVALID;
    return s->svc.classifyClusters(x, y, z, offsets, counts, n_clusters, out);
}

int pitt_srv_arbitrate(int64_t sphere_inliers, int64_t cylinder_inliers, int64_t cone_inliers, int64_t plane_inliers) {
    if (sphere_inliers < 0 || cylinder_inliers < 0 || cone_inliers < 0 || plane_inliers < 0) return PITT_E_INVALID;
    return pitt::SegmentationServices::arbitratePrimitive((size_t)sphere_inliers, (size_t)cylinder_inliers,
                                                          (size_t)cone_inliers, (size_t)plane_inliers);
}

int pitt_srv_find_supports(pitt_srv* s, const float* xyz16, int64_t n, int64_t n_normals,
                           const pitt_srv_support_request* r, int32_t* n_supports, float used_out[13]) {
    if (!s || (n > 0 && !xyz16) || n < 0 || !r || !n_supports) return PITT_E_INVALID;
    pitt_msgs::SupportSegmentation srv;  // the cloud stays in the caller's array (findSupports(xyz16, ...))
    srv.request.min_iterative_cloud_percentual_size = r->min_iterative_cloud_percentual_size;
    srv.request.min_iterative_plane_percentual_size = r->min_iterative_plane_percentual_size;
    srv.request.variance_threshold_for_horizontal = r->variance_threshold_for_horizontal;
    srv.request.ransac_distance_point_in_shape_threshold = r->ransac_distance_point_in_shape_threshold;
    srv.request.ransac_model_normal_distance_weigth = r->ransac_model_normal_distance_weigth;
    srv.request.ransac_max_iteration_threshold = r->ransac_max_iteration_threshold;
    srv.request.horizontal_axis.assign(r->horizontal_axis, r->horizontal_axis + std::max(0, std::min(8, r->n_horizontal_axis)));
    srv.request.support_edge_remove_offset.assign(r->edge_remove_offset,
                                                  r->edge_remove_offset + std::max(0, std::min(8, r->n_edge_remove_offset)));
    // the service object's response is refilled in place (its buffers are reused call after call; a
    // failed call leaves it with no supports)
    bool ok = s->svc.findSupports(xyz16, (size_t)n, (size_t)n_normals, srv.request, s->supports);
    if (s->svc.last_status() < 0) return s->svc.last_status();
    *n_supports = (int32_t)s->supports.supports_description.size();
    if (used_out) {
        const auto& u = s->supports;
        used_out[0] = u.used_min_iterative_cloud_percentual_size;
        used_out[1] = u.used_min_iterative_plane_percentual_size;
        used_out[2] = u.used_max_variance_threshold_for_horizontal;
        used_out[3] = u.used_min_variance_threshold_for_horizontal;
        used_out[4] = (float)u.used_ransac_max_iteration_threshold;
        used_out[5] = u.used_ransac_distance_point_in_shape_threshold;
        used_out[6] = u.used_ransac_model_normal_distance_weigth;
        for (int i = 0; i < 3; ++i) {
            used_out[7 + i] = u.used_horizontal_axis[(size_t)i];
            used_out[10 + i] = u.used_support_edge_remove_offset[(size_t)i];
        }
    }
    return ok ? 1 : 0;
}

int pitt_srv_support_get(pitt_srv* s, int32_t k, int32_t* idx_map, float coef[4], int64_t* n_support,
                         int64_t* n_on_support) {
    if (!s || k < 0 || k >= (int32_t)s->supports.supports_description.size()) return PITT_E_INVALID;
    const pitt_msgs::Support& m = s->supports.supports_description[(size_t)k];
    if (idx_map) std::memcpy(idx_map, m.inliers.data(), m.inliers.size() * 4);
    if (coef) {
        coef[0] = m.support_coefficient_a;
        coef[1] = m.support_coefficient_b;
        coef[2] = m.support_coefficient_c;
        coef[3] = m.support_coefficient_d;
    }
    if (n_support) *n_support = (int64_t)m.support_cloud.size();
    if (n_on_support) *n_on_support = (int64_t)m.on_support_cloud.size();
    return PITT_OK;
}

int pitt_srv_support_cloud(pitt_srv* s, int32_t k, int32_t which, float* out) {
    if (!s || !out || k < 0 || k >= (int32_t)s->supports.supports_description.size()) return PITT_E_INVALID;
    const pitt_msgs::Support& m = s->supports.supports_description[(size_t)k];
    const pitt_msgs::PointCloud& c = which ? m.on_support_cloud : m.support_cloud;
    std::memcpy(out, c.data.data(), c.data.size() * 4);
    return PITT_OK;
}

int pitt_srv_clusterize(pitt_srv* s, const float* xyz16, int64_t n, int32_t* n_clusters) {
    if (!s || (n > 0 && !xyz16) || n < 0 || !n_clusters) return PITT_E_INVALID;
    // the cloud stays in the caller's array; the service object's response is refilled in place
    bool ok = s->svc.clusterize(xyz16, (size_t)n, s->clusters);
    if (s->svc.last_status() < 0) return s->svc.last_status();
    *n_clusters = (int32_t)s->clusters.cluster_objs.size();
    return ok ? 1 : 0;
}

int pitt_srv_cluster_get(pitt_srv* s, int32_t c, int32_t* inliers, int64_t* size, float centroid[3], float* xyz16_out) {
    if (!s || c < 0 || c >= (int32_t)s->clusters.cluster_objs.size()) return PITT_E_INVALID;
    const pitt_msgs::InliersCluster& m = s->clusters.cluster_objs[(size_t)c];
    if (inliers) std::memcpy(inliers, m.inliers.data(), m.inliers.size() * 4);
    if (size) *size = (int64_t)m.inliers.size();
    if (centroid) {
        centroid[0] = m.x_centroid;
        centroid[1] = m.y_centroid;
        centroid[2] = m.z_centroid;
    }
    if (xyz16_out) std::memcpy(xyz16_out, m.cloud.data.data(), m.cloud.data.size() * 4);
    return PITT_OK;
}

int pitt_srv_segment_objects(pitt_srv* s, const float* xyz16, int64_t n, int64_t n_normals, int32_t* n_outputs) {
    if (!s || (n > 0 && !xyz16) || n < 0 || !n_outputs) return PITT_E_INVALID;
    pitt_msgs::NormalCloud nc;
    nc.n = (size_t)n_normals;
    s->outputs = s->svc.segmentObjects(cloud_from(xyz16, n), nc);
    if (s->svc.last_status() < 0) return s->svc.last_status();
    *n_outputs = (int32_t)s->outputs.size();
    return 1;
}

int pitt_srv_output_size(pitt_srv* s, int32_t o, int32_t* n_clusters) {
    if (!s || !n_clusters || o < 0 || o >= (int32_t)s->outputs.size()) return PITT_E_INVALID;
    *n_clusters = (int32_t)s->outputs[(size_t)o].cluster_objs.size();
    return PITT_OK;
}

int pitt_srv_output_cluster(pitt_srv* s, int32_t o, int32_t c, int32_t* inliers, int64_t* size, float centroid[3]) {
    if (!s || o < 0 || o >= (int32_t)s->outputs.size()) return PITT_E_INVALID;
    const auto& objs = s->outputs[(size_t)o].cluster_objs;
    if (c < 0 || c >= (int32_t)objs.size()) return PITT_E_INVALID;
    const pitt_msgs::InliersCluster& m = objs[(size_t)c];
    if (inliers) std::memcpy(inliers, m.inliers.data(), m.inliers.size() * 4);
    if (size) *size = (int64_t)m.inliers.size();
    if (centroid) {
        centroid[0] = m.x_centroid;
        centroid[1] = m.y_centroid;
        centroid[2] = m.z_centroid;
    }
    return PITT_OK;
}

int pitt_srv_segment_objects_dev(pitt_srv* s, const float* x, const float* y, const float* z, int64_t n,
                                 pitt_scene* out) {
    if (!s || !out || n < 0 || (n > 0 && (!x || !y || !z))) return PITT_E_INVALID;
    return s->svc.segmentObjectsDev(x, y, z, n, out);
}

int pitt_srv_resolved_params(pitt_srv* s, pitt_support_params* sp, pitt_cluster_params* cp) {
    if (!s) return PITT_E_INVALID;
    if (sp) *sp = s->svc.supportParams();
    if (cp) *cp = s->svc.clusterParams();
    return PITT_OK;
}

}  // extern "C"
