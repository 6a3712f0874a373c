// pitt_srv.hpp -- C++ mirror of the reference's segmentation-service layer, ROS-free.
//
// The reference's handlers (src/segmentation_services/*.cpp) are `bool h(Req&, Res&)` functions
// over pitt_msgs messages with parameters read from the ROS parameter server.  This header keeps
// that interface -- same handler names, message fields, parameter names, defaults, "-1 means
// default" sentinels and post-processing quirks -- and runs the arithmetic through the C ABI in
// pitt_seg.h (MI355X).  A maintainer with ROS available swaps `pitt_msgs::*` for the generated
// message types and `ParamServer` for ros::NodeHandle.
#pragma once
#include <cmath>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "pitt_seg.h"

namespace pitt_msgs {

// sensor_msgs/PointCloud2 carrying pcl::PointXYZ: point_step 16 (x, y, z, padding).
struct PointCloud {
    std::vector<float> data;  // 4 floats per point
    size_t size() const { return data.size() / 4; }
    float x(size_t i) const { return data[4 * i]; }
    float y(size_t i) const { return data[4 * i + 1]; }
    float z(size_t i) const { return data[4 * i + 2]; }
    void push_back(float px, float py, float pz) {
        data.push_back(px);
        data.push_back(py);
        data.push_back(pz);
        data.push_back(1.0f);
    }
};
// sensor_msgs/PointCloud2 carrying pcl::Normal (only its size matters on the plane path, A1).
struct NormalCloud {
    size_t n = 0;
    std::vector<float> data;  // (nx, ny, nz) per point when the handler reads the normals (cylinder)
    size_t size() const { return n; }
};

struct PrimitiveSegmentation {  // plane_segmentation_srv.cpp:27-74
    struct Request {
        PointCloud cloud;
        NormalCloud normals;
    } request;
    struct Response {
        std::vector<int32_t> inliers;
        std::vector<float> coefficients;
        float x_centroid = 0, y_centroid = 0, z_centroid = 0;  // never set for planes (Q3)
    } response;
};

struct Support {  // supports_segmentation_srv.cpp:313-325
    std::vector<int32_t> inliers;  // index map over the original cloud
    PointCloud support_cloud;
    PointCloud on_support_cloud;
    float support_coefficient_a = 0, support_coefficient_b = 0, support_coefficient_c = 0,
          support_coefficient_d = 0;
};

struct SupportSegmentation {  // supports_segmentation_srv.cpp:241-361
    struct Request {
        PointCloud input_cloud;
        NormalCloud input_norm;
        float min_iterative_cloud_percentual_size = -1.0f;
        float min_iterative_plane_percentual_size = -1.0f;
        float variance_threshold_for_horizontal = -1.0f;
        float ransac_distance_point_in_shape_threshold = -1.0f;
        float ransac_model_normal_distance_weigth = -1.0f;
        int32_t ransac_max_iteration_threshold = -1;
        std::vector<float> horizontal_axis;
        std::vector<float> support_edge_remove_offset;
    } request;
    struct Response {
        std::vector<Support> supports_description;
        float used_min_iterative_cloud_percentual_size = 0;
        float used_min_iterative_plane_percentual_size = 0;
        float used_max_variance_threshold_for_horizontal = 0;
        float used_min_variance_threshold_for_horizontal = 0;
        int32_t used_ransac_max_iteration_threshold = 0;
        float used_ransac_distance_point_in_shape_threshold = 0;
        float used_ransac_model_normal_distance_weigth = 0;
        std::vector<float> used_horizontal_axis;
        std::vector<float> used_support_edge_remove_offset;
    } response;
};

struct InliersCluster {  // cluster_segmentation_srv.cpp:95-101
    std::vector<int32_t> inliers;
    PointCloud cloud;
    float x_centroid = 0, y_centroid = 0, z_centroid = 0;
    std::string shape_id;
};

struct ClusterSegmentation {  // cluster_segmentation_srv.cpp:38-108
    struct Request {
        PointCloud cloud;
    } request;
    struct Response {
        std::vector<InliersCluster> cluster_objs;
    } response;
};

struct ClustersOutput {  // obj_segmentation.cpp:286-311
    std::vector<InliersCluster> cluster_objs;
};

}  // namespace pitt_msgs

namespace srvm {  // src/point_cloud_library/srv_manager.h:25-188 (names, sentinels)
const std::string SRV_NAME_SUPPORT_FILTER = "support_segmentation_srv";
const std::string SRV_NAME_CUSTER_FILTER = "cluster_Segmentation_srv";
const std::string SRV_NAME_RANSAC_PLANE_FILTER = "plane_segmentation_srv";
const std::string PARAM_NAME_CLUSTER_TOLERANCE = "/pitt/srv/cluster_segmentation/tolerance";
const std::string PARAM_NAME_CLUSTER_MIN_RATE = "/pitt/srv/cluster_segmentation/min_rate";
const std::string PARAM_NAME_CLUSTER_MAX_RATE = "/pitt/srv/cluster_segmentation/max_rate";
const std::string PARAM_NAME_CLUSTER_MIN_INPUT_SIZE = "/pitt/srv/cluster_segmentation/min_input_size";
const std::string PARAM_NAME_PLANE_NORMAL_DISTANCE_WEIGHT = "/pitt/srv/plane_segmentation/normal_distance_weight";
const std::string PARAM_NAME_PLANE_DISTANCE_TH = "/pitt/srv/plane_segmentation/distance_th";
const std::string PARAM_NAME_PLANE_MAX_ITERATION_LIMIT = "/pitt/srv/plane_segmentation/max_iter_limit";
const std::string PARAM_NAME_PLANE_EPS_ANGLE_TH = "/pitt/srv/plane_segmentation/eps_angle_th";
const std::string PARAM_NAME_PLANE_MIN_OPENING_ANGLE_DEGREE = "/pitt/srv/plane_segmentation/min_opening_angle_deg";
const std::string PARAM_NAME_PLANE_MAX_OPENING_ANGLE_DEGREE = "/pitt/srv/plane_segmentation/max_opening_angle_deg";
const std::string PARAM_NAME_PLANE_MIN_INLIERS = "/pitt/srv/plane_segmentation/min_inliers";
const std::string SRV_NAME_RANSAC_SPHERE_FILTER = "sphere_segmentation_srv";
const std::string SRV_NAME_RANSAC_CYLINDER_FILTER = "cylinder_segmentation_srv";
const std::string PARAM_NAME_CYLINDER_NORMAL_DISTANCE_WEIGHT = "/pitt/srv/cylinder_segmentation/normal_distance_weight";
const std::string PARAM_NAME_CYLINDER_DISTANCE_TH = "/pitt/srv/cylinder_segmentation/distance_th";
const std::string PARAM_NAME_CYLINDER_MAX_ITERATION_LIMIT = "/pitt/srv/cylinder_segmentation/max_iter_limit";
const std::string PARAM_NAME_CYLINDER_MIN_RADIUS_LIMIT = "/pitt/srv/cylinder_segmentation/min_radius_limit";
const std::string PARAM_NAME_CYLINDER_MAX_RADIUS_LIMIT = "/pitt/srv/cylinder_segmentation/max_radius_limit";
const std::string PARAM_NAME_CYLINDER_EPS_ANGLE_TH = "/pitt/srv/cylinder_segmentation/eps_angle_th";
const std::string PARAM_NAME_CYLINDER_MIN_OPENING_ANGLE_DEGREE = "/pitt/srv/cylinder_segmentation/min_opening_angle_deg";
const std::string PARAM_NAME_CYLINDER_MAX_OPENING_ANGLE_DEGREE = "/pitt/srv/cylinder_segmentation/max_opening_angle_deg";
const std::string SRV_NAME_RANSAC_CONE_FILTER = "cone_segmentation_srv";
const std::string PARAM_NAME_CONE_NORMAL_DISTANCE_WEIGHT = "/pitt/srv/cone_segmentation/normal_distance_weight";
const std::string PARAM_NAME_CONE_DISTANCE_TH = "/pitt/srv/cone_segmentation/distance_th";
const std::string PARAM_NAME_CONE_MAX_ITERATION_LIMIT = "/pitt/srv/cone_segmentation/max_iter_limit";
const std::string PARAM_NAME_CONE_MIN_RADIUS_LIMIT = "/pitt/srv/cone_segmentation/min_radius_limit";
const std::string PARAM_NAME_CONE_MAX_RADIUS_LIMIT = "/pitt/srv/cone_segmentation/max_radius_limit";
const std::string PARAM_NAME_CONE_EPS_ANGLE_TH = "/pitt/srv/cone_segmentation/eps_angle_th";
const std::string PARAM_NAME_CONE_MIN_OPENING_ANGLE_DEGREE = "/pitt/srv/cone_segmentation/min_opening_angle_deg";
const std::string PARAM_NAME_CONE_MAX_OPENING_ANGLE_DEGREE = "/pitt/srv/cone_segmentation/max_opening_angle_deg";
const std::string PARAM_NAME_CONE_MIN_INLIERS = "/pitt/srv/cone_segmentation/min_inliers";
const std::string PARAM_NAME_SPHERE_NORMAL_DISTANCE_WEIGHT = "/pitt/srv/sphere_segmentation/normal_distance_weight";
const std::string PARAM_NAME_SPHERE_DISTANCE_TH = "/pitt/srv/sphere_segmentation/distance_th";
const std::string PARAM_NAME_SPHERE_MAX_ITERATION_LIMIT = "/pitt/srv/sphere_segmentation/max_iter_limit";
const std::string PARAM_NAME_SPHERE_MIN_RADIUS_LIMIT = "/pitt/srv/sphere_segmentation/min_radius_limit";
const std::string PARAM_NAME_SPHERE_MAX_RADIUS_LIMIT = "/pitt/srv/sphere_segmentation/max_radius_limit";
const std::string PARAM_NAME_SPHERE_EPS_ANGLE_TH = "/pitt/srv/sphere_segmentation/eps_angle_th";
const std::string PARAM_NAME_SPHERE_MIN_OPENING_ANGLE_DEGREE = "/pitt/srv/sphere_segmentation/min_opening_angle_deg";
const std::string PARAM_NAME_SPHERE_MAX_OPENING_ANGLE_DEGREE = "/pitt/srv/sphere_segmentation/max_opening_angle_deg";
const std::string PARAM_NAME_MIN_ITERATIVE_CLOUD_PERCENTAGE = "/pitt/srv/supports_segmentation/min_iter_cloud_percent";
const std::string PARAM_NAME_MIN_ITERATIVE_SUPPORT_PERCENTAGE = "/pitt/srv/supports_segmentation/min_iter_support_percent";
const std::string PARAM_NAME_HORIZONTAL_VARIANCE_THRESHOLD = "/pitt/srv/supports_segmentation/horizontal_variance_th";
const std::string PARAM_NAME_RANSAC_IN_SHAPE_DISTANCE_POINT_THRESHOLD = "/pitt/srv/supports_segmentation/in_shape_distance_th";
const std::string PARAM_NAME_RANSAC_MODEL_NORMAL_DISTANCE_WEIGHT = "/pitt/srv/supports_segmentation/normal_distance_weight";
const std::string PARAM_NAME_RANSAC_MAX_ITERATION_THRESHOLD = "/pitt/srv/supports_segmentation/max_iter";
const std::string PARAM_NAME_HORIZONTAL_AXIS = "/pitt/srv/supports_segmentation/horizontal_axis";
const std::string PARAM_NAME_SUPPORT_EDGE_REMOVE_OFFSET = "/pitt/srv/supports_segmentation/edge_remove_offset";
const int DEFAULT_SERVICE_PARAMETER_REQUEST = -1;
const float DEFAULT_SERVICE_PARAMETER_REQUEST_F = -1.0f;

inline float getServiceFloatParameter(float input, const float defaultValue) {
    return input >= 0.0f ? input : defaultValue;
}
inline int getServiceIntParameter(int input, const int defaultValue) { return input >= 0 ? input : defaultValue; }
inline std::vector<float> getService3DArrayParameter(const std::vector<float>& input, const float defaultValue[3]) {
    return input.size() == 3 ? input : std::vector<float>(defaultValue, defaultValue + 3);
}
}  // namespace srvm

namespace pitt {

// ransac_segmentation.cpp:37, :42-46
const float DEFAULT_CONE_OVER_CYLINDER_PRIORITY = 0.9f;
enum { TXT_UNKNOWN_SHAPE_TAG = 0, TXT_PLANE_SHAPE_TAG = 1, TXT_SPHERE_SHAPE_TAG = 2, TXT_CONE_SHAPE_TAG = 3,
       TXT_CYLINDER_SHAPE_TAG = 4 };

// ROS parameter server stand-in with roscpp's typed-read rules: a double read as int is rounded
// (fmod < 0.5 -> floor, else ceil), an int read as double converts, a list reads as vector<float>;
// any other type mismatch leaves the default (NodeHandle::param).
class ParamServer {
public:
    enum Kind { INT, DOUBLE, STRING, LIST, BOOL };
    struct Value {
        Kind kind = DOUBLE;
        int64_t i = 0;
        double d = 0;
        std::string s;
        std::vector<double> list;
    };
    void set(const std::string& k, int v) { Value x; x.kind = INT; x.i = v; m_[k] = x; }
    void set(const std::string& k, double v) { Value x; x.kind = DOUBLE; x.d = v; m_[k] = x; }
    void set(const std::string& k, const std::string& v) { Value x; x.kind = STRING; x.s = v; m_[k] = x; }
    void set(const std::string& k, const std::vector<double>& v) { Value x; x.kind = LIST; x.list = v; m_[k] = x; }
    void erase(const std::string& k) { m_.erase(k); }
    void clear() { m_.clear(); }

    bool get(const std::string& k, double& out) const;
    bool get(const std::string& k, float& out) const;
    bool get(const std::string& k, int& out) const;
    bool get(const std::string& k, std::vector<float>& out) const;
    template <class T, class D>
    void param(const std::string& k, T& out, const D& def) const {
        if (!get(k, out)) out = def;
    }

private:
    std::map<std::string, Value> m_;
};

// The three services plus the clients' glue, bound to one MI355X context.
class SegmentationServices {
public:
    explicit SegmentationServices(pitt_ctx* ctx) : ctx_(ctx) {}
    ParamServer& params() { return params_; }
    int last_status() const { return status_; }

    // plane_segmentation_srv.cpp:27
    bool ransacPlaneDetaction(pitt_msgs::PrimitiveSegmentation::Request& req,
                              pitt_msgs::PrimitiveSegmentation::Response& res);
    // cylinder_segmentation_srv.cpp:82-216 (the model, then the axis height and centroid)
    bool ransacCylinderDetaction(pitt_msgs::PrimitiveSegmentation::Request& req,
                                 pitt_msgs::PrimitiveSegmentation::Response& res);
    // cone_segmentation_srv.cpp:83-216 (the model, then the axis height and the 3/4-height centroid)
    bool ransacConeDetaction(pitt_msgs::PrimitiveSegmentation::Request& req,
                             pitt_msgs::PrimitiveSegmentation::Response& res);
    // sphere_segmentation_srv.cpp:29-96
    bool ransacSphereDetection(pitt_msgs::PrimitiveSegmentation::Request& req,
                               pitt_msgs::PrimitiveSegmentation::Response& res);
    // supports_segmentation_srv.cpp:241
    bool findSupports(pitt_msgs::SupportSegmentation::Request& req, pitt_msgs::SupportSegmentation::Response& res);
    // cluster_segmentation_srv.cpp:38
    bool clusterize(pitt_msgs::ClusterSegmentation::Request& req, pitt_msgs::ClusterSegmentation::Response& res);
    // the two handlers on a cloud given as PointXYZ bytes (4 floats per point) rather than inside the
    // request (the flat C ABI and the ROS nodes pass their converted message this way: no copy of the
    // cloud into a request); the request's cloud fields are not read
    bool findSupports(const float* xyz16, size_t n, size_t n_normals, const pitt_msgs::SupportSegmentation::Request& req,
                      pitt_msgs::SupportSegmentation::Response& res);
    bool clusterize(const float* xyz16, size_t n, pitt_msgs::ClusterSegmentation::Response& res);

    // ransac_segmentation.cpp:175-199: accept iff the response holds > 0 inliers (local minInliers = 0, Q2)
    bool callRansacPlaneSegmentation(const pitt_msgs::PointCloud& cloud, const pitt_msgs::NormalCloud& norm,
                                     pitt_msgs::PrimitiveSegmentation& out);
    // ransac_segmentation.cpp:265-302: the primitive a cluster is tagged with, from the four services'
    // inlier counts (0 when a service call failed or returned no inliers): cone first (with the 0.9f
    // priority over the cylinder, :37, compared in float), then cylinder, plane, sphere; all zero or
    // no rule -> unknown.  Tags as ransac_segmentation.cpp:42-46.
    static int arbitratePrimitive(size_t sphereInl, size_t cylinderInl, size_t coneInl, size_t planeInl);
    // ransac_segmentation.cpp:230-302 for all of a frame's clusters in one pass (pitt_classify_clusters)
    // with the parameters the four handlers read; returns the pitt status
    int classifyClusters(const float* x, const float* y, const float* z, const int64_t* offsets,
                         const int64_t* counts, int32_t n, pitt_cluster_shape* out);
    // the parameters each primitive handler reads from the parameter server on every call
    pitt_sac_params planeParams();
    pitt_sphere_params sphereParams();
    pitt_cylinder_params cylinderParams();
    pitt_cone_params coneParams();
    // obj_segmentation.cpp:143-207 + :261-312: supports (request fields from params, -1 = default),
    // then clusters per support; one ClustersOutput per support with at least one cluster.
    std::vector<pitt_msgs::ClustersOutput> segmentObjects(const pitt_msgs::PointCloud& world_cloud,
                                                          const pitt_msgs::NormalCloud& normals);
    // callSupportFilter's request (obj_segmentation.cpp:147-177: each field from its parameter, -1 when
    // unset) as findSupports resolves it (initializeInputParameters, supports_segmentation_srv.cpp:70-86)
    pitt_support_params supportParams();
    // the parameters clusterize reads per call (cluster_segmentation_srv.cpp:44-50, Q6)
    pitt_cluster_params clusterParams();
    // segmentObjects with the world cloud in HBM (device SoA x/y/z): pitt_segment_objects_dev with the
    // two parameter sets above; the scene stays valid until the next call on the context.  Returns the
    // pitt status.
    int segmentObjectsDev(const float* x, const float* y, const float* z, int64_t n, pitt_scene* out);

private:
    static pitt_support_params resolveSupport(const pitt_msgs::SupportSegmentation::Request& req);
    pitt_msgs::SupportSegmentation::Request supportRequest();

    pitt_ctx* ctx_;
    ParamServer params_;
    int status_ = PITT_OK;
};

}  // namespace pitt
