// obj_segmentation_node.cpp -- drop-in for src/obj_segmentation.cpp, the orchestrator node that turns
// each camera cloud into clusters of objects standing on horizontal supports.
//
// Same interface as the reference node: the raw cloud topic and the flags come from argv (main,
// :326-360: topic, four visualisation flags, centroid log path; "." selects a default), the TF between
// /pitt/ref_frame/input_cloud and /pitt/ref_frame/output_cloud is polled in the main loop (:393-433),
// and one pitt_msgs::ClustersOutput per support with at least one cluster is published on
// "obj_segmentation/ClusterOutput" (:286-312).
//
// What changes is where the frame lives.  The reference sends the cloud through three ROS services per
// frame and then one cluster service call per support, each a serialised PointCloud2 over TCPROS
// (:91, :128, :177, :220).  Here the payload crosses PCIe once and stays in HBM:
//   fromROSMsg (pc_manager.cpp:94-104)             -> pitt_unpack_pointcloud2
//   downSampling, 1 cm VoxelGrid (:238)           -> pitt_voxel_grid (PCL's leaf order, bit-exact)
//   callDeepFilter (:241, :75-106)                -> pitt_deep_filter (threshold parameter, -1 = 3 m)
//   callArmFilter (:244, :108-139)                -> the reference's arm_filter_srv over ROS (robot-specific,
//                                                   out of scope); skipped with ~arm_filter false
//   transformPointCloud (:248)                    -> pitt_transform_cloud
//   > MIN_POINT_IN_ORIGINAL_CLOUD points (:251)
//   callSupportFilter + callClusterSegmentation
//   per support (:261-312)                        -> pitt_srv_segment_objects_dev (supports, then every
//                                                   support's clusters; the parameters as the services read them)
// Only the published clusters (indices, points, centroids) come back to the host.  The normals the
// reference estimates for the support call (:253) are not computed: the support service's plane model
// never reads them and their count always matches the cloud's (pitt_srv.h).  Visualisation is out of
// scope; the raw centroid log (ROS_INFO and the optional file, :305-322) is kept.
#include <pitt_msgs/ArmFilter.h>
#include <pitt_msgs/ClustersOutput.h>
#include <tf/transform_listener.h>

#include <cstdio>
#include <ctime>
#include <fstream>

#include "pitt_ros_common.hpp"

namespace {
const std::string kOutTopic = "obj_segmentation/ClusterOutput";           // srv_manager.h:115
const std::string kDefaultTopic = "/camera/depth/points";                 // :100
const std::string kDeepThreshold = "/pitt/service/deep_filter/z_threshold";  // :37
const std::string kInputFrame = "/pitt/ref_frame/input_cloud", kOutputFrame = "/pitt/ref_frame/output_cloud";
const std::string kDefaultInputFrame = "/camera_depth_optical_frame", kDefaultOutputFrame = "/world";
const int kMinPointInOriginalCloud = 30;  // obj_segmentation.cpp:55
const float kLeaf = 0.01f;                // pc_manager.cpp:19

const std::vector<std::string> kParams = {
    // callSupportFilter's request fields (obj_segmentation.cpp:156-174)
    "/pitt/srv/supports_segmentation/min_iter_cloud_percent", "/pitt/srv/supports_segmentation/min_iter_support_percent",
    "/pitt/srv/supports_segmentation/horizontal_variance_th", "/pitt/srv/supports_segmentation/in_shape_distance_th",
    "/pitt/srv/supports_segmentation/normal_distance_weight", "/pitt/srv/supports_segmentation/max_iter",
    "/pitt/srv/supports_segmentation/horizontal_axis", "/pitt/srv/supports_segmentation/edge_remove_offset",
    // the cluster service's (cluster_segmentation_srv.cpp:44-50)
    "/pitt/srv/cluster_segmentation/tolerance", "/pitt/srv/cluster_segmentation/min_rate",
    "/pitt/srv/cluster_segmentation/max_rate", "/pitt/srv/cluster_segmentation/min_input_size"};

ros::NodeHandle* g_nh = nullptr;
ros::Publisher g_pub;
bool g_arm_filter = true;
std::string g_log_path;
long g_scan_id = 0;
float g_transform[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};  // pclTransform, identity first
pitt_ros::DevBuf g_payload, g_planes;

// srvm::getStringParameter / getBoolParameter / getPathParameter (srv_manager.h:129-161): "." = default
std::string arg_string(const char* a, const std::string& def) { return std::string(a) == "." ? def : a; }
bool arg_bool(const char* a, bool def) { return std::string(a) == "." ? def : std::strtol(a, nullptr, 0) != 0; }
std::string arg_path(const char* a, const std::string& def) {
    std::string s(a);
    if (s == ".") return def;
    const size_t dd = s.find("..");
    if (dd != std::string::npos) {  // "..": the path plus the date (PCManager::getFomrattedData)
        char buf[64];
        const std::time_t t = std::time(nullptr);
        std::strftime(buf, sizeof buf, "%Y-%m-%d_%H-%M-%S", std::localtime(&t));
        return s.substr(0, s.size() - 2) + buf;
    }
    return s;
}

// PCManager::writeToFile(txt, path, append = true), pc_manager.cpp:220-238
void write_to_file(const std::string& txt, const std::string& path) {
    if (path.empty()) return;
    std::ofstream os(path.c_str(), std::ios_base::app | std::ios_base::out);
    if (!os) ROS_ERROR_STREAM(" !! Error writing to: " << path);
    else os << txt;
}

// lexical_cast<std::string>(float): nine significant digits
std::string fstr(float v) {
    char b[32];
    std::snprintf(b, sizeof b, "%.9g", v);
    return b;
}

bool ok_or_log(pitt_ctx* ctx, int rc, const char* what) {
    if (rc != PITT_OK) ROS_ERROR_STREAM(what << " (MI355X) failed: " << pitt_last_error(ctx));
    return rc == PITT_OK;
}

// Device SoA planes <-> PointXYZ arrays on the host (the arm filter's round trip).
bool download_xyz16(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, std::vector<float>& out) {
    std::vector<float> s((size_t)n * 3);
    out.assign((size_t)n * 4, 0.0f);
    if (n == 0) return true;
    if (pitt_memcpy(ctx, s.data(), x, n * 4) != PITT_OK || pitt_memcpy(ctx, s.data() + n, y, n * 4) != PITT_OK ||
        pitt_memcpy(ctx, s.data() + 2 * n, z, n * 4) != PITT_OK)
        return false;
    for (int64_t i = 0; i < n; ++i) {
        out[4 * i] = s[i];
        out[4 * i + 1] = s[n + i];
        out[4 * i + 2] = s[2 * n + i];
        out[4 * i + 3] = 1.0f;
    }
    return true;
}

// callArmFilter, obj_segmentation.cpp:108-139: the four box parameters, the service call, the armless
// cloud back into the planes (capacity n).  False when the call fails: the frame is dropped (:244).
bool call_arm_filter(pitt_ctx* ctx, float* x, float* y, float* z, int64_t* n) {
    pitt_msgs::ArmFilter srv;
    const std::vector<float> unset(1, -1.0f);  // DEFAULT_SERVICE_VEC_PARAMETER_REQUEST
    g_nh->param("/pitt/srv/arm_filter/min_forearm_box", srv.request.forearm_bounding_box_min_value, unset);
    g_nh->param("/pitt/srv/arm_filter/max_forearm_box", srv.request.forearm_bounding_box_max_value, unset);
    g_nh->param("/pitt/srv/arm_filter/min_elbow_box", srv.request.elbow_bounding_box_min_value, unset);
    g_nh->param("/pitt/srv/arm_filter/max_elbow_box", srv.request.elbow_bounding_box_max_value, unset);
    std::vector<float> host;
    if (!download_xyz16(ctx, x, y, z, *n, host)) return false;
    srv.request.input_cloud = pitt_ros::from_xyz16(host.data(), *n);
    ros::ServiceClient client = g_nh->serviceClient<pitt_msgs::ArmFilter>("arm_filter_srv");
    if (!client.call(srv)) {
        ROS_ERROR_STREAM(" error on calling service " << client.getService());
        return false;
    }
    const std::vector<float> armless = pitt_ros::to_xyz16(srv.response.armless_cloud);
    const int64_t m = std::min<int64_t>((int64_t)armless.size() / 4, *n);  // a crop never adds points
    std::vector<float> s((size_t)m * 3);
    for (int64_t i = 0; i < m; ++i)
        for (int k = 0; k < 3; ++k) s[(size_t)(k * m + i)] = armless[(size_t)(4 * i + k)];
    if (m > 0 && (pitt_memcpy(ctx, x, s.data(), m * 4) != PITT_OK || pitt_memcpy(ctx, y, s.data() + m, m * 4) != PITT_OK ||
                  pitt_memcpy(ctx, z, s.data() + 2 * m, m * 4) != PITT_OK))
        return false;
    *n = m;
    return true;
}

// The published clusters of one support: members (on-support indices, ascending), their points, and
// the service's centroid sum / (size + 1) (cluster_segmentation_srv.cpp:92-101, Q7).
bool support_output(pitt_ctx* ctx, const pitt_scene& S, int32_t s, const std::vector<int32_t>& members,
                    pitt_msgs::ClustersOutput* out) {
    const pitt_support_dev& su = S.supports.supports[s];
    const int64_t m = su.n_on_support;
    std::vector<float> on((size_t)m * 3);
    for (int k = 0; k < 3 && m > 0; ++k)
        if (pitt_memcpy(ctx, on.data() + k * m, su.on_support_xyz + k * su.stride, m * 4) != PITT_OK) return false;
    for (int32_t o = 0; o < S.n_objects; ++o) {
        const pitt_object& ob = S.objects[o];
        if (ob.support != s) continue;
        pitt_msgs::InliersCluster cl;
        cl.inliers.assign(members.begin() + ob.offset, members.begin() + ob.offset + ob.size);
        std::vector<float> pts((size_t)ob.size * 4);
        for (int64_t k = 0; k < ob.size; ++k) {
            const int32_t i = cl.inliers[(size_t)k];
            pts[4 * k] = on[(size_t)i];
            pts[4 * k + 1] = on[(size_t)(m + i)];
            pts[4 * k + 2] = on[(size_t)(2 * m + i)];
            pts[4 * k + 3] = 1.0f;
        }
        cl.cloud = pitt_ros::from_xyz16(pts.data(), ob.size);
        const int cnt = (int)ob.size + 1;
        cl.x_centroid = ob.sum_xyz[0] / cnt;
        cl.y_centroid = ob.sum_xyz[1] / cnt;
        cl.z_centroid = ob.sum_xyz[2] / cnt;
        out->cluster_objs.push_back(cl);
    }
    return true;
}

// The whole device chain of one frame; false when a stage fails or drops the frame.
bool segment_frame(const sensor_msgs::PointCloud2& msg, std::string* log) {
    pitt_ctx* ctx = pitt_ros::node().ctx;
    int off[3] = {-1, -1, -1};
    for (const sensor_msgs::PointField& f : msg.fields) {
        if (f.datatype != sensor_msgs::PointField::FLOAT32) continue;
        if (f.name == "x") off[0] = (int)f.offset;
        if (f.name == "y") off[1] = (int)f.offset;
        if (f.name == "z") off[2] = (int)f.offset;
    }
    int64_t n = pitt_ros::n_points(msg);
    if (off[0] < 0 || off[1] < 0 || off[2] < 0) n = 0;  // fromROSMsg without x/y/z: an empty cloud
    // four SoA clouds of capacity n: raw, voxel, closer (reused for the armless cloud), world
    float* planes = (float*)g_planes.get((size_t)std::max<int64_t>(n, 1) * 48);
    void* payload = g_payload.get(std::max<size_t>(msg.data.size(), 16));
    if (!planes || !payload) return false;
    float *raw = planes, *vox = planes + 3 * n, *cl = planes + 6 * n, *w = planes + 9 * n;
    if (n > 0) {
        if (!ok_or_log(ctx, pitt_memcpy(ctx, payload, msg.data.data(), (int64_t)msg.data.size()), "payload upload") ||
            !ok_or_log(ctx,
                       pitt_unpack_pointcloud2(ctx, payload, (int64_t)msg.data.size(), (int32_t)msg.width,
                                               (int32_t)msg.height, (int32_t)msg.point_step, (int64_t)msg.row_step,
                                               off[0], off[1], off[2], raw, raw + n, raw + 2 * n),
                       "PointCloud2 unpack"))
            return false;
    }
    int64_t nv = 0;
    int32_t flags = 0;
    if (!ok_or_log(ctx,
                   pitt_voxel_grid(ctx, raw, raw + n, raw + 2 * n, n, kLeaf, kLeaf, kLeaf, PITT_VOXEL_ORDER_PCL, vox,
                                   vox + n, vox + 2 * n, &nv, &flags),
                   "voxel grid"))
        return false;
    float deep = -1.0f;  // DEFAULT_SERVICE_PARAMETER_REQUEST_F
    g_nh->param(kDeepThreshold, deep, -1.0f);
    int64_t nc = 0;
    if (!ok_or_log(ctx,
                   pitt_deep_filter(ctx, vox, vox + n, vox + 2 * n, nv, deep, cl, cl + n, cl + 2 * n, &nc, nullptr,
                                    nullptr, nullptr, nullptr, nullptr),
                   "deep filter"))
        return false;
    if (g_arm_filter && !call_arm_filter(ctx, cl, cl + n, cl + 2 * n, &nc)) return false;
    if (!ok_or_log(ctx, pitt_transform_cloud(ctx, cl, cl + n, cl + 2 * n, nc, g_transform, 1, w, w + n, w + 2 * n),
                   "transform"))
        return false;
    if (nc <= kMinPointInOriginalCloud) return true;  // :251, nothing published
    pitt_ros::sync_params(*g_nh, kParams);
    pitt_scene S;
    const int rc = pitt_srv_segment_objects_dev(pitt_ros::node().srv, w, w + n, w + 2 * n, nc, &S);
    if (!ok_or_log(ctx, rc, "support / cluster segmentation")) return false;
    int64_t n_members = 0;
    for (int32_t o = 0; o < S.n_objects; ++o) n_members = std::max(n_members, S.objects[o].offset + S.objects[o].size);
    std::vector<int32_t> members((size_t)n_members);
    if (n_members > 0 && !ok_or_log(ctx, pitt_memcpy(ctx, members.data(), S.indices, n_members * 4), "cluster copy"))
        return false;
    for (int32_t s = 0; s < S.supports.n_supports; ++s) {
        pitt_msgs::ClustersOutput out;
        if (!support_output(ctx, S, s, members, &out)) return false;
        if (out.cluster_objs.empty()) continue;  // :286, a support without clusters publishes nothing
        for (size_t j = 0; j < out.cluster_objs.size(); ++j) {
            const pitt_msgs::InliersCluster& c = out.cluster_objs[j];
            *log += std::to_string(g_scan_id) + ", " + std::to_string(s) + ", " + std::to_string(j) + ", " +
                    fstr(c.x_centroid) + ", " + fstr(c.y_centroid) + ", " + fstr(c.z_centroid) + ";\n";
        }
        g_pub.publish(out);
    }
    return true;
}
}  // namespace

// depthAcquisition, obj_segmentation.cpp:229-322
void depthAcquisition(const sensor_msgs::PointCloud2ConstPtr& input) {
    std::string log;
    segment_frame(*input, &log);
    ROS_INFO_STREAM("raw clusters data: [scan id, support idx, cluster idx, centroid X, cenntroid Y, centroid Z;\\n]"
                    << std::endl
                    << log);
    write_to_file(log, g_log_path);
    g_scan_id += 1;
}

int main(int argc, char** argv) {
    ros::init(argc, argv, "obj_segmentation");
    ros::NodeHandle node, pnh("~");
    g_nh = &node;
    std::string topic = kDefaultTopic;
    bool show = false;
    if (argc == 7) {  // :331-346
        topic = arg_string(argv[1], kDefaultTopic);
        for (int a = 2; a <= 5; ++a) show = show || arg_bool(argv[a], false);
        g_log_path = arg_path(argv[6], "");
    } else {
        ROS_WARN_STREAM("input parameter given to \"obj_segmentation\" are not correct. Setting all to the default value.");
    }
    if (show) ROS_WARN_STREAM("obj_segmentation (MI355X): cloud visualisation is not available; flags ignored");
    pnh.param("arm_filter", g_arm_filter, true);
    ROS_INFO_STREAM("obj_segmentation (MI355X) initialised with:" << std::endl
                    << "\t input raw cloud topic name: \t\"" << topic << "\"" << std::endl
                    << "\t arm filter service: \t" << (g_arm_filter ? "called" : "skipped") << std::endl
                    << "\t raw centroid log file path (empty means do not print): \"" << g_log_path << "\"");
    write_to_file("scan id, support idx, cluster idx, centroid X, centroid Y, centroid Z;\n", g_log_path);
    pitt_ros::init_node();
    ros::Subscriber sub = node.subscribe(topic, 1, depthAcquisition);
    g_pub = node.advertise<pitt_msgs::ClustersOutput>(kOutTopic, 10);
    tf::TransformListener listener;
    while (node.ok()) {  // :393-433: the camera -> world transform, refreshed between callbacks
        try {
            std::string in_frame, out_frame;
            node.param<std::string>(kInputFrame, in_frame, kDefaultInputFrame);
            node.param<std::string>(kOutputFrame, out_frame, kDefaultOutputFrame);
            if (in_frame == ".") in_frame = kDefaultInputFrame;
            if (out_frame == ".") out_frame = kDefaultOutputFrame;
            tf::StampedTransform t;
            listener.waitForTransform(out_frame, in_frame, ros::Time(0), ros::Duration(2.0));
            listener.lookupTransform(out_frame, in_frame, ros::Time(0), t);
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c) g_transform[4 * r + c] = (float)t.getBasis()[r][c];
            }
            g_transform[3] = (float)t.getOrigin().x();
            g_transform[7] = (float)t.getOrigin().y();
            g_transform[11] = (float)t.getOrigin().z();
        } catch (tf::TransformException& ex) {
            ROS_WARN_ONCE("%s", ex.what());  // the previous (initially identity) transform stays
        }
        ros::spinOnce();
    }
    pitt_ros::shutdown_node();
    return 0;
}
