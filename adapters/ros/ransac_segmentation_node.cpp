// ransac_segmentation_node.cpp -- drop-in for src/ransac_segmentation.cpp, the orchestrator node that
// tags every tracked cluster with the primitive shape that explains it best.
//
// Same interface as the reference node: it subscribes to "geometric_tracker/trackedCluster"
// (pitt_msgs::ClustersOutput, :352) and publishes pitt_msgs::TrackedShapes on
// "ransac_segmentation/trackedShapes" (:354), one TrackedShape per input cluster, in input order.
//
// The reference handles a frame cluster by cluster (clustersAcquisition, :223-343): k = 50 normals on the
// host (:233), then four blocking service calls -- sphere, cylinder, cone, plane, each a serialised
// cloud plus normals over TCPROS (:239-258) -- then the arbitration on the four inlier counts
// (:265-302).  Here the frame's clusters go to the MI355X together in one call,
// pitt_srv_classify_clusters: normals, the four services with the parameters their handlers read
// (/pitt/srv/{sphere,cylinder,cone,plane}_segmentation/*), and the same arbitration, for all clusters
// at once.  The published fields are the reference's (:315-328): the cluster's id and point-cloud
// centroid, the shape tag, and for a known shape the chosen service's centroid and coefficients.
// Visualisation (argv[1], :347) is out of scope.
#include <pitt_msgs/ClustersOutput.h>
#include <pitt_msgs/TrackedShapes.h>

#include "pitt_ros_common.hpp"

namespace {
const std::vector<std::string> kParams = {
    "/pitt/srv/sphere_segmentation/normal_distance_weight",   "/pitt/srv/sphere_segmentation/distance_th",
    "/pitt/srv/sphere_segmentation/max_iter_limit",           "/pitt/srv/sphere_segmentation/min_radius_limit",
    "/pitt/srv/sphere_segmentation/max_radius_limit",         "/pitt/srv/sphere_segmentation/eps_angle_th",
    "/pitt/srv/sphere_segmentation/min_opening_angle_deg",    "/pitt/srv/sphere_segmentation/max_opening_angle_deg",
    "/pitt/srv/cylinder_segmentation/normal_distance_weight", "/pitt/srv/cylinder_segmentation/distance_th",
    "/pitt/srv/cylinder_segmentation/max_iter_limit",         "/pitt/srv/cylinder_segmentation/min_radius_limit",
    "/pitt/srv/cylinder_segmentation/max_radius_limit",       "/pitt/srv/cylinder_segmentation/eps_angle_th",
    "/pitt/srv/cylinder_segmentation/min_opening_angle_deg",  "/pitt/srv/cylinder_segmentation/max_opening_angle_deg",
    "/pitt/srv/cone_segmentation/normal_distance_weight",     "/pitt/srv/cone_segmentation/distance_th",
    "/pitt/srv/cone_segmentation/max_iter_limit",             "/pitt/srv/cone_segmentation/min_radius_limit",
    "/pitt/srv/cone_segmentation/max_radius_limit",           "/pitt/srv/cone_segmentation/eps_angle_th",
    "/pitt/srv/cone_segmentation/min_opening_angle_deg",      "/pitt/srv/cone_segmentation/max_opening_angle_deg",
    "/pitt/srv/plane_segmentation/normal_distance_weight",    "/pitt/srv/plane_segmentation/distance_th",
    "/pitt/srv/plane_segmentation/max_iter_limit",            "/pitt/srv/plane_segmentation/eps_angle_th",
    "/pitt/srv/plane_segmentation/min_opening_angle_deg",     "/pitt/srv/plane_segmentation/max_opening_angle_deg"};

ros::NodeHandle* g_nh = nullptr;
ros::Publisher g_pub;

// returnPrimitiveNameFromTag, :204-212
const char* shape_name(int tag) {
    switch (tag) {
        case PITT_SHAPE_PLANE: return "plane";
        case PITT_SHAPE_SPHERE: return "sphere";
        case PITT_SHAPE_CONE: return "cone";
        case PITT_SHAPE_CYLINDER: return "cylinder";
        default: return "unknown";
    }
}

// the chosen service's response coefficients (its n_coef values) and centroid
void chosen(const pitt_cluster_shape& s, std::vector<float>* coef, const float** centroid) {
    int srv = -1;
    const float* c = nullptr;
    switch (s.tag) {
        case PITT_SHAPE_SPHERE: srv = PITT_SRV_SPHERE; c = s.sphere; break;
        case PITT_SHAPE_CYLINDER: srv = PITT_SRV_CYLINDER; c = s.cylinder; break;
        case PITT_SHAPE_CONE: srv = PITT_SRV_CONE; c = s.cone; break;
        case PITT_SHAPE_PLANE: srv = PITT_SRV_PLANE; c = s.plane; break;
        default: break;
    }
    coef->clear();
    *centroid = nullptr;
    if (srv < 0) return;
    coef->assign(c, c + s.n_coef[srv]);
    *centroid = s.est_centroid;
}
}  // namespace

// clustersAcquisition, ransac_segmentation.cpp:223-343
void clustersAcquisition(const pitt_msgs::ClustersOutputConstPtr& clusterObj) {
    const std::vector<pitt_msgs::InliersCluster>& clusters = clusterObj->cluster_objs;
    pitt_msgs::TrackedShapes outShapes;
    const int32_t nc = (int32_t)clusters.size();
    if (nc > 0) {
        pitt_ros::sync_params(*g_nh, kParams);
        // the frame's clusters as one SoA (cloudForRosMsg per cluster, :231)
        std::vector<int64_t> off((size_t)nc), cnt((size_t)nc);
        std::vector<std::vector<float>> pts((size_t)nc);
        int64_t total = 0;
        for (int32_t j = 0; j < nc; ++j) {
            pts[(size_t)j] = pitt_ros::to_xyz16(clusters[(size_t)j].cloud);
            off[(size_t)j] = total;
            cnt[(size_t)j] = (int64_t)pts[(size_t)j].size() / 4;
            total += cnt[(size_t)j];
        }
        std::vector<float> x((size_t)std::max<int64_t>(total, 1)), y(x.size()), z(x.size());
        for (int32_t j = 0; j < nc; ++j)
            for (int64_t i = 0; i < cnt[(size_t)j]; ++i) {
                const float* p = &pts[(size_t)j][(size_t)(4 * i)];
                x[(size_t)(off[(size_t)j] + i)] = p[0];
                y[(size_t)(off[(size_t)j] + i)] = p[1];
                z[(size_t)(off[(size_t)j] + i)] = p[2];
            }
        std::vector<pitt_cluster_shape> shapes((size_t)nc);
        const int rc = pitt_srv_classify_clusters(pitt_ros::node().srv, x.data(), y.data(), z.data(), off.data(),
                                                  cnt.data(), nc, shapes.data());
        if (rc != PITT_OK) {
            // the reference treats a failed service call as 0 inliers (:82, :118, :156, :197) and still
            // publishes one shape per cluster, which the arbitration then tags unknown (:298-302)
            ROS_ERROR_STREAM("ransac segmentation (MI355X) failed: " << pitt_last_error(pitt_ros::node().ctx));
            for (pitt_cluster_shape& s : shapes) {
                s = {};
                s.tag = PITT_SHAPE_UNKNOWN;
            }
        }
        for (int32_t j = 0; j < nc; ++j) {
            const pitt_cluster_shape& s = shapes[(size_t)j];
            const pitt_msgs::InliersCluster& in = clusters[(size_t)j];
            ROS_INFO("cluster_%d: %d #INLIER plane: %d sphere: %d cylinder: %d cone: %d selected: %s", in.shape_id,
                     (int)cnt[(size_t)j], s.inliers[PITT_SRV_PLANE], s.inliers[PITT_SRV_SPHERE],
                     s.inliers[PITT_SRV_CYLINDER], s.inliers[PITT_SRV_CONE], shape_name(s.tag));
            pitt_msgs::TrackedShape shape;
            shape.object_id = in.shape_id;
            shape.x_pc_centroid = in.x_centroid;
            shape.y_pc_centroid = in.y_centroid;
            shape.z_pc_centroid = in.z_centroid;
            shape.shape_tag = shape_name(s.tag);
            const float* c = nullptr;
            chosen(s, &shape.coefficients, &c);
            if (c) {
                shape.x_est_centroid = c[0];
                shape.y_est_centroid = c[1];
                shape.z_est_centroid = c[2];
            }
            outShapes.tracked_shapes.push_back(shape);
        }
    }
    ROS_INFO(" ------------------------------------ ");
    g_pub.publish(outShapes);
}

int main(int argc, char** argv) {
    ros::init(argc, argv, "ransac_segmentation");
    ros::NodeHandle nh;
    g_nh = &nh;
    if (argc > 1 && std::string(argv[1]) != "." && std::strtol(argv[1], nullptr, 0) != 0)
        ROS_WARN_STREAM("ransac_segmentation (MI355X): primitive visualisation is not available; flag ignored");
    pitt_ros::init_node();
    ros::Subscriber sub = nh.subscribe("geometric_tracker/trackedCluster", 10, clustersAcquisition);
    g_pub = nh.advertise<pitt_msgs::TrackedShapes>("ransac_segmentation/trackedShapes", 10);
    while (nh.ok()) ros::spinOnce();
    pitt_ros::shutdown_node();
    return 0;
}
