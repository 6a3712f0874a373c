// sphere_segmentation_node.cpp -- drop-in for src/segmentation_services/sphere_segmentation_srv.cpp.
// Same service name (srvm::SRV_NAME_RANSAC_SPHERE_FILTER = "sphere_segmentation_srv"), same request /
// response, same /pitt/srv/sphere_segmentation/* parameters (read per call, :40-55); the handler body
// (SACSegmentationFromNormals with SACMODEL_SPHERE at :58-73, the conversions at :76-77, the centre as
// the centroid at :79-83) runs through pitt_srv_ransac_sphere on the MI355X.
#include <pitt_msgs/PrimitiveSegmentation.h>

#include "pitt_ros_common.hpp"

namespace {
ros::NodeHandle* g_nh = nullptr;
const std::vector<std::string> kParams = {
    "/pitt/srv/sphere_segmentation/normal_distance_weight", "/pitt/srv/sphere_segmentation/distance_th",
    "/pitt/srv/sphere_segmentation/max_iter_limit",         "/pitt/srv/sphere_segmentation/min_radius_limit",
    "/pitt/srv/sphere_segmentation/max_radius_limit",       "/pitt/srv/sphere_segmentation/eps_angle_th",
    "/pitt/srv/sphere_segmentation/min_opening_angle_deg",  "/pitt/srv/sphere_segmentation/max_opening_angle_deg"};
}  // namespace

bool ransacSphereDetection(pitt_msgs::PrimitiveSegmentation::Request& req,
                           pitt_msgs::PrimitiveSegmentation::Response& res) {
    pitt_ros::sync_params(*g_nh, kParams);
    const std::vector<float> cloud = pitt_ros::to_xyz16(req.cloud);
    const int64_t n = (int64_t)cloud.size() / 4;
    std::vector<int32_t> inl((size_t)std::max<int64_t>(n, 1));
    int64_t n_inl = 0;
    float coef[4] = {0, 0, 0, 0}, centroid[3] = {0, 0, 0};
    int32_t n_coef = 0;
    const int rc = pitt_srv_ransac_sphere(pitt_ros::node().srv, cloud.data(), n, pitt_ros::n_points(req.normals),
                                          inl.data(), &n_inl, coef, &n_coef, centroid);
    if (rc < 0) {
        ROS_ERROR_STREAM("sphere segmentation (MI355X) failed: " << pitt_last_error(pitt_ros::node().ctx));
        return false;
    }
    res.inliers.assign(inl.begin(), inl.begin() + n_inl);
    res.coefficients.assign(coef, coef + n_coef);
    if (n_coef > 0) {
        res.x_centroid = centroid[0];
        res.y_centroid = centroid[1];
        res.z_centroid = centroid[2];
    }
    return rc == 1;
}

int main(int argc, char** argv) {
    ros::init(argc, argv, "sphere_segmentation_srv");
    ros::NodeHandle nh;
    g_nh = &nh;
    pitt_ros::init_node();
    ros::ServiceServer service = nh.advertiseService("sphere_segmentation_srv", ransacSphereDetection);
    ros::spin();
    pitt_ros::shutdown_node();
    return 0;
}
