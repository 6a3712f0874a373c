// cylinder_segmentation_node.cpp -- drop-in for src/segmentation_services/cylinder_segmentation_srv.cpp.
// Same service name (srvm::SRV_NAME_RANSAC_CYLINDER_FILTER = "cylinder_segmentation_srv"), same request /
// response, same /pitt/srv/cylinder_segmentation/* parameters (read per call, :93-108); the handler body
// (SACSegmentationFromNormals with SACMODEL_CYLINDER at :111-126, the axis projection and O(n^2) height
// search at :129-178, the centroid at :174-176, the conversions at :194-200) runs through
// pitt_srv_ransac_cylinder on the MI355X.
#include <pitt_msgs/PrimitiveSegmentation.h>

#include "pitt_ros_common.hpp"

namespace {
ros::NodeHandle* g_nh = nullptr;
const std::vector<std::string> kParams = {
    "/pitt/srv/cylinder_segmentation/normal_distance_weight", "/pitt/srv/cylinder_segmentation/distance_th",
    "/pitt/srv/cylinder_segmentation/max_iter_limit",         "/pitt/srv/cylinder_segmentation/min_radius_limit",
    "/pitt/srv/cylinder_segmentation/max_radius_limit",       "/pitt/srv/cylinder_segmentation/eps_angle_th",
    "/pitt/srv/cylinder_segmentation/min_opening_angle_deg",  "/pitt/srv/cylinder_segmentation/max_opening_angle_deg"};
}  // namespace

bool ransacCylinderDetaction(pitt_msgs::PrimitiveSegmentation::Request& req, pitt_msgs::PrimitiveSegmentation::Response& res) {
    pitt_ros::sync_params(*g_nh, kParams);
    const std::vector<float> cloud = pitt_ros::to_xyz16(req.cloud);
    const std::vector<float> normals = pitt_ros::to_normals3(req.normals);
    const int64_t n = (int64_t)cloud.size() / 4;
    std::vector<int32_t> inl((size_t)std::max<int64_t>(n, 1));
    int64_t n_inl = 0;
    float coef[8] = {0, 0, 0, 0, 0, 0, 0, 0}, centroid[3] = {0, 0, 0};
    int32_t n_coef = 0;
    const int rc = pitt_srv_ransac_cylinder(pitt_ros::node().srv, cloud.data(), n, normals.data(),
                                         (int64_t)normals.size() / 3, inl.data(), &n_inl, coef, &n_coef, centroid);
    if (rc < 0) {
        ROS_ERROR_STREAM("cylinder segmentation (MI355X) failed: " << pitt_last_error(pitt_ros::node().ctx));
        return false;
    }
    res.inliers.assign(inl.begin(), inl.begin() + n_inl);
    res.coefficients.assign(coef, coef + n_coef);  // the model values, then the height (:194-196)
    res.x_centroid = centroid[0];
    res.y_centroid = centroid[1];
    res.z_centroid = centroid[2];
    return rc == 1;
}

int main(int argc, char** argv) {
    ros::init(argc, argv, "cylinder_segmentation_srv");
    ros::NodeHandle nh;
    g_nh = &nh;
    pitt_ros::init_node();
    ros::ServiceServer service = nh.advertiseService("cylinder_segmentation_srv", ransacCylinderDetaction);
    ros::spin();
    pitt_ros::shutdown_node();
    return 0;
}
