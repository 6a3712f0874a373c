// supports_segmentation_node.cpp -- drop-in for src/segmentation_services/supports_segmentation_srv.cpp.
// Service "support_segmentation_srv"; the request's -1 / wrong-length fields select the defaults
// (initializeInputParameters, :70-86); the whole while(loop) of findSupports (:241-361: RANSAC on the
// shrinking cloud, removePlaneInliner, isHorizontalPlane, createNewIdxMap incl. Q4, getPointOnPlane
// incl. Q5 / Q10) runs through pitt_srv_find_supports on the MI355X.
#include <pitt_msgs/SupportSegmentation.h>

#include "pitt_ros_common.hpp"

namespace {
void fill_vec(const std::vector<float>& v, int32_t* n, float* out) {
    *n = (int32_t)v.size();
    for (size_t i = 0; i < v.size() && i < 8; ++i) out[i] = v[i];
}
}  // namespace

bool findSupports(pitt_msgs::SupportSegmentation::Request& req, pitt_msgs::SupportSegmentation::Response& res) {
    pitt_srv* srv = pitt_ros::node().srv;
    const std::vector<float> cloud = pitt_ros::to_xyz16(req.input_cloud);
    const int64_t n = (int64_t)cloud.size() / 4;
    pitt_srv_support_request r;
    r.min_iterative_cloud_percentual_size = req.min_iterative_cloud_percentual_size;
    r.min_iterative_plane_percentual_size = req.min_iterative_plane_percentual_size;
    r.variance_threshold_for_horizontal = req.variance_threshold_for_horizontal;
    r.ransac_distance_point_in_shape_threshold = req.ransac_distance_point_in_shape_threshold;
    r.ransac_model_normal_distance_weigth = req.ransac_model_normal_distance_weigth;
    r.ransac_max_iteration_threshold = req.ransac_max_iteration_threshold;
    fill_vec(req.horizontal_axis, &r.n_horizontal_axis, r.horizontal_axis);
    fill_vec(req.support_edge_remove_offset, &r.n_edge_remove_offset, r.edge_remove_offset);
    int32_t n_sup = 0;
    float used[13];
    const int rc = pitt_srv_find_supports(srv, cloud.data(), n, pitt_ros::n_points(req.input_norm), &r, &n_sup, used);
    if (rc < 0) {
        ROS_ERROR_STREAM("support segmentation (MI355X) failed: " << pitt_last_error(pitt_ros::node().ctx));
        return false;
    }
    for (int32_t s = 0; s < n_sup; ++s) {
        pitt_msgs::Support sup;
        sup.inliers.resize((size_t)n);
        float coef[4];
        int64_t ns = 0, no = 0;
        pitt_srv_support_get(srv, s, sup.inliers.data(), coef, &ns, &no);
        std::vector<float> a((size_t)std::max<int64_t>(ns, 1) * 4), b((size_t)std::max<int64_t>(no, 1) * 4);
        pitt_srv_support_cloud(srv, s, 0, a.data());
        pitt_srv_support_cloud(srv, s, 1, b.data());
        sup.support_cloud = pitt_ros::from_xyz16(a.data(), ns);
        sup.on_support_cloud = pitt_ros::from_xyz16(b.data(), no);
        sup.support_coefficient_a = coef[0];
        sup.support_coefficient_b = coef[1];
        sup.support_coefficient_c = coef[2];
        sup.support_coefficient_d = coef[3];
        res.supports_description.push_back(sup);
    }
    res.used_min_iterative_cloud_percentual_size = used[0];
    res.used_min_iterative_plane_percentual_size = used[1];
    res.used_max_variance_threshold_for_horizontal = used[2];
    res.used_min_variance_threshold_for_horizontal = used[3];
    res.used_ransac_max_iteration_threshold = (int32_t)used[4];
    res.used_ransac_distance_point_in_shape_threshold = used[5];
    res.used_ransac_model_normal_distance_weigth = used[6];
    res.used_horizontal_axis.assign(used + 7, used + 10);
    res.used_support_edge_remove_offset.assign(used + 10, used + 13);
    return rc == 1;
}

int main(int argc, char** argv) {
    ros::init(argc, argv, "support_segmentation_srv");
    ros::NodeHandle nh;
    pitt_ros::init_node();
    ros::ServiceServer service = nh.advertiseService("support_segmentation_srv", findSupports);
    ros::spin();
    pitt_ros::shutdown_node();
    return 0;
}
