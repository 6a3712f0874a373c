// cluster_segmentation_node.cpp -- drop-in for src/segmentation_services/cluster_segmentation_srv.cpp.
// Service "cluster_Segmentation_srv" (srv_manager.h:27's spelling); the /pitt/srv/cluster_segmentation/*
// parameters are read per call (:44-50, including Q6: min_input_size read from the tolerance name);
// EuclideanClusterExtraction (:57-69) and the per-cluster inliers / cloud / centroid (:72-101, Q7's
// counter starting at 1) run through pitt_srv_clusterize on the MI355X.
#include <pitt_msgs/ClusterSegmentation.h>

#include "pitt_ros_common.hpp"

namespace {
ros::NodeHandle* g_nh = nullptr;
const std::vector<std::string> kParams = {
    "/pitt/srv/cluster_segmentation/tolerance", "/pitt/srv/cluster_segmentation/min_rate",
    "/pitt/srv/cluster_segmentation/max_rate", "/pitt/srv/cluster_segmentation/min_input_size"};
}  // namespace

bool clusterize(pitt_msgs::ClusterSegmentation::Request& req, pitt_msgs::ClusterSegmentation::Response& res) {
    pitt_ros::sync_params(*g_nh, kParams);
    pitt_srv* srv = pitt_ros::node().srv;
    const std::vector<float> cloud = pitt_ros::to_xyz16(req.cloud);
    const int64_t n = (int64_t)cloud.size() / 4;
    int32_t n_cl = 0;
    const int rc = pitt_srv_clusterize(srv, cloud.data(), n, &n_cl);
    if (rc < 0) {
        ROS_ERROR_STREAM("cluster segmentation (MI355X) failed: " << pitt_last_error(pitt_ros::node().ctx));
        return false;
    }
    for (int32_t c = 0; c < n_cl; ++c) {
        int64_t size = 0;
        float centroid[3];
        pitt_srv_cluster_get(srv, c, nullptr, &size, centroid, nullptr);  // size first
        pitt_msgs::InliersCluster cl;
        cl.inliers.resize((size_t)size);
        std::vector<float> xyz((size_t)std::max<int64_t>(size, 1) * 4);
        pitt_srv_cluster_get(srv, c, cl.inliers.data(), &size, centroid, xyz.data());
        cl.cloud = pitt_ros::from_xyz16(xyz.data(), size);
        cl.x_centroid = centroid[0];
        cl.y_centroid = centroid[1];
        cl.z_centroid = centroid[2];
        res.cluster_objs.push_back(cl);
    }
    return rc == 1;
}

int main(int argc, char** argv) {
    ros::init(argc, argv, "cluster_Segmentation_srv");
    ros::NodeHandle nh;
    g_nh = &nh;
    pitt_ros::init_node();
    ros::ServiceServer service = nh.advertiseService("cluster_Segmentation_srv", clusterize);
    ros::spin();
    pitt_ros::shutdown_node();
    return 0;
}
