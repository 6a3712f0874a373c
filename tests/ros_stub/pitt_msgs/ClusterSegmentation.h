// Stand-in for pitt_msgs/ClusterSegmentation + InliersCluster (compile checks only).
#pragma once
#include <cstdint>
#include <vector>
#include "sensor_msgs/PointCloud2.h"
namespace pitt_msgs {
struct InliersCluster {
    std::vector<int32_t> inliers;
    sensor_msgs::PointCloud2 cloud;
    float x_centroid = 0, y_centroid = 0, z_centroid = 0;
    int32_t shape_id = 0;
};
struct ClusterSegmentation {
    struct Request {
        sensor_msgs::PointCloud2 cloud;
    };
    struct Response {
        std::vector<InliersCluster> cluster_objs;
    };
};
}  // namespace pitt_msgs
