// Stand-in for pitt_msgs/ArmFilter (fields as obj_segmentation.cpp:122-129 uses them).
#pragma once
#include <vector>
#include "sensor_msgs/PointCloud2.h"
namespace pitt_msgs {
struct ArmFilter {
    struct Request {
        sensor_msgs::PointCloud2 input_cloud;
        std::vector<float> forearm_bounding_box_min_value, forearm_bounding_box_max_value;
        std::vector<float> elbow_bounding_box_min_value, elbow_bounding_box_max_value;
    } request;
    struct Response {
        sensor_msgs::PointCloud2 armless_cloud;
    } response;
};
}  // namespace pitt_msgs
