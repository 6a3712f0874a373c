// Stand-in for pitt_msgs/DeepFilter (deep_filter_srv.cpp:27-56 usage; compile checks only).
#pragma once
#include "sensor_msgs/PointCloud2.h"
namespace pitt_msgs {
struct DeepFilter {
    struct Request {
        sensor_msgs::PointCloud2 input_cloud;
        float deep_threshold = 0;
    };
    struct Response {
        sensor_msgs::PointCloud2 cloud_closer, cloud_further;
        float used_deep_threshold = 0;
    };
};
}  // namespace pitt_msgs
