// Stand-in for pitt_msgs/PrimitiveSegmentation (SURVEY.md s8(b) schema; compile checks only).
#pragma once
#include <cstdint>
#include <vector>
#include "sensor_msgs/PointCloud2.h"
namespace pitt_msgs {
struct PrimitiveSegmentation {
    struct Request {
        sensor_msgs::PointCloud2 cloud, normals;
    };
    struct Response {
        std::vector<int32_t> inliers;
        std::vector<float> coefficients;
        float x_centroid = 0, y_centroid = 0, z_centroid = 0;
    };
};
}  // namespace pitt_msgs
