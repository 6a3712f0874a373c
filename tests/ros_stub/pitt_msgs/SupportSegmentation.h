// Stand-in for pitt_msgs/SupportSegmentation + Support (SURVEY.md s8(b) schema; compile checks only).
#pragma once
#include <cstdint>
#include <vector>
#include "sensor_msgs/PointCloud2.h"
namespace pitt_msgs {
struct Support {
    std::vector<int32_t> inliers;
    sensor_msgs::PointCloud2 support_cloud, on_support_cloud;
    float support_coefficient_a = 0, support_coefficient_b = 0, support_coefficient_c = 0, support_coefficient_d = 0;
};
struct SupportSegmentation {
    struct Request {
        sensor_msgs::PointCloud2 input_cloud, input_norm;
        float min_iterative_cloud_percentual_size = 0, min_iterative_plane_percentual_size = 0;
        float variance_threshold_for_horizontal = 0, ransac_distance_point_in_shape_threshold = 0;
        float ransac_model_normal_distance_weigth = 0;
        int32_t ransac_max_iteration_threshold = 0;
        std::vector<float> horizontal_axis, support_edge_remove_offset;
    };
    struct Response {
        std::vector<Support> supports_description;
        float used_min_iterative_cloud_percentual_size = 0, used_min_iterative_plane_percentual_size = 0;
        float used_max_variance_threshold_for_horizontal = 0, used_min_variance_threshold_for_horizontal = 0;
        int32_t used_ransac_max_iteration_threshold = 0;
        float used_ransac_distance_point_in_shape_threshold = 0, used_ransac_model_normal_distance_weigth = 0;
        std::vector<float> used_horizontal_axis, used_support_edge_remove_offset;
    };
};
}  // namespace pitt_msgs
