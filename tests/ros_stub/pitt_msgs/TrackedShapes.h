// Stand-in for pitt_msgs/TrackedShape(s) (fields as ransac_segmentation.cpp:315-328 writes them).
#pragma once
#include <cstdint>
#include <string>
#include <vector>
namespace pitt_msgs {
struct TrackedShape {
    int32_t object_id = 0;
    float x_pc_centroid = 0, y_pc_centroid = 0, z_pc_centroid = 0;
    std::string shape_tag;
    float x_est_centroid = 0, y_est_centroid = 0, z_est_centroid = 0;
    std::vector<float> coefficients;
};
struct TrackedShapes {
    std::vector<TrackedShape> tracked_shapes;
};
}  // namespace pitt_msgs
