// Runs adapters/ros/pitt_ros_common.hpp's PointCloud2 conversions on well-formed and malformed
// messages (tests/test_ros_adapters.py).  Prints one line per case: name, converted floats.
#include <cstdio>
#include <cstring>

#include "pitt_ros_common.hpp"

static sensor_msgs::PointCloud2 cloud(uint32_t w, uint32_t h, uint32_t step, uint32_t row, size_t bytes,
                                      const char* a, const char* b, const char* c, uint32_t off0 = 0) {
    sensor_msgs::PointCloud2 m;
    m.width = w;
    m.height = h;
    m.point_step = step;
    m.row_step = row;
    const char* names[3] = {a, b, c};
    for (int k = 0; k < 3; ++k) {
        sensor_msgs::PointField f;
        f.name = names[k];
        f.offset = off0 + 4 * k;
        f.datatype = sensor_msgs::PointField::FLOAT32;
        f.count = 1;
        m.fields.push_back(f);
    }
    m.data.resize(bytes);
    for (size_t i = 0; i + 4 <= bytes; i += 4) {
        const float v = (float)(i / 4);
        std::memcpy(&m.data[i], &v, 4);
    }
    return m;
}

static void show(const char* name, const std::vector<float>& v) {
    std::printf("%s %zu", name, v.size());
    for (size_t i = 0; i < v.size() && i < 8; ++i) std::printf(" %g", v[i]);
    std::printf("\n");
}

int main() {
    // 2 x 3 organised, point_step 16, row_step 48: exactly sized
    show("ok", pitt_ros::to_xyz16(cloud(3, 2, 16, 48, 96, "x", "y", "z")));
    // padded rows (row_step 64): last row ends at 64 + 48
    show("ok_padded_rows", pitt_ros::to_xyz16(cloud(3, 2, 16, 64, 112, "x", "y", "z")));
    show("short_payload", pitt_ros::to_xyz16(cloud(3, 2, 16, 48, 95, "x", "y", "z")));
    show("row_step_small", pitt_ros::to_xyz16(cloud(3, 2, 16, 32, 96, "x", "y", "z")));
    show("field_beyond_step", pitt_ros::to_xyz16(cloud(3, 2, 12, 36, 72, "x", "y", "z", 4)));
    sensor_msgs::PointCloud2 be = cloud(3, 2, 16, 48, 96, "x", "y", "z");
    be.is_bigendian = true;
    show("big_endian", pitt_ros::to_xyz16(be));
    show("no_fields", pitt_ros::to_xyz16(cloud(3, 2, 16, 48, 96, "a", "b", "c")));
    show("normals_ok", pitt_ros::to_normals3(cloud(2, 1, 16, 32, 32, "normal_x", "normal_y", "normal_z")));
    show("normals_short", pitt_ros::to_normals3(cloud(2, 1, 16, 32, 20, "normal_x", "normal_y", "normal_z")));
    show("normals_missing", pitt_ros::to_normals3(cloud(2, 1, 16, 32, 32, "a", "b", "c")));
    return 0;
}
