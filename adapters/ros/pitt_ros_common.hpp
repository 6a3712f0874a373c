// pitt_ros_common.hpp -- shared pieces of the ROS handler shims.
//
// Compiled only where ROS 1 (roscpp, sensor_msgs) and the pitt_msgs package exist (a catkin
// workspace next to the reference package; adapters/ros/CMakeLists.txt).  It is not built in this
// repository's CI: the shims call nothing but the C ABI in include/pitt_srv.h and include/pitt_seg.h,
// and tests/test_host_and_abi.py checks that every pitt_* symbol they use is declared there.
//
// What lives here:
//   * one pitt context + one pitt_srv service object per node process (the reference's handlers run
//     serially under ros::spin, so one context is enough);
//   * sensor_msgs::PointCloud2 <-> the 16-byte PointXYZ arrays the service ABI takes (fromROSMsg /
//     toROSMsg of PCManager::cloudForRosMsg / cloudToRosMsg, pc_manager.cpp:80-104);
//   * forwarding of the node's /pitt/srv/... ROS parameters to the service object with their XmlRpc
//     type, so the mirror applies roscpp's typed-read rules exactly as NodeHandle::param would.
#pragma once
#include <hip/hip_runtime_api.h>
#include <ros/ros.h>
#include <sensor_msgs/PointCloud2.h>
#include <sensor_msgs/PointField.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "pitt_srv.h"

namespace pitt_ros {

struct Node {
    pitt_ctx* ctx = nullptr;
    pitt_srv* srv = nullptr;
};

inline Node& node() {
    static Node n;
    return n;
}

// A grow-only device buffer (the nodes' per-message staging: payload, SoA planes).
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void* get(size_t b) {
        if (b > bytes) {
            if (p) (void)hipFree(p);
            p = nullptr;
            bytes = 0;
            if (hipMalloc(&p, b) != hipSuccess) return nullptr;
            bytes = b;
        }
        return p;
    }
};

// pitt_create on device 0 (or $PITT_DEVICE) and the service object; throws when no gfx950 device.
inline void init_node() {
    Node& n = node();
    if (n.ctx) return;
    const char* dev = std::getenv("PITT_DEVICE");
    if (pitt_create(&n.ctx, dev ? std::atoi(dev) : 0) != PITT_OK) throw std::runtime_error("pitt_create failed");
    n.srv = pitt_srv_create(n.ctx);
    if (!n.srv) throw std::runtime_error("pitt_srv_create failed");
}

inline void shutdown_node() {
    Node& n = node();
    if (n.srv) pitt_srv_destroy(n.srv);
    if (n.ctx) pitt_destroy(n.ctx);
    n.srv = nullptr;
    n.ctx = nullptr;
}

// Forward the ROS parameters the handlers read (srv_manager.h:35-95) with their stored type.
inline void sync_params(ros::NodeHandle& nh, const std::vector<std::string>& names) {
    pitt_srv* srv = node().srv;
    for (const std::string& name : names) {
        XmlRpc::XmlRpcValue v;
        if (!nh.getParam(name, v)) {
            pitt_srv_param_erase(srv, name.c_str());
            continue;
        }
        switch (v.getType()) {
            case XmlRpc::XmlRpcValue::TypeInt:
                pitt_srv_param_set_int(srv, name.c_str(), static_cast<int>(v));
                break;
            case XmlRpc::XmlRpcValue::TypeDouble:
                pitt_srv_param_set_double(srv, name.c_str(), static_cast<double>(v));
                break;
            case XmlRpc::XmlRpcValue::TypeArray: {
                std::vector<double> list;
                for (int i = 0; i < v.size(); ++i) {
                    if (v[i].getType() == XmlRpc::XmlRpcValue::TypeInt) list.push_back(static_cast<int>(v[i]));
                    else if (v[i].getType() == XmlRpc::XmlRpcValue::TypeDouble) list.push_back(static_cast<double>(v[i]));
                }
                pitt_srv_param_set_list(srv, name.c_str(), list.data(), static_cast<int32_t>(list.size()));
                break;
            }
            default:  // a string or bool where a number is expected: NodeHandle::param keeps the default
                pitt_srv_param_erase(srv, name.c_str());
        }
    }
}

// The payload layout check pitt_unpack_pointcloud2 applies on the device (preprocess.hip), done on
// the host before any byte is read: little-endian only, every located field (offset + 4) inside
// point_step, row_step >= width * point_step, and the last point's last byte inside data.
// Returns false, with the reason, for a message whose layout would read past its payload.
inline bool layout_ok(const sensor_msgs::PointCloud2& msg, const int* off, int nf, std::string* why) {
    const size_t n = (size_t)msg.width * msg.height;
    if (msg.is_bigendian) {
        *why = "big-endian payload";
        return false;
    }
    for (int k = 0; k < nf; ++k)
        if (off[k] >= 0 && (size_t)off[k] + 4 > msg.point_step) {
            *why = "field offset + 4 beyond point_step";
            return false;
        }
    if (n == 0) return true;
    if ((size_t)msg.row_step < (size_t)msg.width * msg.point_step) {
        *why = "row_step < width * point_step";
        return false;
    }
    if ((size_t)(msg.height - 1) * msg.row_step + (size_t)msg.width * msg.point_step > msg.data.size()) {
        *why = "payload shorter than its layout";
        return false;
    }
    return true;
}

// fromROSMsg into PointXYZ (x, y, z, pad): fields located by name, FLOAT32 only, any point_step /
// row_step; a cloud without x/y/z fields converts to zero points (fromROSMsg warns likewise).  A
// malformed layout (layout_ok) converts to zero points as well, with an error on the log.
inline std::vector<float> to_xyz16(const sensor_msgs::PointCloud2& msg) {
    int off[3] = {-1, -1, -1};
    const char* names[3] = {"x", "y", "z"};
    for (const sensor_msgs::PointField& f : msg.fields)
        for (int k = 0; k < 3; ++k)
            if (f.name == names[k] && f.datatype == sensor_msgs::PointField::FLOAT32) off[k] = (int)f.offset;
    const size_t n = (size_t)msg.width * msg.height;
    std::vector<float> out;
    if (off[0] < 0 || off[1] < 0 || off[2] < 0) return out;
    std::string why;
    if (!layout_ok(msg, off, 3, &why)) {
        ROS_ERROR_STREAM("PointCloud2 rejected: " << why);
        return out;
    }
    out.resize(4 * n);
    for (uint32_t r = 0; r < msg.height; ++r)
        for (uint32_t c = 0; c < msg.width; ++c) {
            const uint8_t* p = &msg.data[(size_t)r * msg.row_step + (size_t)c * msg.point_step];
            float* o = &out[4 * ((size_t)r * msg.width + c)];
            for (int k = 0; k < 3; ++k) std::memcpy(&o[k], p + off[k], 4);
            o[3] = 1.0f;
        }
    return out;
}

// toROSMsg of a PointCloud<PointXYZ> (height 1, fields x/y/z FLOAT32 at 0/4/8, point_step 16).
inline sensor_msgs::PointCloud2 from_xyz16(const float* xyz16, int64_t n, bool is_dense = true) {
    sensor_msgs::PointCloud2 m;
    m.height = 1;
    m.width = (uint32_t)n;
    const char* names[3] = {"x", "y", "z"};
    for (int k = 0; k < 3; ++k) {
        sensor_msgs::PointField f;
        f.name = names[k];
        f.offset = 4 * k;
        f.datatype = sensor_msgs::PointField::FLOAT32;
        f.count = 1;
        m.fields.push_back(f);
    }
    m.is_bigendian = false;
    m.point_step = 16;
    m.row_step = 16 * (uint32_t)n;
    m.is_dense = is_dense;
    m.data.resize((size_t)16 * n);
    if (n > 0) std::memcpy(m.data.data(), xyz16, (size_t)16 * n);
    return m;
}

// fromROSMsg into PointCloud<Normal> (PCManager::normForRosMsg, pc_manager.cpp:92-97), keeping the
// (normal_x, normal_y, normal_z) triples: fields located by name, FLOAT32 only; a missing field leaves
// pcl::Normal's default 0.  A malformed layout gives no normals (the services then fail their
// normals-size check and answer empty, as PCL does for a size mismatch).
inline std::vector<float> to_normals3(const sensor_msgs::PointCloud2& msg) {
    int off[3] = {-1, -1, -1};
    const char* names[3] = {"normal_x", "normal_y", "normal_z"};
    for (const sensor_msgs::PointField& f : msg.fields)
        for (int k = 0; k < 3; ++k)
            if (f.name == names[k] && f.datatype == sensor_msgs::PointField::FLOAT32) off[k] = (int)f.offset;
    const size_t n = (size_t)msg.width * msg.height;
    std::string why;
    if (!layout_ok(msg, off, 3, &why)) {
        ROS_ERROR_STREAM("normals PointCloud2 rejected: " << why);
        return std::vector<float>();
    }
    std::vector<float> out(3 * n, 0.0f);
    for (uint32_t r = 0; r < msg.height; ++r)
        for (uint32_t c = 0; c < msg.width; ++c) {
            const uint8_t* p = &msg.data[(size_t)r * msg.row_step + (size_t)c * msg.point_step];
            float* o = &out[3 * ((size_t)r * msg.width + c)];
            for (int k = 0; k < 3; ++k)
                if (off[k] >= 0) std::memcpy(&o[k], p + off[k], 4);
        }
    return out;
}

inline int64_t n_points(const sensor_msgs::PointCloud2& msg) { return (int64_t)msg.width * msg.height; }

}  // namespace pitt_ros
