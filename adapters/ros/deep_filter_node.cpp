// deep_filter_node.cpp -- drop-in for src/segmentation_services/deep_filter_srv.cpp.
// Service "deep_filter_srv"; req.deep_threshold keeps its sentinel (getServiceFloatParameter, a value
// >= 0 is used, else 3.0 m, :19/:31).  The PointCloud2 payload is uploaded once, unpacked on the device
// (fromROSMsg, pc_manager.cpp:94-104 -> pitt_unpack_pointcloud2), optionally downsampled by the 1 cm
// VoxelGrid that depthAcquisition applies before calling this service (obj_segmentation.cpp:238 ->
// pitt_voxel_grid, when the node runs with ~voxel_leaf > 0), then split (deepFiltering :37-44 ->
// pitt_deep_filter); both outputs come back in input order.
#include <hip/hip_runtime.h>
#include <pitt_msgs/DeepFilter.h>

#include "pitt_ros_common.hpp"

namespace {
double g_leaf = 0.0;

pitt_ros::DevBuf g_payload, g_planes, g_out;

bool copy_ok(hipError_t e) {
    if (e != hipSuccess) ROS_ERROR_STREAM("deep filter: HIP copy failed: " << hipGetErrorString(e));
    return e == hipSuccess;
}

bool download_xyz16(const float* x, const float* y, const float* z, int64_t n, std::vector<float>& out) {
    std::vector<float> sx((size_t)n), sy((size_t)n), sz((size_t)n);
    out.assign((size_t)n * 4, 0.0f);
    if (n == 0) return true;
    if (!copy_ok(hipMemcpy(sx.data(), x, (size_t)n * 4, hipMemcpyDeviceToHost)) ||
        !copy_ok(hipMemcpy(sy.data(), y, (size_t)n * 4, hipMemcpyDeviceToHost)) ||
        !copy_ok(hipMemcpy(sz.data(), z, (size_t)n * 4, hipMemcpyDeviceToHost)))
        return false;
    for (int64_t i = 0; i < n; ++i) {
        out[4 * i] = sx[i];
        out[4 * i + 1] = sy[i];
        out[4 * i + 2] = sz[i];
        out[4 * i + 3] = 1.0f;
    }
    return true;
}
}  // namespace

bool deepFiltering(pitt_msgs::DeepFilter::Request& req, pitt_msgs::DeepFilter::Response& res) {
    pitt_ctx* ctx = pitt_ros::node().ctx;
    const sensor_msgs::PointCloud2& m = req.input_cloud;
    int off[3] = {-1, -1, -1};
    for (const sensor_msgs::PointField& f : m.fields) {
        if (f.datatype != sensor_msgs::PointField::FLOAT32) continue;
        if (f.name == "x") off[0] = (int)f.offset;
        if (f.name == "y") off[1] = (int)f.offset;
        if (f.name == "z") off[2] = (int)f.offset;
    }
    int64_t n = pitt_ros::n_points(m);
    if (off[0] < 0 || off[1] < 0 || off[2] < 0) n = 0;
    float* planes = (float*)g_planes.get((size_t)std::max<int64_t>(n, 1) * 12);
    float* outp = (float*)g_out.get((size_t)std::max<int64_t>(n, 1) * 24);
    void* payload = g_payload.get(std::max<size_t>(m.data.size(), 16));
    if (!planes || !outp || !payload) return false;
    float *x = planes, *y = planes + n, *z = planes + 2 * n;
    if (n > 0) {
        if (!copy_ok(hipMemcpy(payload, m.data.data(), m.data.size(), hipMemcpyHostToDevice))) return false;
        if (pitt_unpack_pointcloud2(ctx, payload, (int64_t)m.data.size(), (int32_t)m.width, (int32_t)m.height,
                                    (int32_t)m.point_step, (int64_t)m.row_step, off[0], off[1], off[2], x, y,
                                    z) != PITT_OK) {
            ROS_ERROR_STREAM("PointCloud2 unpack failed: " << pitt_last_error(ctx));
            return false;
        }
        if (g_leaf > 0.0) {  // PCManager::downSampling in front of the service (obj_segmentation.cpp:238)
            int64_t nv = 0;
            int32_t flags = 0;
            float* v = outp;
            if (pitt_voxel_grid(ctx, x, y, z, n, (float)g_leaf, (float)g_leaf, (float)g_leaf, PITT_VOXEL_ORDER_PCL, v,
                                v + n, v + 2 * n, &nv, &flags) != PITT_OK)
                return false;
            if (!copy_ok(hipMemcpy(x, v, (size_t)nv * 4, hipMemcpyDeviceToDevice)) ||
                !copy_ok(hipMemcpy(x + nv, v + n, (size_t)nv * 4, hipMemcpyDeviceToDevice)) ||
                !copy_ok(hipMemcpy(x + 2 * nv, v + 2 * n, (size_t)nv * 4, hipMemcpyDeviceToDevice)))
                return false;
            y = x + nv;
            z = x + 2 * nv;
            n = nv;
        }
    }
    float* c = outp;           // closer: capacity n per plane
    float* f = outp + 3 * n;   // further
    int64_t nc = 0, nf = 0;
    float used = 0.0f;
    if (pitt_deep_filter(ctx, x, y, z, n, req.deep_threshold, c, c + n, c + 2 * n, &nc, f, f + n, f + 2 * n, &nf,
                         &used) != PITT_OK) {
        ROS_ERROR_STREAM("deep filter (MI355X) failed: " << pitt_last_error(ctx));
        return false;
    }
    std::vector<float> closer, further;
    if (!download_xyz16(c, c + n, c + 2 * n, nc, closer) || !download_xyz16(f, f + n, f + 2 * n, nf, further))
        return false;
    res.cloud_closer = pitt_ros::from_xyz16(closer.data(), nc);
    res.cloud_further = pitt_ros::from_xyz16(further.data(), nf);
    res.used_deep_threshold = used;
    return true;
}

int main(int argc, char** argv) {
    ros::init(argc, argv, "deep_filter_srv");
    ros::NodeHandle nh, pnh("~");
    pnh.param("voxel_leaf", g_leaf, 0.0);
    pitt_ros::init_node();
    ros::ServiceServer service = nh.advertiseService("deep_filter_srv", deepFiltering);
    ros::spin();
    pitt_ros::shutdown_node();
    return 0;
}
