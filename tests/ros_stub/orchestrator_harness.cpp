// In-process harness for the two orchestrator nodes (tests/test_ros_orchestrators_gpu.py).  A node's
// source is compiled with -Dmain=pitt_node_main against these stubs and linked with this file and
// libpitt_seg.so; the harness feeds one message through ros::stub, runs the node's main (its loop
// ends after two spins), and writes what the node published to a binary file.
//
//   harness obj    <cloud.bin> <out.bin> [--pose 12 comma-separated values] [--arm none|missing|identity|crop:<x>]
//                  [--param name=int:<v>|dbl:<v>|list:<a,b,c>]...
//   harness ransac <clusters.bin> <out.bin> [--param ...]...
//
// cloud.bin: int64 width, height, point_step, row_step, off_x, off_y, off_z, then the payload bytes.
// --arm: none = ~arm_filter false; missing = no arm_filter_srv (the call fails); identity / crop:<x> =
// a stand-in service returning the cloud, or its points with x <= <x>, in order.
// clusters.bin: int64 count, then per cluster int32 shape_id, float centroid[3], int64 n, float xyz[3 n].
#include <pitt_msgs/ArmFilter.h>
#include <pitt_msgs/ClustersOutput.h>
#include <pitt_msgs/TrackedShapes.h>
#include <tf/transform_listener.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "pitt_ros_common.hpp"

int pitt_node_main(int argc, char** argv);

namespace {
std::vector<double> csv(const std::string& s) {
    std::vector<double> v;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ',')) v.push_back(std::strtod(tok.c_str(), nullptr));
    return v;
}

void set_param(const std::string& spec) {
    const size_t eq = spec.find('='), colon = spec.find(':', eq);
    const std::string name = spec.substr(0, eq), kind = spec.substr(eq + 1, colon - eq - 1), val = spec.substr(colon + 1);
    XmlRpc::XmlRpcValue v;
    if (kind == "int") v = XmlRpc::XmlRpcValue((int)std::strtol(val.c_str(), nullptr, 0));
    else if (kind == "dbl") v = XmlRpc::XmlRpcValue(std::strtod(val.c_str(), nullptr));
    else {
        v.type_ = XmlRpc::XmlRpcValue::TypeArray;
        for (double d : csv(val)) v.a_.push_back(XmlRpc::XmlRpcValue(d));
    }
    ros::NodeHandle::params()[name] = v;
}

template <class T>
void put(std::ofstream& o, const T& v) {
    o.write(reinterpret_cast<const char*>(&v), sizeof(T));
}
template <class T>
T get(std::ifstream& i) {
    T v{};
    i.read(reinterpret_cast<char*>(&v), sizeof(T));
    return v;
}

std::vector<float> xyz_of(const sensor_msgs::PointCloud2& m) {
    const std::vector<float> p = pitt_ros::to_xyz16(m);
    std::vector<float> out;
    for (size_t i = 0; i + 3 < p.size(); i += 4) out.insert(out.end(), {p[i], p[i + 1], p[i + 2]});
    return out;
}

int run_obj(const std::string& in, const std::string& out, const std::string& arm) {
    std::ifstream f(in, std::ios::binary);
    sensor_msgs::PointCloud2 msg;
    msg.width = (uint32_t)get<int64_t>(f);
    msg.height = (uint32_t)get<int64_t>(f);
    msg.point_step = (uint32_t)get<int64_t>(f);
    msg.row_step = (uint32_t)get<int64_t>(f);
    const char* names[3] = {"x", "y", "z"};
    for (int k = 0; k < 3; ++k) {
        sensor_msgs::PointField fl;
        fl.name = names[k];
        fl.offset = (uint32_t)get<int64_t>(f);
        fl.datatype = sensor_msgs::PointField::FLOAT32;
        fl.count = 1;
        msg.fields.push_back(fl);
    }
    msg.data.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    msg.is_dense = false;
    const std::string topic = "/camera/depth/points";
    if (arm == "none") {
        set_param("arm_filter=int:0");
    } else if (arm != "missing") {  // the reference's arm filter service, stood in by the identity or a crop on x
        const bool crop = arm.rfind("crop:", 0) == 0;
        const float cx = crop ? std::strtof(arm.c_str() + 5, nullptr) : 0.0f;  // compared in float, as the test's oracle side
        ros::stub::services()["arm_filter_srv"] = [crop, cx](void* p) {
            pitt_msgs::ArmFilter& s = *static_cast<pitt_msgs::ArmFilter*>(p);
            const std::vector<float> pts = pitt_ros::to_xyz16(s.request.input_cloud);
            std::vector<float> keep;
            for (size_t i = 0; i + 3 < pts.size(); i += 4)
                if (!crop || pts[i] <= cx) keep.insert(keep.end(), {pts[i], pts[i + 1], pts[i + 2], 1.0f});
            s.response.armless_cloud = pitt_ros::from_xyz16(keep.data(), (int64_t)keep.size() / 4);
            return true;
        };
    }
    bool sent = false;
    ros::stub::on_spin() = [&]() {
        if (!sent) ros::stub::deliver(topic, msg);
        sent = true;
    };
    ros::stub::spins() = 2;
    char a0[] = "obj_segmentation", a1[] = "/camera/depth/points", dot[] = ".";
    char* argv[] = {a0, a1, dot, dot, dot, dot, dot, nullptr};
    const int rc = pitt_node_main(7, argv);
    std::ofstream o(out, std::ios::binary);
    const auto pubs = ros::stub::published<pitt_msgs::ClustersOutput>("obj_segmentation/ClusterOutput");
    put<int64_t>(o, (int64_t)pubs.size());
    for (const auto& m : pubs) {
        put<int64_t>(o, (int64_t)m.cluster_objs.size());
        for (const auto& c : m.cluster_objs) {
            put<int64_t>(o, (int64_t)c.inliers.size());
            o.write(reinterpret_cast<const char*>(c.inliers.data()), (std::streamsize)(c.inliers.size() * 4));
            put<float>(o, c.x_centroid);
            put<float>(o, c.y_centroid);
            put<float>(o, c.z_centroid);
            const std::vector<float> p = xyz_of(c.cloud);
            put<int64_t>(o, (int64_t)p.size() / 3);
            o.write(reinterpret_cast<const char*>(p.data()), (std::streamsize)(p.size() * 4));
        }
    }
    return rc;
}

int run_ransac(const std::string& in, const std::string& out) {
    std::ifstream f(in, std::ios::binary);
    pitt_msgs::ClustersOutput msg;
    const int64_t nc = get<int64_t>(f);
    for (int64_t j = 0; j < nc; ++j) {
        pitt_msgs::InliersCluster c;
        c.shape_id = get<int32_t>(f);
        c.x_centroid = get<float>(f);
        c.y_centroid = get<float>(f);
        c.z_centroid = get<float>(f);
        const int64_t n = get<int64_t>(f);
        std::vector<float> xyz16((size_t)std::max<int64_t>(n, 1) * 4, 1.0f);
        for (int64_t i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k) xyz16[(size_t)(4 * i + k)] = get<float>(f);
        c.cloud = pitt_ros::from_xyz16(xyz16.data(), n);
        msg.cluster_objs.push_back(c);
    }
    bool sent = false;
    ros::stub::on_spin() = [&]() {
        if (!sent) ros::stub::deliver("geometric_tracker/trackedCluster", msg);
        sent = true;
    };
    ros::stub::spins() = 2;
    char a0[] = "ransac_segmentation", a1[] = "0";
    char* argv[] = {a0, a1, nullptr};
    const int rc = pitt_node_main(2, argv);
    std::ofstream o(out, std::ios::binary);
    const auto pubs = ros::stub::published<pitt_msgs::TrackedShapes>("ransac_segmentation/trackedShapes");
    put<int64_t>(o, (int64_t)pubs.size());
    for (const auto& m : pubs) {
        put<int64_t>(o, (int64_t)m.tracked_shapes.size());
        for (const auto& s : m.tracked_shapes) {
            put<int32_t>(o, s.object_id);
            put<float>(o, s.x_pc_centroid);
            put<float>(o, s.y_pc_centroid);
            put<float>(o, s.z_pc_centroid);
            put<int64_t>(o, (int64_t)s.shape_tag.size());
            o.write(s.shape_tag.data(), (std::streamsize)s.shape_tag.size());
            put<float>(o, s.x_est_centroid);
            put<float>(o, s.y_est_centroid);
            put<float>(o, s.z_est_centroid);
            put<int64_t>(o, (int64_t)s.coefficients.size());
            o.write(reinterpret_cast<const char*>(s.coefficients.data()), (std::streamsize)(s.coefficients.size() * 4));
        }
    }
    return rc;
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: harness obj|ransac <in> <out> [options]\n");
        return 2;
    }
    std::string arm = "identity";
    for (int a = 4; a + 1 < argc; a += 2) {
        const std::string k = argv[a], v = argv[a + 1];
        if (k == "--param") set_param(v);
        else if (k == "--arm") arm = v;
        else if (k == "--pose") {
            const std::vector<double> p = csv(v);
            for (size_t i = 0; i < 12 && i < p.size(); ++i) tf::stub::pose()[i] = p[i];
        }
    }
    const std::string mode = argv[1];
    if (mode == "obj") return run_obj(argv[2], argv[3], arm);
    if (mode == "ransac") return run_ransac(argv[2], argv[3]);
    return 2;
}
