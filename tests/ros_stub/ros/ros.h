// Stand-in for <ros/ros.h>: the declarations adapters/ros uses (compile checks only).
#pragma once
#include <iostream>
#include <map>
#include <string>
#include <vector>

namespace XmlRpc {
class XmlRpcValue {
  public:
    enum Type { TypeInvalid, TypeBoolean, TypeInt, TypeDouble, TypeString, TypeArray };
    Type getType() const { return type_; }
    explicit operator int() const { return i_; }
    explicit operator double() const { return d_; }
    int size() const { return (int)a_.size(); }
    XmlRpcValue& operator[](int k) { return a_[(size_t)k]; }
    Type type_ = TypeInvalid;
    int i_ = 0;
    double d_ = 0.0;
    std::vector<XmlRpcValue> a_;
};
}  // namespace XmlRpc

namespace ros {
inline void init(int&, char**, const std::string&) {}
inline void spin() {}
class ServiceServer {
  public:
    ~ServiceServer() {}  // the real one unadvertises on destruction
};
class NodeHandle {
  public:
    NodeHandle() {}
    explicit NodeHandle(const std::string&) {}
    bool getParam(const std::string& k, XmlRpc::XmlRpcValue& v) const {
        auto it = params().find(k);
        if (it == params().end()) return false;
        v = it->second;
        return true;
    }
    template <class T, class D>
    bool param(const std::string&, T& v, const D& d) const {
        v = d;
        return false;
    }
    template <class Req, class Res>
    ServiceServer advertiseService(const std::string&, bool (*)(Req&, Res&)) {
        return ServiceServer();
    }
    static std::map<std::string, XmlRpc::XmlRpcValue>& params() {
        static std::map<std::string, XmlRpc::XmlRpcValue> p;
        return p;
    }
};
}  // namespace ros

#define ROS_ERROR_STREAM(x) (std::cerr << "[ERROR] " << x << std::endl)
#define ROS_WARN_STREAM(x) (std::cerr << "[WARN] " << x << std::endl)
#define ROS_INFO_STREAM(x) (std::cerr << "[INFO] " << x << std::endl)
