// Stand-in for <ros/ros.h>: the declarations adapters/ros uses (compile checks, plus the in-process
// harness of tests/test_ros_orchestrators_gpu.py: topics are delivered and publications captured through
// ros::stub, spinOnce runs ros::stub::on_spin, ok() turns false after ros::stub::spins() spins).
#pragma once
#include <cstdio>
#include <functional>
#include <iostream>
#include <map>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

namespace XmlRpc {
class XmlRpcValue {
  public:
    enum Type { TypeInvalid, TypeBoolean, TypeInt, TypeDouble, TypeString, TypeArray };
    XmlRpcValue() {}
    XmlRpcValue(int v) : type_(TypeInt), i_(v) {}
    XmlRpcValue(double v) : type_(TypeDouble), d_(v) {}
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
namespace stub {
// topic -> type-erased subscriber callback; topic -> captured publications (type-erased copies)
inline std::map<std::string, std::function<void(const void*)>>& subscribers() {
    static std::map<std::string, std::function<void(const void*)>> s;
    return s;
}
inline std::map<std::string, std::vector<std::shared_ptr<const void>>>& publications() {
    static std::map<std::string, std::vector<std::shared_ptr<const void>>> p;
    return p;
}
inline std::function<void()>& on_spin() {
    static std::function<void()> f;
    return f;
}
inline int& spins() {  // spinOnce calls left before ok() turns false
    static int n = 0;
    return n;
}
// service name -> handler (a type-erased pointer to the srv struct); no handler: call() fails
inline std::map<std::string, std::function<bool(void*)>>& services() {
    static std::map<std::string, std::function<bool(void*)>> s;
    return s;
}
template <class M>
void deliver(const std::string& topic, const M& msg) {
    auto it = subscribers().find(topic);
    if (it != subscribers().end()) it->second(&msg);
}
template <class M>
std::vector<M> published(const std::string& topic) {
    std::vector<M> out;
    for (const auto& p : publications()[topic]) out.push_back(*static_cast<const M*>(p.get()));
    return out;
}
}  // namespace stub

inline void init(int&, char**, const std::string&) {}
inline void spin() {}
inline bool ok() { return stub::spins() > 0; }
inline void spinOnce() {
    if (stub::spins() > 0) --stub::spins();
    if (stub::on_spin()) stub::on_spin()();
}

class Time {
  public:
    Time() {}
    explicit Time(double) {}
};
class Duration {
  public:
    explicit Duration(double) {}
    bool sleep() const { return true; }
};

class ServiceServer {
  public:
    ~ServiceServer() {}  // the real one unadvertises on destruction
};
class Subscriber {
  public:
    ~Subscriber() {}  // the real one unsubscribes on destruction
};
class Publisher {
  public:
    Publisher() {}
    explicit Publisher(const std::string& t) : topic_(t) {}
    template <class M>
    void publish(const M& m) const {
        stub::publications()[topic_].push_back(std::make_shared<M>(m));
    }

  private:
    std::string topic_;
};
class ServiceClient {
  public:
    ServiceClient() {}
    explicit ServiceClient(const std::string& s) : service_(s) {}
    template <class S>
    bool call(S& srv) {
        auto it = stub::services().find(service_);
        return it != stub::services().end() && it->second(&srv);
    }
    std::string getService() const { return service_; }

  private:
    std::string service_;
};

class NodeHandle {
  public:
    NodeHandle() {}
    explicit NodeHandle(const std::string&) {}
    bool ok() const { return ros::ok(); }
    bool getParam(const std::string& k, XmlRpc::XmlRpcValue& v) const {
        auto it = params().find(k);
        if (it == params().end()) return false;
        v = it->second;
        return true;
    }
    // roscpp's typed read for numbers (an int stored where a float is read converts); anything else
    // keeps the default
    template <class T, class D>
    bool param(const std::string& k, T& v, const D& d) const {
        v = d;
        if constexpr (std::is_arithmetic<T>::value) {
            auto it = params().find(k);
            if (it == params().end()) return false;
            if (it->second.getType() == XmlRpc::XmlRpcValue::TypeInt) v = (T)(int)it->second;
            else if (it->second.getType() == XmlRpc::XmlRpcValue::TypeDouble && std::is_floating_point<T>::value)
                v = (T)(double)it->second;
            else return false;
            return true;
        }
        return false;
    }
    template <class Req, class Res>
    ServiceServer advertiseService(const std::string&, bool (*)(Req&, Res&)) {
        return ServiceServer();
    }
    template <class M>
    Subscriber subscribe(const std::string& topic, int, void (*cb)(const std::shared_ptr<const M>&)) {
        stub::subscribers()[topic] = [cb](const void* m) {
            cb(std::make_shared<const M>(*static_cast<const M*>(m)));
        };
        return Subscriber();
    }
    template <class M>
    Publisher advertise(const std::string& topic, int) {
        return Publisher(topic);
    }
    template <class S>
    ServiceClient serviceClient(const std::string& name) {
        return ServiceClient(name);
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
#define ROS_INFO(...) (std::fprintf(stderr, "[INFO] "), std::fprintf(stderr, __VA_ARGS__), std::fprintf(stderr, "\n"))
#define ROS_WARN_ONCE(...) (std::fprintf(stderr, "[WARN] "), std::fprintf(stderr, __VA_ARGS__), std::fprintf(stderr, "\n"))
