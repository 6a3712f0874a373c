// Stand-in for <tf/transform_listener.h> (compile checks, plus the harness: lookupTransform returns
// tf::stub::pose(), a row-major 3x4 [R | t], or throws when tf::stub::fail() is set).
#pragma once
#include <stdexcept>
#include <string>

#include "ros/ros.h"

namespace tf {
class Vector3 {
  public:
    Vector3(double x = 0, double y = 0, double z = 0) : v_{x, y, z} {}
    double x() const { return v_[0]; }
    double y() const { return v_[1]; }
    double z() const { return v_[2]; }
    const double& operator[](int k) const { return v_[k]; }

  private:
    double v_[3];
};
class Matrix3x3 {
  public:
    const Vector3& operator[](int r) const { return row_[r]; }
    Vector3 row_[3];
};
class StampedTransform {
  public:
    const Matrix3x3& getBasis() const { return basis_; }
    const Vector3& getOrigin() const { return origin_; }
    Matrix3x3 basis_;
    Vector3 origin_;
};
class TransformException : public std::runtime_error {
  public:
    explicit TransformException(const std::string& w) : std::runtime_error(w) {}
};
namespace stub {
inline double* pose() {
    static double p[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    return p;
}
inline bool& fail() {
    static bool f = false;
    return f;
}
}  // namespace stub
class TransformListener {
  public:
    bool waitForTransform(const std::string&, const std::string&, const ros::Time&, const ros::Duration&) const {
        return !stub::fail();
    }
    void lookupTransform(const std::string&, const std::string&, const ros::Time&, StampedTransform& t) const {
        if (stub::fail()) throw TransformException("no transform (stub)");
        const double* p = stub::pose();
        for (int r = 0; r < 3; ++r) t.basis_.row_[r] = Vector3(p[4 * r], p[4 * r + 1], p[4 * r + 2]);
        t.origin_ = Vector3(p[3], p[7], p[11]);
    }
};
}  // namespace tf
