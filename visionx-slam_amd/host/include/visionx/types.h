// types.h — the minimal value types the reference takes from Eigen, Sophus and OpenCV
// (vcpkg.json:5-15), restated so the host adapters build without those libraries.
//   Vec2d / Vec3d      <- Eigen::Vector2d / Eigen::Vector3d   (frame.h:18, landmark.h:18)
//   SE3d               <- Sophus::SE3d (unit quaternion x y z w + translation), T_cw
//   ImageU8            <- cv::Mat 8UC1 / 8UC3 (frame.h:38), row-major, owned
//   DepthImage         <- cv::Mat CV_16U / CV_32F / CV_64F depth (frame.h:39, tracking.cpp:610-623)
//   DescriptorMat      <- cv::Mat N x 32 CV_8U (frame.h:43-44)
//   DMatch             <- cv::DMatch (feature_matcher.h:12)
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace visionx {

struct Vec2d {
    double x = 0, y = 0;
    Vec2d() = default;
    Vec2d(double x_, double y_) : x(x_), y(y_) {}
    double operator[](int i) const { return i == 0 ? x : y; }
};

struct Vec3d {
    double x = 0, y = 0, z = 0;
    Vec3d() = default;
    Vec3d(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
    double operator[](int i) const { return i == 0 ? x : i == 1 ? y : z; }
    Vec3d operator+(const Vec3d& o) const { return {x + o.x, y + o.y, z + o.z}; }
};

struct SE3d {
    double qx = 0, qy = 0, qz = 0, qw = 1;  // unit quaternion (Sophus/Eigen coefficient order)
    double tx = 0, ty = 0, tz = 0;
    Vec3d operator*(const Vec3d& p) const {  // Sophus SE3 * point (Eigen _transformVector)
        const double ux = qy * p.z - qz * p.y, uy = qz * p.x - qx * p.z, uz = qx * p.y - qy * p.x;
        const double vx = 2 * ux, vy = 2 * uy, vz = 2 * uz;
        return {p.x + qw * vx + (qy * vz - qz * vy) + tx, p.y + qw * vy + (qz * vx - qx * vz) + ty,
                p.z + qw * vz + (qx * vy - qy * vx) + tz};
    }
};

struct ImageU8 {
    int rows = 0, cols = 0, channels = 0;
    std::vector<uint8_t> data;  // rows * cols * channels, row-major
    bool empty() const { return data.empty(); }
    size_t step() const { return (size_t)cols * channels; }
    const uint8_t* ptr() const { return data.data(); }
};

struct DepthImage {
    int rows = 0, cols = 0;
    int type = 0;                // 0 CV_16U (metres * 5000), 1 CV_32F, 2 CV_64F (vx_slam.h VX_DEPTH_*)
    size_t step = 0;             // bytes per row
    std::vector<uint8_t> data;   // rows * step
    bool empty() const { return data.empty(); }
    const uint8_t* ptr() const { return data.data(); }
};

struct DescriptorMat {
    int rows = 0;                // one 32-byte row per feature
    std::vector<uint8_t> data;   // rows * 32
    bool empty() const { return rows == 0; }
    const uint8_t* ptr() const { return data.data(); }
};

struct DMatch {
    int queryIdx = -1, trainIdx = -1, imgIdx = 0;
    float distance = 0.f;
};

}  // namespace visionx
