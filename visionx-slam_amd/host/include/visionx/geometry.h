// geometry.h — the geometry RANSAC call of Tracking::TrackWithPnP (core/frontend/tracking.cpp:
// 414-447) over the MI355X C ABI:
//
//   cv::solvePnPRansac(pts_3d, pts_2d, K, cv::Mat(), rvec, tvec, false, iterations,
//                      max_reproj_error, 0.99, inliers)          -> vx_pnp_ransac
//   cv::Rodrigues(rvec, R); Sophus::SE3d T_cw(R, t)              -> PoseFromRvecTvec
//
// Same argument order and meaning as the OpenCV call the reference makes (objectPoints as
// cv::Point3f, imagePoints as cv::Point2f, K from the frame's Camera, no distortion), same return
// value (model found) and outputs (rvec, tvec, inlier indices ascending).
#pragma once

#include <vector>

#include "vx_slam.h"
#include "visionx/frame.h"

namespace visionx {

struct Point3f {  // cv::Point3f
    float x = 0, y = 0, z = 0;
    Point3f() = default;
    Point3f(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
};
struct Point2f {  // cv::Point2f
    float x = 0, y = 0;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};

// useExtrinsicGuess must be false (the reference's value; the GPU path has no guess input):
// std::invalid_argument otherwise.  inliers may be null.
bool SolvePnPRansac(const std::vector<Point3f>& objectPoints, const std::vector<Point2f>& imagePoints,
                    const Camera& K, Vec3d& rvec, Vec3d& tvec, bool useExtrinsicGuess = false,
                    int iterationsCount = 100, float reprojectionError = 8.0f, double confidence = 0.99,
                    std::vector<int>* inliers = nullptr);

// cv::Rodrigues + Sophus::SE3d(R, t) (tracking.cpp:429-447): the unit quaternion of rvec
SE3d PoseFromRvecTvec(const Vec3d& rvec, const Vec3d& tvec);

// E = cv::findEssentialMat(pts_last, pts_curr, K, cv::RANSAC, prob, threshold, mask);
// inliers = cv::recoverPose(E, pts_last, pts_curr, K, R, t, mask)   (tracking.cpp:521-528)
// in one call: returns -1 when findEssentialMat finds no E (E.empty()), else recoverPose's inlier
// count; R (row-major) and t give T_cl (x_curr = R x_last + t, |t| = 1); mask (optional) is
// recoverPose's output mask, E (optional) the row-major essential matrix.
int FindEssentialMatRecoverPose(const std::vector<Point2f>& pts_last, const std::vector<Point2f>& pts_curr,
                                const Camera& K, double R[9], Vec3d& t, std::vector<uint8_t>* mask = nullptr,
                                double prob = 0.999, double threshold = 1.0, double E[9] = nullptr);

// Sophus::SE3d T_cl(R, t) of a rotation matrix (row-major) and translation
SE3d PoseFromRt(const double R[9], const Vec3d& t);

}  // namespace visionx
