// geometry.cpp — SolvePnPRansac over vx_pnp_ransac (see geometry.h).
#include "visionx/geometry.h"

#include <cmath>
#include <stdexcept>
#include <string>

namespace visionx {

namespace vxhost {
vx_ctx* ThreadContext();  // feature.cpp
}

bool SolvePnPRansac(const std::vector<Point3f>& objectPoints, const std::vector<Point2f>& imagePoints,
                    const Camera& K, Vec3d& rvec, Vec3d& tvec, bool useExtrinsicGuess, int iterationsCount,
                    float reprojectionError, double confidence, std::vector<int>* inliers) {
    if (useExtrinsicGuess) throw std::invalid_argument("SolvePnPRansac: useExtrinsicGuess is not supported");
    if (objectPoints.size() != imagePoints.size())
        throw std::invalid_argument("SolvePnPRansac: objectPoints / imagePoints size mismatch");
    static_assert(sizeof(Point3f) == 3 * sizeof(float) && sizeof(Point2f) == 2 * sizeof(float), "packed points");
    const int n = (int)objectPoints.size();
    vx_pnp_options o;
    vx_pnp_default_options(n, &o);
    o.max_iterations = iterationsCount;
    o.reproj_error = reprojectionError;
    o.confidence = confidence;
    const double intr[4] = {K.fx(), K.fy(), K.cx(), K.cy()};
    std::vector<uint8_t> mask(n > 0 ? n : 1);
    vx_pnp_result r;
    vx_ctx* c = vxhost::ThreadContext();
    const int rc = vx_pnp_ransac(c, reinterpret_cast<const float*>(objectPoints.data()),
                                 reinterpret_cast<const float*>(imagePoints.data()), n, intr, &o, mask.data(), &r);
    if (rc != VX_OK) throw std::runtime_error(std::string("vx_pnp_ransac: ") + vx_last_error(c));
    if (inliers) {
        inliers->clear();
        for (int i = 0; i < n && r.ok; ++i)
            if (mask[i]) inliers->push_back(i);
    }
    if (!r.ok) return false;
    rvec = Vec3d(r.rvec[0], r.rvec[1], r.rvec[2]);
    tvec = Vec3d(r.tvec[0], r.tvec[1], r.tvec[2]);
    return true;
}

SE3d PoseFromRvecTvec(const Vec3d& rvec, const Vec3d& tvec) {
    const double th = std::sqrt(rvec.x * rvec.x + rvec.y * rvec.y + rvec.z * rvec.z);
    const double s = th > 0.0 ? std::sin(0.5 * th) / th : 0.5;
    SE3d T;
    T.qx = rvec.x * s;
    T.qy = rvec.y * s;
    T.qz = rvec.z * s;
    T.qw = std::cos(0.5 * th);
    T.tx = tvec.x;
    T.ty = tvec.y;
    T.tz = tvec.z;
    return T;
}

int FindEssentialMatRecoverPose(const std::vector<Point2f>& pts_last, const std::vector<Point2f>& pts_curr,
                                const Camera& K, double R[9], Vec3d& t, std::vector<uint8_t>* mask, double prob,
                                double threshold, double E[9]) {
    if (pts_last.size() != pts_curr.size())
        throw std::invalid_argument("FindEssentialMatRecoverPose: point list size mismatch");
    const int n = (int)pts_last.size();
    vx_essential_options o;
    vx_essential_default_options(&o);
    o.confidence = prob;
    o.threshold = threshold;
    const double intr[4] = {K.fx(), K.fy(), K.cx(), K.cy()};
    std::vector<uint8_t> m(n > 0 ? n : 1);
    vx_essential_result r;
    vx_ctx* c = vxhost::ThreadContext();
    const int rc = vx_essential_ransac(c, reinterpret_cast<const float*>(pts_last.data()),
                                       reinterpret_cast<const float*>(pts_curr.data()), n, intr, &o, m.data(), &r);
    if (rc != VX_OK) throw std::runtime_error(std::string("vx_essential_ransac: ") + vx_last_error(c));
    if (mask) mask->assign(m.begin(), m.begin() + n);
    if (!r.ok) return -1;
    for (int k = 0; k < 9; ++k) {
        R[k] = r.R[k];
        if (E) E[k] = r.E[k];
    }
    t = Vec3d(r.t[0], r.t[1], r.t[2]);
    return r.n_inliers;
}

// Shepperd's method (largest of trace / diagonal), as Eigen::Quaterniond(Matrix3d)
SE3d PoseFromRt(const double* R, const Vec3d& t) {
    double x, y, z, w;
    const double tr = R[0] + R[4] + R[8];
    if (tr > 0.0) {
        const double s = std::sqrt(tr + 1.0) * 2.0;
        w = 0.25 * s; x = (R[7] - R[5]) / s; y = (R[2] - R[6]) / s; z = (R[3] - R[1]) / s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        const double s = std::sqrt(1.0 + R[0] - R[4] - R[8]) * 2.0;
        w = (R[7] - R[5]) / s; x = 0.25 * s; y = (R[1] + R[3]) / s; z = (R[2] + R[6]) / s;
    } else if (R[4] > R[8]) {
        const double s = std::sqrt(1.0 + R[4] - R[0] - R[8]) * 2.0;
        w = (R[2] - R[6]) / s; x = (R[1] + R[3]) / s; y = 0.25 * s; z = (R[5] + R[7]) / s;
    } else {
        const double s = std::sqrt(1.0 + R[8] - R[0] - R[4]) * 2.0;
        w = (R[3] - R[1]) / s; x = (R[2] + R[6]) / s; y = (R[5] + R[7]) / s; z = 0.25 * s;
    }
    const double inv = 1.0 / std::sqrt(x * x + y * y + z * z + w * w);
    SE3d T;
    T.qx = x * inv; T.qy = y * inv; T.qz = z * inv; T.qw = w * inv;
    T.tx = t.x; T.ty = t.y; T.tz = t.z;
    return T;
}

}  // namespace visionx
