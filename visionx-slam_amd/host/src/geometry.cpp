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

}  // namespace visionx
