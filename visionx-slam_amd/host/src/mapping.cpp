// mapping.cpp — KeyFrameLandmarks over vx_depth_landmarks / vx_triangulate (see mapping.h).
#include "visionx/mapping.h"

#include <cstdio>
#include <stdexcept>
#include <string>

namespace visionx {

namespace vxhost {
vx_ctx* ThreadContext();  // feature.cpp
}

static void check(vx_ctx* c, int rc, const char* what) {
    if (rc != VX_OK) throw std::runtime_error(std::string(what) + ": " + vx_last_error(c));
}

static void pose7(const SE3d& T, double* p) {
    p[0] = T.qx; p[1] = T.qy; p[2] = T.qz; p[3] = T.qw;
    p[4] = T.tx; p[5] = T.ty; p[6] = T.tz;
}

// tracking.cpp:586-650
void KeyFrameLandmarks::CreateLandmarksFromDepth(const Frame::Ptr& frame) {
    if (!map_ || !frame) return;
    const DepthImage& depth = frame->Depth();
    if (depth.empty()) return;
    const auto cam = frame->GetCamera();
    if (!cam) return;
    auto& features = frame->Features();
    const int n = (int)features.size();
    uv_.resize(2 * (size_t)n);
    has_.resize(n);
    for (int i = 0; i < n; ++i) {
        uv_[2 * i] = features[i].position.x;
        uv_[2 * i + 1] = features[i].position.y;
        has_[i] = features[i].has_landmark ? 1 : 0;
    }
    const double intr[4] = {cam->fx(), cam->fy(), cam->cx(), cam->cy()};
    double T[7];
    pose7(frame->Pose(), T);
    idx_.assign(n, -1);
    pw_.resize(3 * (size_t)n);
    int created = 0;
    vx_ctx* c = vxhost::ThreadContext();
    check(c, vx_depth_landmarks(c, uv_.data(), has_.data(), n, depth.ptr(), depth.type, depth.rows, depth.cols,
                                (int64_t)depth.step, intr, T, idx_.data(), pw_.data(), &created),
          "vx_depth_landmarks");
    for (int i = 0; i < n; ++i) {  // the loop body of tracking.cpp:634-643, in feature order
        if (idx_[i] < 0) continue;
        const double* p = &pw_[3 * (size_t)idx_[i]];
        auto lm = std::make_shared<Landmark>(landmark_id_++, Vec3d(p[0], p[1], p[2]));
        lm->AddObservation(frame->Id(), (size_t)i);
        map_->InsertLandmark(lm);
        features[i].landmark_id_ = lm->Id();
        features[i].has_landmark = true;
        features[i].is_outlier = false;
    }
}

// tracking.cpp:856-929
void KeyFrameLandmarks::TriangulateWithLastKeyFrame(Frame::Ptr last_frame, Frame::Ptr curr_frame) {
    if (!last_frame || !curr_frame) {
        std::fprintf(stderr, "[TriangulateWithLastKeyFrame] Invalid frames.\n");
        return;
    }
    std::vector<DMatch> matches;
    matcher_->Match(last_frame, curr_frame, matches);
    auto cam = curr_frame->GetCamera();
    auto cam1 = last_frame->GetCamera();
    if (!cam || !cam1 || matches.empty()) return;
    auto& f1 = last_frame->Features();
    auto& f2 = curr_frame->Features();
    const int n1 = (int)f1.size(), n2 = (int)f2.size(), nm = (int)matches.size();
    uv_.resize(2 * (size_t)n1);
    has_.resize(n1);
    uv2_.resize(2 * (size_t)n2);
    has2_.resize(n2);
    for (int i = 0; i < n1; ++i) {
        uv_[2 * i] = f1[i].position.x;
        uv_[2 * i + 1] = f1[i].position.y;
        has_[i] = f1[i].has_landmark ? 1 : 0;
    }
    for (int i = 0; i < n2; ++i) {
        uv2_[2 * i] = f2[i].position.x;
        uv2_[2 * i + 1] = f2[i].position.y;
        has2_[i] = f2[i].has_landmark ? 1 : 0;
    }
    m_.resize(nm);
    for (int k = 0; k < nm; ++k) m_[k] = vx_match{matches[k].queryIdx, matches[k].trainIdx, matches[k].distance};
    const double i1[4] = {cam1->fx(), cam1->fy(), cam1->cx(), cam1->cy()};
    const double i2[4] = {cam->fx(), cam->fy(), cam->cx(), cam->cy()};
    double T1[7], T2[7];
    pose7(last_frame->Pose(), T1);
    pose7(curr_frame->Pose(), T2);
    idx_.assign(nm, -1);
    pw_.resize(3 * (size_t)nm);
    int created = 0;
    vx_ctx* c = vxhost::ThreadContext();
    check(c, vx_triangulate(c, uv_.data(), has_.data(), n1, i1, T1, uv2_.data(), has2_.data(), n2, i2, T2, m_.data(),
                            nm, options_.triangulation_min_angle_deg, options_.triangulation_max_reproj_error,
                            idx_.data(), pw_.data(), &created),
          "vx_triangulate");
    for (int k = 0; k < nm; ++k) {  // the loop body of tracking.cpp:915-925, in match order
        if (idx_[k] < 0) continue;
        const double* p = &pw_[3 * (size_t)idx_[k]];
        const auto& m = matches[k];
        auto lm = std::make_shared<Landmark>(landmark_id_++, Vec3d(p[0], p[1], p[2]));
        lm->AddObservation(last_frame->Id(), (size_t)m.queryIdx);
        lm->AddObservation(curr_frame->Id(), (size_t)m.trainIdx);
        map_->InsertLandmark(lm);
        f1[m.queryIdx].landmark_id_ = lm->Id();
        f1[m.queryIdx].has_landmark = true;
        f1[m.queryIdx].is_outlier = false;
        f2[m.trainIdx].landmark_id_ = lm->Id();
        f2[m.trainIdx].has_landmark = true;
        f2[m.trainIdx].is_outlier = false;
    }
}

}  // namespace visionx
