// mapping.h — the landmark-creation half of Tracking::CreateKeyFrame (core/frontend/tracking.cpp:
// 577-580), run on every new keyframe right before LocalBA, over the MI355X C ABI:
//
//   CreateLandmarksFromDepth     tracking.cpp:586-650   -> vx_depth_landmarks
//   TriangulateWithLastKeyFrame  tracking.cpp:856-929   -> Match() + vx_triangulate
//   (TriangulatePoint / ProjectionMatrix, tracking.cpp:843-854, 931-945, run inside the kernel)
//
// Same member names, option names / defaults (Tracking::Options, tracking.h:43-44) and side effects
// as the reference: landmarks get consecutive ids from landmark_id_, observations are added and
// the features' landmark_id_ / has_landmark / is_outlier are set in the reference's order.
#pragma once

#include <memory>
#include <vector>

#include "visionx/feature.h"

namespace visionx {

class KeyFrameLandmarks {
public:
    struct Options {
        double triangulation_max_reproj_error = 5.0;  // tracking.h:43
        double triangulation_min_angle_deg = 1.0;     // tracking.h:44
    };
    KeyFrameLandmarks(Map::Ptr map, FeatureMatcher::Ptr matcher, const Options& options)
        : map_(std::move(map)), matcher_(std::move(matcher)), options_(options) {}

    void CreateLandmarksFromDepth(const Frame::Ptr& frame);
    void TriangulateWithLastKeyFrame(Frame::Ptr last_frame, Frame::Ptr curr_frame);

    uint64_t landmark_id_ = 0;  // Tracking::landmark_id_ (tracking.h): next landmark id

private:
    Map::Ptr map_;
    FeatureMatcher::Ptr matcher_;
    Options options_;
    std::vector<double> uv_, uv2_, pw_;
    std::vector<uint8_t> has_, has2_;
    std::vector<int32_t> idx_;
    std::vector<vx_match> m_;
};

}  // namespace visionx
