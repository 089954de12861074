// device_map.h — visionx::Map kept resident on the GPU (vx_dmap, include/vx_slam.h) for the drop-in
// LocalBA: the integration forwards the reference's map edits here at the points Tracking makes them
// (INTEGRATION.md §3), and LocalBA::Optimize(map, ref_kf) then runs as one vx_ba_optimize_dmap call
// instead of walking the map under its mutexes (local_ba.cpp:77-104, map.cpp:31-47) and shipping a
// snapshot every keyframe.
//
//   Map::InsertKeyFrame          (map.cpp:5-8, tracking.cpp:255,581)    -> InsertKeyFrame
//   Map::InsertLandmark          (map.cpp:10-13, tracking.cpp:644,918)  -> InsertLandmark
//   Landmark::AddObservation     (landmark.h:32-35, tracking.cpp:916)   -> AddObservation
//   Landmark::RemoveObservation  (landmark.h:37-40, tracking.cpp:766)   -> RemoveObservation
//   Map::RemoveKeyFrame          (map.cpp:15-18, tracking.cpp:772)      -> RemoveKeyFrame
//   Map::RemoveLandmark          (map.cpp:20-23, tracking.cpp:746)      -> RemoveLandmark
//   Landmark::SetBad             (landmark.h:56-59, tracking.cpp:671)   -> SetBad
//   Frame::SetPose               (frame.h:34, tracking.cpp:447,541)     -> SetPose
//   Feature::landmark_id_ / has_landmark / is_outlier edits
//                                (tracking.cpp:646-648,741-743,767-769,920-925) -> UpdateFeatures
//
// Landmark insertions and observation additions are queued and sent in batches (one host-to-device
// copy per batch) when any other edit or an Optimize comes; order is preserved.  Not thread-safe:
// like the reference's hot path it is driven from the tracking thread.
#pragma once

#include <cstdint>
#include <memory>
#include <unordered_map>
#include <vector>

#include "vx_slam.h"
#include "visionx/frame.h"

namespace visionx {

class DeviceMap {
public:
    using Ptr = std::shared_ptr<DeviceMap>;
    explicit DeviceMap(vx_ctx* ctx);
    DeviceMap();  // on the calling thread's context (vxhost::ThreadContext)
    ~DeviceMap();
    DeviceMap(const DeviceMap&) = delete;
    DeviceMap& operator=(const DeviceMap&) = delete;

    void InsertKeyFrame(const Frame::Ptr& kf);
    // the landmark and the observations it already holds
    void InsertLandmark(const Landmark::Ptr& lm);
    void AddObservation(uint64_t lm_id, uint64_t kf_id, size_t feature_idx);
    void RemoveObservation(uint64_t lm_id, uint64_t kf_id);
    void RemoveKeyFrame(uint64_t kf_id);
    void RemoveLandmark(uint64_t lm_id);
    void SetBad(uint64_t lm_id, bool bad = true);
    void SetPose(uint64_t kf_id, const SE3d& T_cw);
    // re-reads features `idx` of keyframe kf (landmark_id_, has_landmark, is_outlier)
    void UpdateFeatures(const Frame::Ptr& kf, const std::vector<int>& idx);
    // every keyframe (id order) and landmark of an existing map, with their observations
    void Mirror(const Map& map);

    // queued edits to the device (Optimize does this itself)
    void Flush();
    vx_dmap* handle() { return dm_; }
    vx_ctx* context() { return ctx_; }
    // the objects behind the resident rows, for writing results back (nullptr: removed)
    // (references: no reference-count traffic in the per-landmark write-back loop)
    const Frame::Ptr& FrameAt(int64_t row) const { return row < (int64_t)frames_.size() ? frames_[row] : kNoFrame; }
    const Landmark::Ptr& LandmarkAt(int64_t row) const {
        return row < (int64_t)landmarks_.size() ? landmarks_[row] : kNoLandmark;
    }

private:
    void Check(int rc, const char* what) const;
    void FlushLandmarks();
    void FlushObservations();
    vx_ctx* ctx_ = nullptr;
    vx_dmap* dm_ = nullptr;
    inline static const Frame::Ptr kNoFrame{};
    inline static const Landmark::Ptr kNoLandmark{};
    std::vector<Frame::Ptr> frames_;        // by resident keyframe row
    std::vector<Landmark::Ptr> landmarks_;  // by resident landmark row
    std::unordered_map<uint64_t, int64_t> lm_row_, kf_row_;
    // queued: landmarks (id, position, bad, object), then observations (landmark id, keyframe id, index)
    std::vector<uint64_t> q_lm_id_;
    std::vector<double> q_lm_pos_;
    std::vector<uint8_t> q_lm_bad_;
    std::vector<Landmark::Ptr> q_lm_obj_;
    std::vector<uint64_t> q_ob_lm_, q_ob_kf_, q_ob_fi_;
};

}  // namespace visionx
