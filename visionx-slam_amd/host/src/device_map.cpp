// device_map.cpp — visionx::DeviceMap over vx_dmap (see device_map.h).
#include "visionx/device_map.h"

#include <stdexcept>
#include <string>

#include "visionx/feature.h"

namespace visionx {

DeviceMap::DeviceMap(vx_ctx* ctx) : ctx_(ctx) { Check(vx_dmap_create(ctx_, &dm_), "vx_dmap_create"); }
DeviceMap::DeviceMap() : DeviceMap(vxhost::ThreadContext()) {}
DeviceMap::~DeviceMap() {
    if (dm_) vx_dmap_destroy(dm_);
}

void DeviceMap::Check(int rc, const char* what) const {
    if (rc != VX_OK) throw std::runtime_error(std::string(what) + ": " + vx_last_error(ctx_));
}

static uint8_t FeatureFlags(const Feature& f) { return (f.has_landmark ? 1 : 0) | (f.is_outlier ? 2 : 0); }

void DeviceMap::InsertKeyFrame(const Frame::Ptr& kf) {
    Flush();
    const SE3d T = kf->Pose();
    const double pose[7] = {T.qx, T.qy, T.qz, T.qw, T.tx, T.ty, T.tz};
    const auto cam = kf->GetCamera();
    double intr[4] = {0, 0, 0, 0};
    if (cam) {
        intr[0] = cam->fx();
        intr[1] = cam->fy();
        intr[2] = cam->cx();
        intr[3] = cam->cy();
    }
    const auto& feats = kf->Features();
    std::vector<double> uv(2 * feats.size());
    std::vector<uint64_t> lm(feats.size());
    std::vector<uint8_t> fl(feats.size());
    for (size_t i = 0; i < feats.size(); ++i) {
        uv[2 * i] = feats[i].position.x;
        uv[2 * i + 1] = feats[i].position.y;
        lm[i] = feats[i].landmark_id_;
        fl[i] = FeatureFlags(feats[i]);
    }
    Check(vx_dmap_add_keyframe(dm_, kf->Id(), pose, intr, cam ? 1 : 0, (int)feats.size(), uv.data(), lm.data(),
                               fl.data()),
          "vx_dmap_add_keyframe");
    kf_row_[kf->Id()] = (int64_t)frames_.size();
    frames_.push_back(kf);
}

void DeviceMap::InsertLandmark(const Landmark::Ptr& lm) {
    const Vec3d p = lm->Position();
    q_lm_id_.push_back(lm->Id());
    q_lm_pos_.insert(q_lm_pos_.end(), {p.x, p.y, p.z});
    q_lm_bad_.push_back(lm->IsBad() ? 1 : 0);
    q_lm_obj_.push_back(lm);
    for (const auto& [kid, fi] : lm->Observations()) AddObservation(lm->Id(), kid, fi);
}

void DeviceMap::AddObservation(uint64_t lm_id, uint64_t kf_id, size_t feature_idx) {
    q_ob_lm_.push_back(lm_id);
    q_ob_kf_.push_back(kf_id);
    q_ob_fi_.push_back((uint64_t)feature_idx);
}

void DeviceMap::FlushLandmarks() {
    if (q_lm_id_.empty()) return;
    Check(vx_dmap_add_landmarks(dm_, (int)q_lm_id_.size(), q_lm_id_.data(), q_lm_pos_.data(), q_lm_bad_.data()),
          "vx_dmap_add_landmarks");
    for (auto& l : q_lm_obj_) {
        lm_row_[l->Id()] = (int64_t)landmarks_.size();
        landmarks_.push_back(std::move(l));
    }
    q_lm_id_.clear();
    q_lm_pos_.clear();
    q_lm_bad_.clear();
    q_lm_obj_.clear();
}

void DeviceMap::FlushObservations() {
    if (q_ob_lm_.empty()) return;
    Check(vx_dmap_add_observations(dm_, (int)q_ob_lm_.size(), q_ob_lm_.data(), q_ob_kf_.data(), q_ob_fi_.data()),
          "vx_dmap_add_observations");
    q_ob_lm_.clear();
    q_ob_kf_.clear();
    q_ob_fi_.clear();
}

// landmarks before observations: an observation names a landmark inserted before it, and the order
// inside each queue is the call order
void DeviceMap::Flush() {
    FlushLandmarks();
    FlushObservations();
}

void DeviceMap::RemoveObservation(uint64_t lm_id, uint64_t kf_id) {
    Flush();
    Check(vx_dmap_remove_observations(dm_, 1, &lm_id, &kf_id), "vx_dmap_remove_observations");
}

void DeviceMap::RemoveKeyFrame(uint64_t kf_id) {
    Flush();
    Check(vx_dmap_remove_keyframe(dm_, kf_id), "vx_dmap_remove_keyframe");
    auto it = kf_row_.find(kf_id);
    if (it != kf_row_.end()) {
        frames_[it->second] = nullptr;
        kf_row_.erase(it);
    }
}

void DeviceMap::RemoveLandmark(uint64_t lm_id) {
    Flush();
    Check(vx_dmap_remove_landmarks(dm_, 1, &lm_id), "vx_dmap_remove_landmarks");
    auto it = lm_row_.find(lm_id);
    if (it != lm_row_.end()) {
        landmarks_[it->second] = nullptr;
        lm_row_.erase(it);
    }
}

void DeviceMap::SetBad(uint64_t lm_id, bool bad) {
    Flush();
    const uint8_t b = bad ? 1 : 0;
    Check(vx_dmap_set_landmark_bad(dm_, 1, &lm_id, &b), "vx_dmap_set_landmark_bad");
}

void DeviceMap::SetPose(uint64_t kf_id, const SE3d& T) {
    Flush();
    const double pose[7] = {T.qx, T.qy, T.qz, T.qw, T.tx, T.ty, T.tz};
    Check(vx_dmap_set_poses(dm_, 1, &kf_id, pose), "vx_dmap_set_poses");
}

void DeviceMap::UpdateFeatures(const Frame::Ptr& kf, const std::vector<int>& idx) {
    Flush();
    const auto& feats = kf->Features();
    std::vector<uint64_t> lm(idx.size());
    std::vector<uint8_t> fl(idx.size());
    for (size_t i = 0; i < idx.size(); ++i) {
        const Feature& f = feats.at((size_t)idx[i]);
        lm[i] = f.landmark_id_;
        fl[i] = FeatureFlags(f);
    }
    Check(vx_dmap_set_features(dm_, kf->Id(), (int)idx.size(), idx.data(), lm.data(), fl.data()),
          "vx_dmap_set_features");
}

void DeviceMap::Mirror(const Map& map) {
    for (const auto& kv : map.KeyFrames()) InsertKeyFrame(kv.second);
    for (const auto& kv : map.Landmarks()) InsertLandmark(kv.second);
    Flush();
}

}  // namespace visionx
