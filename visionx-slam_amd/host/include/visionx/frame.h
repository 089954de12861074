// frame.h / camera.h / landmark.h / map.h mirrors — same member names and locking semantics as
// the reference data model (core/frame/frame.h:16-64, core/camera/camera.h:8-37,
// core/map/landmark.h:12-68, core/map/map.h:13-34) over the restated value types.
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "visionx/types.h"

namespace visionx {

class Camera {  // camera.h:8-37 (only the getters are on the hot path, camera.h:29-32)
public:
    using Ptr = std::shared_ptr<Camera>;
    Camera(double fx, double fy, double cx, double cy, double k1 = 0, double k2 = 0, double p1 = 0,
           double p2 = 0)
        : fx_(fx), fy_(fy), cx_(cx), cy_(cy), k1_(k1), k2_(k2), p1_(p1), p2_(p2) {}
    double fx() const { return fx_; }
    double fy() const { return fy_; }
    double cx() const { return cx_; }
    double cy() const { return cy_; }

private:
    double fx_, fy_, cx_, cy_, k1_, k2_, p1_, p2_;
};

struct Feature {  // frame.h:16-23
    Vec2d position;
    float response = 0.0f;
    uint64_t landmark_id_ = 0;
    bool has_landmark = false;
    bool is_outlier = false;
};

class Frame {  // frame.h:25-64
public:
    using Ptr = std::shared_ptr<Frame>;
    Frame(uint64_t id, double timestamp, std::shared_ptr<Camera> camera, const ImageU8& image,
          const DepthImage& depth = DepthImage())
        : id_(id), timestamp_(timestamp), camera_(std::move(camera)), image_(image), depth_(depth) {}

    SE3d Pose() const {
        std::lock_guard<std::mutex> lock(pose_mutex_);
        return T_cw_;
    }
    void SetPose(const SE3d& T_cw) {
        std::lock_guard<std::mutex> lock(pose_mutex_);
        T_cw_ = T_cw;
    }
    uint64_t Id() const { return id_; }
    double Timestamp() const { return timestamp_; }
    const ImageU8& Image() const { return image_; }
    const DepthImage& Depth() const { return depth_; }
    std::vector<Feature>& Features() { return features_; }
    const std::vector<Feature>& Features() const { return features_; }
    DescriptorMat& Descriptors() { return descriptors_; }
    const DescriptorMat& Descriptors() const { return descriptors_; }
    std::shared_ptr<Camera> GetCamera() const { return camera_; }

private:
    uint64_t id_ = 0;
    double timestamp_ = 0.0;
    SE3d T_cw_;
    mutable std::mutex pose_mutex_;
    std::shared_ptr<Camera> camera_;
    ImageU8 image_;
    DepthImage depth_;
    std::vector<Feature> features_;
    DescriptorMat descriptors_;
};

class Landmark {  // landmark.h:12-68
public:
    using Ptr = std::shared_ptr<Landmark>;
    Landmark(uint64_t id, const Vec3d& pos) : id_(id), pos_(pos) {}
    uint64_t Id() const { return id_; }
    Vec3d Position() const {
        std::lock_guard<std::mutex> lock(mutex_);
        return pos_;
    }
    void SetPosition(const Vec3d& pos) {
        std::lock_guard<std::mutex> lock(mutex_);
        pos_ = pos;
    }
    void AddObservation(uint64_t keyframe_id, size_t feature_idx) {
        std::lock_guard<std::mutex> lock(mutex_);
        observations_[keyframe_id] = feature_idx;
    }
    void RemoveObservation(uint64_t keyframe_id) {
        std::lock_guard<std::mutex> lock(mutex_);
        observations_.erase(keyframe_id);
    }
    size_t ObservationCount() const {
        std::lock_guard<std::mutex> lock(mutex_);
        return observations_.size();
    }
    const std::unordered_map<uint64_t, size_t>& Observations() const { return observations_; }
    bool IsBad() const {
        std::lock_guard<std::mutex> lock(mutex_);
        return is_bad_;
    }
    void SetBad(bool bad = true) {
        std::lock_guard<std::mutex> lock(mutex_);
        is_bad_ = bad;
    }

private:
    uint64_t id_;
    Vec3d pos_;
    std::unordered_map<uint64_t, size_t> observations_;
    mutable std::mutex mutex_;
    bool is_bad_ = false;
};

class Map {  // map.h:13-34
public:
    using Ptr = std::shared_ptr<Map>;
    void InsertKeyFrame(Frame::Ptr frame) {
        std::lock_guard<std::mutex> lock(mutex_);
        keyframes_[frame->Id()] = frame;
    }
    void InsertLandmark(Landmark::Ptr landmark) {
        std::lock_guard<std::mutex> lock(mutex_);
        landmarks_[landmark->Id()] = landmark;
    }
    void RemoveKeyFrame(uint64_t id) {
        std::lock_guard<std::mutex> lock(mutex_);
        keyframes_.erase(id);
    }
    void RemoveLandmark(uint64_t id) {
        std::lock_guard<std::mutex> lock(mutex_);
        landmarks_.erase(id);
    }
    void removeAll() {
        std::lock_guard<std::mutex> lock(mutex_);
        keyframes_.clear();
        landmarks_.clear();
    }
    Frame::Ptr GetFrame(uint64_t id) const {
        std::lock_guard<std::mutex> lock(mutex_);
        auto it = keyframes_.find(id);
        return it == keyframes_.end() ? nullptr : it->second;
    }
    const std::map<uint64_t, Frame::Ptr>& KeyFrames() const { return keyframes_; }
    size_t LandmarkSize() const {
        std::lock_guard<std::mutex> lock(mutex_);
        return landmarks_.size();
    }
    Landmark::Ptr GetLandmark(uint64_t id) const {
        std::lock_guard<std::mutex> lock(mutex_);
        auto it = landmarks_.find(id);
        return it == landmarks_.end() ? nullptr : it->second;
    }
    const std::unordered_map<uint64_t, Landmark::Ptr>& Landmarks() const { return landmarks_; }

private:
    std::map<uint64_t, Frame::Ptr> keyframes_;
    std::unordered_map<uint64_t, Landmark::Ptr> landmarks_;
    mutable std::mutex mutex_;
};

}  // namespace visionx
