// feature.h — the reference's plugin interfaces and their MI355X implementations.
//
//   FeatureExtractor  core/feature/feature_extractor.h:10-16   (virtual void Extract(Frame&))
//   FeatureMatcher    core/feature/feature_matcher.h:7-13      (virtual int Match(last, curr, matches))
//   ORBExtractor      core/feature/orb_extractor.h:9-19        -> vx_orb_extract (include/vx_slam.h)
//   ORBMatcher        core/feature/orb_matcher.h:11-26         -> vx_match_knn2_ratio
//   LocalBA           core/backend/local_ba.h:10-27            -> vx_ba_optimize_map (snapshot) or
//                                                               vx_ba_optimize_dmap (DeviceMap attached)
//
// Same class names, constructor defaults and member signatures as the reference, so
// core/system/system.cpp:15-16 and core/frontend/tracking.cpp:25-34 compile against them
// unchanged.  Device work goes through one vx_ctx per calling thread (the reference runs the hot
// path on its single tracking thread, core/system/system.cpp:39-52).
#pragma once

#include <memory>
#include <utility>
#include <vector>

#include "vx_slam.h"
#include "visionx/frame.h"

namespace visionx {

class FeatureExtractor {
public:
    using Ptr = std::shared_ptr<FeatureExtractor>;
    virtual ~FeatureExtractor() = default;
    virtual void Extract(Frame& frame) = 0;
};

class FeatureMatcher {
public:
    using Ptr = std::shared_ptr<FeatureMatcher>;
    virtual ~FeatureMatcher() = default;
    virtual int Match(const Frame::Ptr& last, const Frame::Ptr& curr, std::vector<DMatch>& matches) = 0;
};

class ORBExtractor : public FeatureExtractor {
public:
    ORBExtractor(int n_features = 1000, float scale_factor = 1.2f, int n_levels = 8);
    void Extract(Frame& frame) override;
    // Extension for multi-camera rigs (the C5 workload): Extract() of every frame of one time step
    // in one batched launch sequence (vx_orb_extract_batch).  Each frame's Features() /
    // Descriptors() end up exactly as Extract(frame) leaves them; frames of differing size or
    // channel count, or empty ones, are extracted one by one.
    void ExtractBatch(const std::vector<Frame::Ptr>& frames);

private:
    vx_orb_params params_;
    std::vector<vx_keypoint> kp_;
    std::vector<uint8_t> desc_;
};

class ORBMatcher : public FeatureMatcher {
public:
    struct Options {
        float nn_ratio = 0.8f;
        int min_matches = 50;
    };
    ORBMatcher() : ORBMatcher(Options()) {}
    explicit ORBMatcher(const Options& options);
    int Match(const Frame::Ptr& last, const Frame::Ptr& curr, std::vector<DMatch>& matches) override;
    // Extension: Match(last_i, curr_i, matches[i]) for up to VX_MAX_MATCH_PAIRS pairs in one launch
    // pair (vx_match_knn2_ratio_batch); returns the per-pair counts Match() would return.
    std::vector<int> MatchBatch(const std::vector<std::pair<Frame::Ptr, Frame::Ptr>>& pairs,
                                std::vector<std::vector<DMatch>>& matches);

private:
    void Finish(std::vector<DMatch>& matches, int n);
    Options options_;
    std::vector<vx_match> buf_;
};

// Flattened window of a Map (what LocalBA::Optimize can read or write), laid out as vx_map_view.
// Allocator of FlatMap's large arrays: page-locked host memory (vx_host_alloc), so that the
// snapshot's upload in vx_ba_optimize_map is a DMA from these very arrays (pageable ones go through
// the runtime's bounce buffers: ~0.5 ms of the C3 call).  The arrays keep their
// capacity from call to call, so the (slow) page-locked allocation happens only while they grow.
template <class T>
struct PinnedAllocator {
    using value_type = T;
    PinnedAllocator() = default;
    template <class U>
    PinnedAllocator(const PinnedAllocator<U>&) {}
    T* allocate(size_t n) {
        void* p = vx_host_alloc(n * sizeof(T));
        if (!p) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) { vx_host_free(p); }
    template <class U>
    bool operator==(const PinnedAllocator<U>&) const { return true; }
    template <class U>
    bool operator!=(const PinnedAllocator<U>&) const { return false; }
};
template <class T>
using pinned_vector = std::vector<T, PinnedAllocator<T>>;

struct FlatMap {
    std::vector<uint64_t> kf_id;
    std::vector<double> kf_pose, kf_intr;
    std::vector<uint8_t> kf_has_cam;
    std::vector<int64_t> kf_feat_ptr;
    pinned_vector<double> feat_uv;
    pinned_vector<uint64_t> feat_lm_id;
    pinned_vector<uint8_t> feat_flags;
    pinned_vector<uint64_t> lm_id;
    pinned_vector<double> lm_pos;
    pinned_vector<uint8_t> lm_bad;
    pinned_vector<int64_t> lm_obs_ptr;
    pinned_vector<uint64_t> obs_kf_id, obs_feat_idx;
    std::vector<Frame::Ptr> frames;        // keyframes in kf_id order
    std::vector<Landmark::Ptr> landmarks;  // parallel to lm_id: first-reference order in the window, NOT ascending ids
    vx_map_view view();                    // pointers into the vectors above
    // (Flatten's working arrays, kept with their capacity between calls)
    std::vector<uint8_t> scratch_has;
    std::vector<uint64_t> scratch_ids, scratch_tmp;
    std::vector<Landmark*> scratch_obj;
    std::vector<int64_t> scratch_cnt;
    std::vector<uint64_t> scratch_key, scratch_hash;
    std::vector<uint32_t> scratch_first, scratch_bucket;
    std::vector<uint8_t> scratch_firstocc;
    std::vector<int64_t> scratch_kreg;  // per (keyframe, hash region): feature counts, then bucket offsets
};

class DeviceMap;

class LocalBA {
public:
    struct Options {
        int window_size = 5;
        int max_iterations = 5;
        int min_pose_observations = 20;
        int min_point_observations = 2;
        double huber_delta = 5.0;
        double max_reproj_error = 5.0;
    };
    explicit LocalBA(const Options& options) : options_(options) {}
    void Optimize(const Map::Ptr& map, const Frame::Ptr& ref_kf);
    // Resident mode: with a DeviceMap attached (one that mirrors `map`, device_map.h), Optimize is one
    // vx_ba_optimize_dmap call on the resident map — no Flatten, no snapshot upload — and then
    // writes the window poses and optimised positions back into the Frame / Landmark objects
    // (Frame::SetPose / Landmark::SetPosition, local_ba.cpp:173,237).  nullptr: the snapshot path.
    // (turns on vx_dmap_prefetch_results: the results come back with Optimize's one synchronisation)
    void UseDeviceMap(std::shared_ptr<DeviceMap> dm);

    // The keyframes SelectKeyFrames picks (local_ba.cpp:42-62), every landmark their features
    // reference, and those landmarks' full observation maps.
    static FlatMap Flatten(const Map& map, const Frame::Ptr& ref_kf, int window_size);
    // the same into `out`, reusing its capacity (what Optimize's snapshot path does call after call)
    static void Flatten(const Map& map, const Frame::Ptr& ref_kf, int window_size, FlatMap& out);
    const vx_ba_stats& LastStats() const { return stats_; }

private:
    vx_ba_options VxOptions() const;
    void OptimizeResident(const Frame::Ptr& ref_kf);
    Options options_;
    vx_ba_stats stats_{};
    std::shared_ptr<DeviceMap> dmap_;
    std::vector<int64_t> kf_rows_, lm_rows_;
    std::vector<int32_t> kr32_, lr32_;  // (the copying fallback's rows, as the view's)
    std::vector<double> kf_out_, lm_out_;
    FlatMap flat_;  // the snapshot path's window, reused call after call
};

namespace vxhost {
vx_ctx* ThreadContext();  // the calling thread's context (device $VX_DEVICE, default 0)
}

}  // namespace visionx
