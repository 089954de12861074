// dmap.hpp — the device-resident map (vx_dmap, include/vx_slam.h), shared
// by its update API (dmap.hip), the plan build from it (ba_window.hip, build_plan_dmap) and the
// scatter of a run back into it (ba.hip, vx_ba_plan_apply_dmap).
#pragma once
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "vx_internal.hpp"

struct vx_dmap {
    vx_ctx* c = nullptr;
    // host mirrors of the small per-keyframe tables (SelectKeyFrames and the window's feature
    // ranges are host work over keyframe ids only), the id -> index maps, and the feature flags
    // (for the per-keyframe count of has_landmark features that sizes the pose-stage split)
    std::vector<uint64_t> kf_id;
    std::vector<int64_t> kf_feat_ptr{0};
    std::vector<uint8_t> kf_has_cam;
    std::vector<int> kf_valid_cnt;
    std::vector<uint8_t> feat_flags;
    std::unordered_map<uint64_t, int> kf_index, lm_index;
    int64_t n_lm = 0, n_obs = 0;
    // device arrays, insertion order, grown by doubling (used sizes from the counts above)
    vx::DevBuf kf_pose, kf_intr;                 // 7 / 4 doubles per keyframe
    vx::DevBuf feat_uv, feat_lm, feat_fl;        // 2 doubles / u64 / u8 per feature
    vx::DevBuf lm_id, lm_pos, lm_bad;            // u64 / 3 doubles / u8 per landmark
    vx::DevBuf obs_lm, obs_kf, obs_fi;           // i32 landmark index / u64 / u64 per observation
    // landmark-major observation CSR (a stable sort of the observation list by landmark index),
    // rebuilt lazily when landmarks or observations were added since the last plan build
    bool csr_dirty = true;
    vx::DevBuf optr, okf, ofi, sort_keys, sort_keys2, sort_vals, sort_vals2, tmp, cnt;
};

namespace vx {
// stable landmark-major CSR of the observation list into m->optr / okf / ofi
int dmap_build_csr(vx_ctx* c, vx_dmap* m);
}  // namespace vx
