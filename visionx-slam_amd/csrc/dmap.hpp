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
    std::vector<uint8_t> kf_alive;               // 0 after Map::RemoveKeyFrame (row kept as dead storage)
    std::vector<int> kf_valid_cnt;
    std::vector<uint8_t> feat_flags;
    std::unordered_map<uint64_t, int> kf_index, lm_index;  // live keyframes / landmarks only
    // (landmark row, keyframe id) -> observation id of the live pair: Landmark::observations_ is
    // keyed by keyframe id, so AddObservation of a present pair overwrites it in place and
    // RemoveObservation tombstones it (obs_lm = kDeadObs: skipped by the CSR rebuild).  Ids are
    // issued in insertion order and never change; the device table id_row maps each to its current
    // row, so compacting the rows (on the device) leaves this map alone.  A removed landmark's
    // pairs stay here (they can no longer be named) until purged with the rest of its kind.
    struct PairHash {
        size_t operator()(const std::pair<int, uint64_t>& k) const {
            uint64_t x = k.second * 0x9e3779b97f4a7c15ull ^ ((uint64_t)(uint32_t)k.first << 1);
            return (size_t)(x ^ (x >> 29));
        }
    };
    std::unordered_map<std::pair<int, uint64_t>, int64_t, PairHash> obs_index;
    int64_t n_lm = 0, n_obs = 0;                 // rows (removed ones included)
    // observation ids issued.  id_row (8 B per id) grows with every observation ever added:
    // compaction shrinks the rows, not the ids (re-issuing them would rewrite obs_index on the host
    // at every compaction).  10^7 observations added over a map's life = 80 MB of HBM, ~0.03 % of
    // the 288 GB; a session that must bound it recreates the vx_dmap (documented growth).
    int64_t n_ids = 0;
    int64_t n_kf_live = 0, n_lm_live = 0, n_obs_live = 0;
    std::vector<int> lm_obs_live;                // live observations per landmark row
    std::vector<uint8_t> lm_removed;             // 1 after Map::RemoveLandmark (row kept as dead storage)
    // device arrays, insertion order, grown by doubling (used sizes from the counts above)
    vx::DevBuf kf_pose, kf_intr;                 // 7 / 4 doubles per keyframe
    vx::DevBuf feat_uv, feat_lm, feat_fl;        // 2 doubles / u64 / u8 per feature
    vx::DevBuf lm_id, lm_pos, lm_bad;            // u64 / 3 doubles / u8 per landmark
    vx::DevBuf obs_lm, obs_kf, obs_fi;           // i32 landmark index / u64 / u64 per observation
    vx::DevBuf obs_id, id_row;                   // i64 id per row / i64 row per id (-1: compacted away)
    vx::DevBuf obs_lm2, obs_kf2, obs_fi2, obs_id2, cflag, cpos;  // compaction targets (swapped in)
    // landmark-major observation CSR (a stable sort of the observation list by landmark index),
    // rebuilt lazily when landmarks or observations were added since the last plan build
    bool csr_dirty = true;
    vx::DevBuf optr, okf, ofi, sort_keys, sort_keys2, sort_vals, sort_vals2, tmp, cnt;
    // landmark id -> row, open addressing on the device (ba_lean.hip): rows [0, ht_rows) inserted,
    // kept across calls (a removed landmark's row stays, its lm_bad says so); rebuilt when it grows
    vx::DevBuf ht_key, ht_val;
    unsigned ht_cap = 0;
    int64_t ht_rows = 0;
    // the lean one-call LocalBA (vx_ba_optimize_dmap): its device buffers, sized by capacity and
    // reused call after call, and the window of its last call (for vx_ba_dmap_results)
    struct Lean {
        vx::DevBuf win, f_l, f_code, f_pv, f_back, pscan, wuv, l_ref, l_pv, l_cnt, key, ex, l_slot, inv, cnt, mask,
            lobs_ptr, lm_pos0, lm_pos, puv, plm, lkf, llm, luv, lm_blk, kf_pose0, kf_pose, kf_intr, kf_rot, kf_flags,
            kf_obs_ptr, kf_part, kf_cost, state, dyn, tmp, pkf;
        vx::DevBuf pack;                   // the call's read-back packed by k_lb_apply: header | results
        vx::PinnedBuf win_host, rb_host, res_host;  // (res_host: vx_ba_dmap_results staging)
        size_t res_off = 0;                // (prefetched results: their offset in res_host)
        int nk = 0;                        // window of the last call (0: none)
        int status = 1, n_opt = 0, iterations = 0;
        std::vector<int> win_rows;         // its keyframe rows
        bool ran = false;
        vx_ba_plan* fallback = nullptr;    // the last call's plan when it took the general build
        bool prefetch = false;             // vx_dmap_prefetch_results
        bool prefetched = false;           // res_host holds the last call's results (lean build)
        int64_t pf_nl = 0;                 // (their landmark capacity)
    } lean;
    // scratch of the Schur plan build from this map (vx_sba_plan_create_dmap)
    struct SbaScratch {
        vx::DevBuf pkey, skey, perm, k2, v2, scnt, pc, pptr, kcnt, oflag, orank, bidx, ekey, eval, ekey2, tmp;
        vx::PinnedBuf rb;
    } sba;
    ~vx_dmap();
};

namespace vx {
// obs_lm of a removed observation: sorts after every live landmark row under the CSR's radix bits
constexpr int kDeadObs = 0x7fffffff;
// lm_bad value of a removed landmark (Map::RemoveLandmark): the plan build's landmark table skips it
constexpr uint8_t kLmRemoved = 2;
// stable landmark-major CSR of the observation list into m->optr / okf / ofi (compacting the
// observation rows first when dead ones — removed pairs, removed landmarks' pairs — exceed a quarter)
int dmap_build_csr(vx_ctx* c, vx_dmap* m);
}  // namespace vx
