// sba_plan.hpp — the Schur-complement BA plan (vx_sba_plan) shared by its host build (sba.hip,
// build_sba_plan, from a vx_map_view snapshot) and its device build from the resident map
// (ba_lean.hip, vx_sba_plan_create_dmap).
#pragma once
#include <cstdint>
#include <vector>

#include "vx_internal.hpp"

struct vx_sba_plan {
    vx_ctx* c = nullptr;
    vx_sba_options opt{};

    int status = 1;
    int shard_rank = 0, shard_count = 1;
    int n_window_kf = 0, n_landmarks_global = 0;
    int nk = 0, n_opt = 0, n_lm = 0, n_oo = 0, n_obs = 0;
    int64_t n_pairs = 0;
    int n_blocks = 0, n_lm_blocks = 0, n_comp = 0, max_np = 0;
    int max_panel = 1;  // most panel tiles (rhs row included) of one column of any component's factor
    int max_nt = 0;          // most 16 x 16 tile columns of one component
    int max_trail_rest = 0;  // most trailing-update tiles of one step outside its look-ahead column
    long long s_total = 0, l_total = 0;
    std::vector<int> kf_map_idx, lm_map_idx;
    std::vector<int> comp_kf_ptr_h, comp_kf_h, comp_np_h;
    std::vector<long long> comp_off_h, comp_loff_h;
    int64_t n_lfactor_tiles = 0, n_trail_updates = 0;  // symbolic factorisation (all components)
    int64_t n_trail_rhs = 0;  // (of the updates: those of the rhs row)
    vx::OwnedGraph graph;  // the run's launch sequence, replayed by hipGraphLaunch
    vx::DevBuf pose0, pose, intr, kf_flags, kf_comp, kf_local, lm0, lm, obs_uv, obs_kf, obs_lm, lm_ptr, lm_blk,
        kf_ptr, kf_obs, blk_ij, blk_ptr, pairs, comp_kf_ptr, comp_kf, comp_off, comp_loff, comp_np, comp_hdr, tl, wy,
        lm_sys,
        red, red_sum, L, Linv, dx, state;
    bool ran = false;
    bool from_dmap = false;
    vx::DevBuf lm_map_dev, kf_map_dev;  // dmap plans: slot -> resident landmark row, window row -> keyframe row
    // the multi-workgroup factor's launch k per component: 8 ints {L offset lo, hi, look-ahead tiles
    // [la_beg, split), rest [split, t_end), panel of column k + 1 [p0, p1), nt} (nt = 0: no step k)
    std::vector<int> fac_steps_h;
    vx::DevBuf fac_steps;
    // the two-column schedule (launch t factors columns 2t + 2 and 2t + 3): 16 ints per component and
    // launch {L offset lo, hi, phase-1 list [b, e), phase-2 list [b, e), rest [b, e), panel of c0
    // [b, e), panel of c1 [b, e), nt, c0, 0}; max_pairs launches
    std::vector<int> fac_pairs_h;
    vx::DevBuf fac_pairs;
    int max_pairs = 0;
    // the blocked factor (k_sba_fac_blk; launch t factors block t of up to 4 tile columns): 16 ints
    // per component and launch (FacBlk); max_blks launches; blk_ok: every column fits the block LDS;
    // max_blk_trail: most trailing tiles of one launch
    std::vector<int> fac_blks_h;
    vx::DevBuf fac_blks;
    int max_blks = 0, max_blk_trail = 0, max_blk_la = 0;  // (max_blk_la: most look-ahead tiles of one launch)
    bool blk_ok = false;
    int max_back = 0;  // most back-substitution tiles of one component (k_sba_backsub stages the lists in LDS)
    int diag_split = 1;  // k_sba_blocks workgroups per diagonal block (sba_plan_finish)
    vx::DevBuf bpart;    // their partial sums
    vx::PinnedBuf stage;  // host staging of the finish's table uploads (sba_plan_finish) ...
    vx::DevBuf stage_dev;  // ... and its device copy, scattered into the tables by one launch
};


namespace vx {
constexpr int kSbaLmThreads = 256;  // k_sba_lm: max observations (and landmarks) per workgroup
// The tail every SBA plan build ends with: p->nk / n_opt / n_oo / n_lm / n_blocks / n_pairs and the
// observation, landmark, pair and block tables on the device; flags (bit0 camera, bit1 fixed) and
// the block list (i, j) on the host.  Covisibility components, the symbolic tile factorisation, their
// uploads and the run buffers.
int sba_plan_finish(vx_ctx* c, vx_sba_plan* p, const std::vector<int>& flags, const std::vector<int2>& bij,
                    const PlanClock* clk = nullptr);
}  // namespace vx
