// ba_plan.hpp — the LocalBA plan (vx_ba_plan) shared by its two builders: the host reference
// build (ba.hip, build_plan) and the device build (ba_window.hip, build_plan_device).
#pragma once
#include <cstdint>
#include <vector>

#include "vx_internal.hpp"

// byte offsets of the fused layout's index tables inside one device block (ba.hip build_fused)
struct FusedOffsets {
    size_t blk = 0, lm_slot = 0, lm_run = 0, lobs_rec = 0, kent = 0, lobs_src = 0, pobs_src = 0, pobs_code = 0;
};

struct vx_ba_plan {
    vx_ctx* c = nullptr;
    vx_ba_options opt{};
    int status = 1;
    int shard_rank = 0, shard_count = 1;
    int n_window_kf = 0, n_landmarks_global = 0;
    int n_kf = 0, n_opt = 0, n_lm = 0;
    int64_t n_pose_obs = 0, n_lm_obs = 0;
    std::vector<int> kf_map_idx, lm_map_idx;
    int n_split = 1;
    vx::DevBuf kf_pose0, kf_pose, kf_intr, kf_rot, kf_flags, kf_obs_ptr, kf_part, kf_cost, lm_pos0, lm_pos,
        pobs_uv, pobs_lm, lobs_ptr, lobs_kf, lobs_lm, lm_blk, lobs_uv, state;
    int n_lm_blocks = 1;
    int max_lm_obs = 0;         // most landmark-stage observations of one landmark
    bool choice_made = false;   // kernel set decided (ba.hip choose_lds_poses; sharded: over all ranks)
    bool lds_poses = true;
    bool ran = false;
    vx::OwnedGraph graph;  // the run's launch sequence, replayed by hipGraphLaunch
    bool graph_eager = false;  // sharded: capturing the RCCL sequence failed once -> stay eager
    vx::DevBuf kf_map_dev, lm_map_dev;  // plans built from a vx_dmap: window row / slot -> map index
    bool from_dmap = false;
    bool global_poses = false;  // VX_PLAN_GLOBAL_POSES
    // fused path (one k_ba_iter launch per iteration, ba.hip build_fused): landmark workgroups in
    // keyframe-locality order, each with its keyframe table (kent), its landmark-stage observations
    // and the pose-stage observations of its landmarks grouped by keyframe; per-keyframe partial
    // slots (n_kf x f_maxl x 32 doubles) summed in slot order by every workgroup that needs the pose
    bool fused = false;
    bool fused_all = false;  // sharded: every rank has a fused layout (decided at the first run)
    int f_blocks = 0, f_maxl = 0, f_threads = 512;
    vx::DevBuf f_tab, f_lobs_uv, f_pobs_uv, f_pobs_p, f_part;  // f_tab: the index tables, one upload
    vx::DevBuf f_rowpart;                                         // sharded: all-reduced per-row partials
    vx::DevBuf f_lpos, f_epose;  // k_ba_iter's fused-order landmark positions and per-entry pose copies
    vx::DevBuf f_costpart;       // compact {cost, observations} of every partial slot (stop rule)
    vx::DevBuf f_arow;           // $VX_BA_ATOMIC_ROWS: 3 rotating n_kf x 32 per-row sums (float atomics)
    bool f_atomic = false;
    // persistent window (k_ba_win, one launch per run): rows / arrival counters by run parity,
    // nprod, the generation word (ba.hip WinArgs); win_off after a run whose wait ran out
    vx::DevBuf f_win;
    bool f_persist = false, win_off = false;
    size_t win_rows_off = 0, win_cnt_off = 0, win_done_off = 0, win_nprod_off = 0, win_gen_off = 0;
    int f_stop_b = 0;            // workgroup running the stop rule
    vx::PinnedBuf f_stage;                                        // their host staging block
    vx::PinnedBuf fetch_host;  // vx_ba_plan_fetch: the state, both pose parities and the positions, one copy each
    // sharded plans, $VX_BA_PEER=1: the one-shot peer reduction of the row sums in place of the
    // per-iteration ncclAllReduce (ba.hip, k_peer_publish / k_peer_gather).  peer_mem: this rank's
    // block ([2][n_kf x kStride] doubles by generation parity, then the flag); peer_base[r]: rank r's
    // block as this device sees it (IPC-mapped, or another plan's block in the one-GPU emulation)
    bool peer = false;
    void* peer_mem = nullptr;
    std::vector<void*> peer_base, peer_opened;
    unsigned long long peer_gen = 0;
    FusedOffsets f_off;                                           // byte offsets of the tables in f_tab
    size_t f_npp = 0;                                             // pose-observation positions (padded)
};

struct vx_dmap;

// every buffer of a plan: vx_ba_plan_destroy parks them in the context (vx_ctx::plan_husks) and the
// next plan of that context adopts them, so a LocalBA::Optimize per keyframe allocates and frees
// nothing once the buffers have grown to the window's size (hipFree synchronises the device)
#define VX_PLAN_BUFFERS(X)                                                                              \
    X(kf_pose0) X(kf_pose) X(kf_intr) X(kf_rot) X(kf_flags) X(kf_obs_ptr) X(kf_part) X(kf_cost) X(lm_pos0) \
    X(lm_pos) X(pobs_uv) X(pobs_lm) X(lobs_ptr) X(lobs_kf) X(lobs_lm) X(lm_blk) X(lobs_uv) X(state)       \
    X(kf_map_dev) X(lm_map_dev) X(f_tab) X(f_lobs_uv) X(f_pobs_uv) X(f_pobs_p) X(f_part) X(f_rowpart)    \
    X(f_stage) X(f_lpos) X(f_epose) X(f_costpart) X(f_arow) X(f_win) X(fetch_host)

namespace vx {
// a new plan of context c (buffers adopted from a parked plan when there is one)
vx_ba_plan* plan_new(vx_ctx* c);
#ifndef VX_BA_POSE_BLOCK  // build-time overrides for sweeps only (scripts/ba_variants.sh)
#define VX_BA_POSE_BLOCK 512
#endif
#ifndef VX_BA_MAX_SPLIT
#define VX_BA_MAX_SPLIT 4
#endif
constexpr int kBaPoseBlock = VX_BA_POSE_BLOCK;  // k_pose_kf threads per workgroup (ba.hip kPoseBlock)
constexpr int kBaLmBlock = 512;    // k_landmark_solve observations / landmarks per workgroup
constexpr int kBaMaxSplit = VX_BA_MAX_SPLIT;     // pose-stage workgroups per keyframe

// Pose-stage workgroups per keyframe: about one observation per thread.  mx is the largest window
// keyframe's landmark-feature count before sharding (a count every rank sees alike, so the
// all-reduced partial layout is the same on every rank); a shard holds ~1/shard_count of those
// observations, so sharded plans use fewer slices — which also shrinks the per-iteration
// all-reduce (n_kf x n_split x 32 doubles) up to kBaMaxSplit times.  Any n_split >= 1 is correct.
inline int ba_split(int64_t mx, int shard_count) {
    const int64_t per = (int64_t)kBaPoseBlock * (shard_count > 1 ? shard_count : 1);
    const int64_t s = (mx + per - 1) / per;
    return (int)(s < 1 ? 1 : (s > kBaMaxSplit ? kBaMaxSplit : s));
}

int alloc_run_buffers(vx_ctx* c, vx_ba_plan* p);
// the fused layout from the plan's CSRs (host copies: kf_obs_ptr n_kf + 1, pose-observation landmark
// slots, landmark-stage pointers n_opt + 1 and keyframe rows); p->fused stays false when a window
// does not fit it (sharded plans, a workgroup needing more than kBaFusedK keyframes)
int build_fused(vx_ctx* c, vx_ba_plan* p, const std::vector<int>& kf_obs_ptr, const std::vector<int>& plm,
                const std::vector<int>& lptr, const std::vector<int>& lkf);
// the same layout built on the device from the plan's device CSRs (ba_fused_build.hip): same tables,
// byte for byte (tests/test_gpu_fused_build.py), without the CSR download or host packing
int build_fused_device(vx_ctx* c, vx_ba_plan* p);
constexpr int kBaFusedK = 64;      // keyframes per fused workgroup
constexpr int kFusedMaxGroups = 8192;  // most fused workgroups of a plan (host and device builds alike)
constexpr int kBaFTSmall = 512, kBaFTLarge = 1024;  // threads per fused workgroup
constexpr int kBaFTNarrow = 256;                     // (opt-in, $VX_BA_FUSED_THREADS=256)
constexpr int kBaStride = 32;      // doubles per partial block
constexpr int kBaMaxKfLds = 448;   // most window keyframes of the LDS-pose / fused kernels
// whether the plan can take the fused layout at all (window size, options, $VX_BA_FUSED)
bool fused_eligible(const vx_ba_plan* p);
// threads per fused workgroup for n_lobs landmark-stage observations (and the packing cap)
int fused_threads(vx_ctx* c, int64_t n_lobs, int* cap);
// table offsets in f_tab for nb workgroups of ft threads and n_pp pose-observation positions; returns
// the block's bytes
size_t fused_offsets(int nb, int ft, size_t n_pp, FusedOffsets& F);
inline int fused_blk_ints(int ft) { return 4 * (1 + ft / 64 / 2); }
// after the tables are in f_tab: the observation payloads gathered into the fused order, the
// partial buffers cleared, the layout enabled
// (stop_b: the workgroup that evaluates the stop rule — the one with the lightest pose stage)
int fused_finish(vx_ctx* c, vx_ba_plan* p, int nb, int ft, int maxl, size_t n_pp, int stop_b);
// Positions of a fused workgroup's entries (k_ba_iter: position P is taken by wave P % waves, i.e.
// by SIMD P % 4): LPT over the SIMDs — entries by pose-stage rounds, most first (ties: lower index),
// each to the SIMD with the fewest rounds so far (ties: fewer entries, lower SIMD) that has fewer
// than 16 entries, at position SIMD + 4 x (its entries so far).  pos[j] for the n entries; returns
// the number of positions (highest + 1; unused positions are holes).  Both layout builders use it.
__host__ __device__ inline int fused_place_entries(const int* rounds, int n, int* pos) {
    int load[4] = {0, 0, 0, 0}, cnt[4] = {0, 0, 0, 0}, n_pos = 0;
    unsigned long long done = 0;
    for (int it = 0; it < n; ++it) {
        int j = -1;
        for (int i = 0; i < n; ++i)  // next entry: most rounds, then lowest index
            if (!((done >> i) & 1) && (j < 0 || rounds[i] > rounds[j])) j = i;
        done |= 1ull << j;
        int s = -1;
        for (int q = 0; q < 4; ++q)
            if (cnt[q] < 16 && (s < 0 || load[q] < load[s] || (load[q] == load[s] && cnt[q] < cnt[s]))) s = q;
        pos[j] = s + 4 * cnt[s];
        ++cnt[s];
        load[s] += rounds[j];
        n_pos = pos[j] + 1 > n_pos ? pos[j] + 1 : n_pos;
    }
    return n_pos;
}

// the stop-rule workgroup's key: lower = lighter pose stage (most rounds of a wave, then entries)
__host__ __device__ inline long long fused_stop_key(int max_wave_rounds, int n_ent, int b) {
    return ((long long)(max_wave_rounds * 64 + n_ent) << 32) | (unsigned)b;
}
// SelectKeyFrames + landmark set + both CSRs built on the device from the map snapshot (§8f rank 2)
int build_plan_device(vx_ctx* c, const vx_map_view* m, uint64_t ref_kf_id, int has_ref, vx_ba_plan* p);
// the same plan from a device-resident map (vx_dmap; its CSR rebuilt first if stale)
int build_plan_dmap(vx_ctx* c, vx_dmap* m, uint64_t ref_kf_id, int has_ref, vx_ba_plan* p);
// greedy k_landmark_solve workgroup packing over the landmark-stage CSR pointers: {first landmark,
// first observation} per workgroup, n_blocks + 1 pairs; *max_cnt = most observations of one landmark
std::vector<int> pack_lm_blocks(const std::vector<int>& lptr, int n_opt, int* max_cnt);

// ---- lean resident LocalBA (ba_lean.hip, vx_ba_optimize_dmap): a plan whose counts stay on the
// device.  dyn[] holds what the build finds out: optimisable landmarks (slots [0, n_opt)), table
// size n_lm, landmark-stage workgroups, status (1: nothing to optimise), pose- and landmark-stage
// observations, optimisable landmarks over all shards, most landmark-stage observations of one
// landmark, fixed landmarks.
enum : int { kDynNOpt = 0, kDynNLm, kDynBlocks, kDynStatus, kDynPoseObs, kDynLmObs, kDynGlobal, kDynMaxObs,
             kDynNFixed,
             // Schur plans from the resident map (vx_sba_plan_create_dmap): optimised-landmark
             // observations, co-observation pairs, most observations of one landmark, blocks of the
             // reduced system, k_sba_lm workgroups
             kDynSbaOo, kDynSbaPairs, kDynSbaMaxObs, kDynSbaBlocks, kDynSbaLmBlocks, kDynInts = 16 };
struct DynPlan {
    int n_kf = 0, n_split = 1, grid_blocks = 0;
    vx_ba_options opt{};
    const double* kf_pose0 = nullptr;
    double* kf_pose = nullptr;
    const double* kf_intr = nullptr;
    double* kf_rot = nullptr;
    const int* kf_flags = nullptr;
    const int* kf_obs_ptr = nullptr;
    double* kf_part = nullptr;
    double* kf_cost = nullptr;
    const double* lm_pos0 = nullptr;
    double* lm_pos = nullptr;
    const double2* pobs_uv = nullptr;
    const int* pobs_lm = nullptr;
    const int* lobs_ptr = nullptr;
    const int* lobs_kf = nullptr;
    const int* lobs_lm = nullptr;
    const int* lm_blk = nullptr;
    const double2* lobs_uv = nullptr;
    void* state = nullptr;
    const int* dyn = nullptr;
};
int ba_run_dyn(vx_ctx* c, const DynPlan& d);
size_t ba_state_bytes();
size_t ba_state_iter_offset();  // byte offset of BAState::iterations (the run's last iteration count)
// a host copy of BAState -> the stats' iterations / cost / obs
void ba_state_to_stats(const void* host_state, vx_ba_stats* s);
constexpr int kBaStrideDoubles = 32;  // (= kBaStride: doubles per pose-stage partial block)
}  // namespace vx
