// vx_internal.hpp — context, device buffers, error plumbing and stage profiling shared by the
// ORB, matching and bundle-adjustment translation units of libvxslam.so.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <vector>

#include "vx_slam.h"

#ifndef VX_NO_RCCL
#include <rccl/rccl.h>
#endif

namespace vx {

// $VX_PLAN_TIMING: host timestamps of a plan build's stages on stderr (ms since the build began)
struct PlanClock {
    bool on = std::getenv("VX_PLAN_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void mark(const char* what) const {
        if (on)
            std::fprintf(stderr, "[vx plan] %-28s %.3f ms\n", what,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};

constexpr int kMaxLevels = 12;

// Profiling stages (vx_prof_*).
enum Stage : int {
    kStGray = 0,
    kStResize,
    kStFast,
    kStSelect,
    kStBlur,          // (unused: the blur is computed inside k_fast)
    kStDescribe,
    kStMatchPartial,
    kStMatchMerge,
    kStBaReset,
    kStBaPose,
    kStBaPoseSum,
    kStBaAllreduce,
    kStBaSolve,
    kStBaLandmark,
    kStPyramid,
    kStSbaLandmark,
    kStSbaBlocks,
    kStSbaSolve,
    kStSbaUpdate,
    kStSbaAllreduce,
    kStLmDepth,
    kStLmTriangulate,
    kStLmCompact,
    kStPnpHyp,
    kStPnpRefine,
    kStEmHyp,
    kStEmSelect,
    kStBaIter,        // fused LocalBA iteration (k_ba_iter)
    kStBaPrologue,    // iteration 0's pose stage of the fused path
    kStBaWin,         // the whole LocalBA window in one persistent launch (k_ba_win)
    kStCount
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    // grow-only; returns hipSuccess or the allocation error
    hipError_t ensure(size_t want) {
        if (want <= bytes) return hipSuccess;
        release();
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct PinnedBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    // cached = true: host-cached (non-coherent) pages for a staging block the CPU fills with many
    // scattered writes; the default (coherent) pages are uncached on the host side
    hipError_t ensure(size_t want, bool cached = false) {
        if (want <= bytes) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipHostMalloc(&p, want, cached ? hipHostMallocNonCoherent : hipHostMallocDefault);
        if (e == hipSuccess) bytes = want;
        return e;
    }
};

// Host-computed geometry of one ORB configuration (image size + params).  Mirrors the layer
// layout of ORB_Impl::detectAndCompute (levels stored unpadded, back to back).
struct OrbGeometry {
    int W = 0, H = 0;
    vx_orb_params p{};
    int L = 0;
    int lw[kMaxLevels], lh[kMaxLevels];
    int64_t off[kMaxLevels];        // byte offset of level l in the pyramid buffer
    float scale[kMaxLevels], inv_scale[kMaxLevels];
    int quota[kMaxLevels];
    int64_t pyr_bytes = 0;
    // resize tables for levels 1..L-1: int4 {ofs, c0, c1, 0} per destination column / row
    int64_t xtab[kMaxLevels], ytab[kMaxLevels];
    int64_t tab_entries = 0;
    // fused pyramid (k_pyramid): level-0 tiles, per (tile column | tile row, level) int4
    // {need_lo, need_hi, own_lo, own_hi} at tabs[pr_x] / tabs[pr_y], LDS bytes per ping-pong buffer
    bool pyr_fused = false;
    int pr_ntx = 0, pr_nty = 0;
    int pr_tile = 64, pr_block = 1024;
    int64_t pr_x = 0, pr_y = 0;
    int pr_buf = 0;
    int pr_area0 = 0;               // max level-0 need area (pixels)
    int pr_w0 = 0, pr_h0 = 0;       // max level-0 need width / height
    int pr_tabn = 0;                // max packed coefficient entries per tile
    int n_cu = 256;                 // compute units of the device (batched pyramid choice)
    // FAST tiles (64 x 16 pixels per workgroup) and output cells (row x tile column)
    int ntx[kMaxLevels], nty[kMaxLevels];
    int tile_base[kMaxLevels];     // first tile (workgroup) of level l
    int total_tiles = 0;
    int64_t cell_base[kMaxLevels]; // first cell of level l
    int64_t cells_total = 0;
    int level_cap[kMaxLevels];     // max strict-NMS corners of level l
    int64_t stage_base[kMaxLevels];// selection staging (4 * level_cap + 4 records) of level l
    int64_t stage_total = 0;
    int max_w = 0;
    int out_cap = 0;               // keypoint capacity of one slot
};

struct Slot {
    DevBuf kp, desc, count;  // vx_keypoint[cap], uint8[cap*32], int32[4] {n, overflow, ..}
    int cap = 0;
    bool valid = false;
};

struct ProfEvent {
    hipEvent_t a, b;
    int stage;
};

// Launch sequences of the async entry points captured into hipGraphs and replayed with one
// hipGraphLaunch (the per-frame pipeline is otherwise bound by host-side launch cost: ~18 kernel
// launches per frame).  Keyed by everything the captured sequence bakes in (device pointers,
// sizes, a geometry / plan serial); least-recently-used entries are evicted.
struct GraphCache {
    struct Entry {
        std::vector<uint64_t> key;
        hipGraphExec_t exec = nullptr;
        uint64_t last = 0;
    };
    std::vector<Entry> entries;
    uint64_t tick = 0;
    int captured = 0, launched = 0;
};

}  // namespace vx

struct vx_ba_plan;

struct vx_event {
    int device = 0;
    hipEvent_t ev = nullptr;
};

struct vx_ctx {
    int device = 0;
    int n_cus = 0;  // compute units of the device (lazily queried)
    float grid_share = 1.0f;  // vx_set_grid_share: CUs the single-round grids (k_pyramid) size for
    hipStream_t stream = nullptr;
    hipEvent_t order_event = nullptr;  // vx_stream_wait_ctx: recorded on this stream
    std::string err;

    // ---- ORB
    vx::OrbGeometry geo;
    bool geo_valid = false;
    int kp_order = VX_ORDER_STL;  // vx_orb_set_order: keypoint order inside a level
    int orb_debug = 0;            // vx_orb_set_debug flags (test hooks)
    int scratch_slot = -1;        // slot whose single-frame extraction last wrote the shared ORB scratch
                                  // (pyramid, blur, candidates, stages); -1 after a batch
    vx::DevBuf orb_dbg;           // their device record (k_select_stl)
    vx::DevBuf img_in, pyr, blur, tabs, cand, band_count, hist, stage, level_count;
    vx::Slot slots[VX_MAX_SLOTS];
    vx::Slot batch[VX_BATCH_BANKS];  // vx_orb_extract_batch_async outputs, frame-major
    int batch_n[VX_BATCH_BANKS] = {0};

    // ---- matching
    vx::DevBuf mq, mt, mq_n, partial, matches, match_count;
    vx::PinnedBuf host_stage;
    int match_cap = 0;
    bool match_valid = false;
    vx::DevBuf mb_best, mb_matches, mb_count;  // vx_match_batch_async: per-pair results
    vx::DevBuf mb_in;                           // vx_match_knn2_ratio_batch: uploaded rows + counts
    vx::PinnedBuf mb_host;
    int mb_valid = 0, mb_cap = 0;

    // ---- landmark creation (landmarks.hip): inputs, per-item flags / points, compacted outputs
    vx::DevBuf lm_in0, lm_in1, lm_in2, lm_in3, lm_in4, lm_depth, lm_valid, lm_pw, lm_index, lm_out, lm_count, lm_aux;

    // ---- PnP RANSAC (ransac.hip): packed inputs (pinned staging + device), hypothesis records,
    // packed outputs (results + inlier mask)
    vx::PinnedBuf rs_host, rs_host_out;
    vx::DevBuf rs_in, rs_hyp, rs_out;  // (shared by vx_essential_ransac, essential.hip)

    // ---- device-side LocalBA plan build scratch (ba_window.hip)
    struct PlanScratch {
        vx::DevBuf wptr, wlm, wfl, cam, wid, wuv, lid, bad, optr, okf, ofi, pos, hkey, hval, f_lm, f_pv, f_first,
            l_ref, l_opt, l_slot, l_first, counts, scan_a, scan_b, scan_c, inv, cnt, tmp;
        vx::DevBuf fb, fb_groups, fb_tmp;  // device build of the fused layout (ba_fused_build.hip)
        vx::PinnedBuf fb_host;             // its two small read-backs
        vx::PinnedBuf rb_host, up_host;    // build_core's read-back and its table uploads
        vx::PinnedBuf win_host;            // the resident-map build's window tables, one upload ...
        vx::DevBuf win;                    // ... into one device block
    } plan_scratch;
    vx_dmap* snap_map = nullptr;  // vx_ba_optimize_map's scratch map: the view loaded for the lean build (ba_lean.hip)
    // LocalBA plans of this context: parked buffer sets of destroyed plans (adopted by the next
    // vx_ba_plan_create) and the live plans (detached when the context goes first)
    std::vector<vx_ba_plan*> plan_husks, plan_live;

    // ---- hipGraph replay of the async entry points ($VX_GRAPHS=0 disables)
    vx::GraphCache graphs;
    bool use_graphs = true;
    uint64_t geo_gen = 0;  // bumped whenever the ORB geometry (and its buffers) is rebuilt

    // ---- profiling
    bool prof = false;
    unsigned prof_mask = 0;
    std::vector<vx::ProfEvent> pending;
    std::vector<hipEvent_t> event_pool;
    double prof_ms[vx::kStCount] = {0};
    int64_t prof_n[vx::kStCount] = {0};

    // ---- multi-GPU
#ifndef VX_NO_RCCL
    ncclComm_t comm = nullptr;
#endif
    int nranks = 1, rank = 0;
};

namespace vx {

int set_error(vx_ctx* c, int code, const char* fmt, ...);
// frees the parked plan buffers and detaches the live plans of c (vx_destroy; ba.hip)
void plan_pool_release(vx_ctx* c);
int hip_fail(vx_ctx* c, hipError_t e, const char* what);

// Event bracket around launches of one stage (no-op when profiling is off).
struct ProfScope {
    vx_ctx* c;
    int stage;
    hipStream_t s;
    hipEvent_t a = nullptr;
    ProfScope(vx_ctx* c_, int st, hipStream_t on = nullptr);  // default: the context stream
    ~ProfScope();
};
void prof_collect(vx_ctx* c);

// Per-dispatch timing for a single-kernel stage: the events handed to hipExtLaunchKernelGGL carry
// the dispatch's own start / end timestamps (the duration rocprofv3 reports), not a bracket that
// also spans the stream's dispatch boundaries.  Both null when the stage is not being profiled.
struct KTiming {
    hipEvent_t a = nullptr, b = nullptr;
};
KTiming prof_kernel_events(vx_ctx* c, int stage);
void prof_kernel_done(vx_ctx* c, int stage, KTiming t);

template <class F, class... Args>
inline hipError_t launch(vx_ctx* c, int stage, F kernel, dim3 grid, dim3 block, uint32_t shm, hipStream_t s,
                         Args... args) {
    const KTiming t = prof_kernel_events(c, stage);
    if (t.a) {
        hipExtLaunchKernelGGL(kernel, grid, block, shm, s, t.a, t.b, 0, args...);
        prof_kernel_done(c, stage, t);
    } else {
        hipLaunchKernelGGL(kernel, grid, block, shm, s, args...);
    }
    return hipGetLastError();
}

int orb_prepare(vx_ctx* c, const vx_orb_params* p, int w, int h);

// Runs `enqueue` (which only enqueues work on c->stream) through the context's graph cache: the
// first call with a key runs eagerly (so every buffer it needs gets allocated outside a capture),
// the second captures the sequence into a hipGraph, later ones replay it.  Profiling (events
// around launches) and the intra-frame fork bypass the cache.
int graph_run(vx_ctx* c, const std::vector<uint64_t>& key, int (*enqueue)(vx_ctx*, void*), void* arg);
// A graph owned by a long-lived object (a BA plan): captured on its second run, replayed after,
// destroyed with its owner (independently of the context's cache).
struct OwnedGraph {
    hipGraphExec_t exec = nullptr;
    bool seen = false;
    OwnedGraph() = default;
    OwnedGraph(const OwnedGraph&) = delete;
    OwnedGraph& operator=(const OwnedGraph&) = delete;
    ~OwnedGraph();
    void reset();  // forget the captured sequence (the next run is eager, then captured again)
};
int graph_run_owned(vx_ctx* c, OwnedGraph& g, int (*enqueue)(vx_ctx*, void*), void* arg);

// A kernel's >64 KB dynamic-LDS attribute, set once per DEVICE (hipFuncSetAttribute applies to the
// current device only; a function-local static would set it on whichever device came first).
// `done` is a per-call-site bit set of the devices already configured.
inline hipError_t lds_attr_once(int device, const void* fn, int bytes, std::atomic<uint64_t>& done) {
    const uint64_t bit = (device >= 0 && device < 64) ? (1ull << device) : 0;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess && bit) done.fetch_or(bit, std::memory_order_release);
    return e;
}

}  // namespace vx

#define VX_HIP(ctx, call)                                       \
    do {                                                        \
        hipError_t e__ = (call);                                \
        if (e__ != hipSuccess) return vx::hip_fail(ctx, e__, #call); \
    } while (0)

#define VX_LAUNCH_CHECK(ctx, what)                              \
    do {                                                        \
        hipError_t e__ = hipGetLastError();                     \
        if (e__ != hipSuccess) return vx::hip_fail(ctx, e__, what); \
    } while (0)
