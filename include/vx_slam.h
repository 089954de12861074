/*
 * vx_slam.h — C ABI of the MI355X-native (gfx950) VisionX-SLAM hot path.
 *
 * One shared library (visionx-slam_amd/lib/libvxslam.so) exports these entry points.  They
 * are plain C: pointers, sizes and status codes, no C++/torch types, no exceptions across the
 * boundary.  Every call returns VX_OK (0) or a negative VX_ERR_*; vx_last_error() gives text.
 *
 * Reference interfaces replaced (paths relative to QinZiwen/VisionX-SLAM):
 *   vx_orb_extract        <- FeatureExtractor::Extract(Frame&)   core/feature/feature_extractor.h:15
 *                            ORBExtractor::Extract               core/feature/orb_extractor.cpp:9-27
 *                            ORBExtractor(n=1000, 1.2f, 8)       core/feature/orb_extractor.h:11-13
 *   vx_orb_extract_batch* <- ORBExtractor::Extract once per camera of a multi-camera time step
 *                            (orb_extractor.cpp:9-27; BASELINE config C5's 8 streams), B frames per launch
 *   vx_match_knn2_ratio   <- FeatureMatcher::Match(last, curr, matches)
 *                                                                core/feature/feature_matcher.h:11-12
 *                            ORBMatcher::Match + Options         core/feature/orb_matcher.cpp:11-43,
 *                                                                orb_matcher.h:11-14
 *   vx_match_*batch*      <- ORBMatcher::Match once per camera pair (orb_matcher.cpp:11-43), up to
 *                            VX_MAX_MATCH_PAIRS pairs per launch
 *   vx_ba_optimize_map    <- LocalBA::Optimize(map, ref_kf)      core/backend/local_ba.h:23,
 *                                                                local_ba.cpp:66-249
 *                            LocalBA::Options                    core/backend/local_ba.h:12-19
 *   vx_depth_landmarks    <- Tracking::CreateLandmarksFromDepth  core/frontend/tracking.cpp:586-650
 *   vx_triangulate        <- Tracking::TriangulateWithLastKeyFrame + TriangulatePoint
 *                                                                core/frontend/tracking.cpp:856-945
 *   vx_pnp_ransac         <- cv::solvePnPRansac in Tracking::TrackWithPnP
 *                                                                core/frontend/tracking.cpp:414-423
 *   vx_essential_ransac   <- cv::findEssentialMat + cv::recoverPose in
 *                            Tracking::EstimatePoseByEssential   core/frontend/tracking.cpp:503-547
 *   vx_dmap_*             <- visionx::Map (map.h:13-35) kept resident on the device, updated like
 *                            Map::InsertKeyFrame / InsertLandmark / Landmark::AddObservation
 *   vx_ba_plan_create_dmap <- the gather of local_ba.cpp:42-108 from the resident map
 *   vx_sba_*              (no reference counterpart: north_star's Schur-complement dense solve)
 *
 * The host-side C++ adapters that keep the reference call surface (same class names and
 * signatures) are in visionx-slam_amd/host/; the bindings a reference maintainer adds are in
 * INTEGRATION.md.
 *
 * Threading: a vx_ctx is not thread-safe; use one per calling thread (the reference calls the
 * hot path from its single tracking thread, core/system/system.cpp:39-52).  Synchronous calls
 * return after results are in caller memory.  *_async calls enqueue on the context's HIP stream
 * and work on device-resident data; vx_synchronize() / the *_fetch calls complete them.
 */
#ifndef VX_SLAM_H
#define VX_SLAM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VX_OK 0
#define VX_ERR_INVALID (-1)   /* bad argument */
#define VX_ERR_HIP (-2)       /* HIP runtime failure (message in vx_last_error) */
#define VX_ERR_CAPACITY (-3)  /* caller buffer too small; *n_out holds the required count */
#define VX_ERR_COMM (-4)      /* RCCL failure */
#define VX_ERR_STATE (-5)     /* call sequence error (e.g. fetch before extract) */

#define VX_MAX_SLOTS 4        /* device-resident keypoint/descriptor slots per context */
#define VX_BATCH_BANKS 2      /* batched-extraction output banks per context */
#define VX_MAX_BATCH 64       /* frames per batched extraction call */
#define VX_MAX_MATCH_PAIRS 16 /* descriptor-set pairs per batched matching call */

typedef struct vx_ctx vx_ctx;

/* cv::KeyPoint fields the reference keeps (orb_extractor.cpp:19-24 keeps pt and response;
 * octave and angle are exported too so callers can reproduce cv::KeyPoint). */
typedef struct {
    float x, y;        /* level-0 pixel coordinates */
    float response;    /* Harris response (HARRIS_SCORE) */
    float angle;       /* degrees [0, 360), intensity centroid */
    int32_t octave;    /* pyramid level */
} vx_keypoint;

/* cv::DMatch with imgIdx = 0 */
typedef struct {
    int32_t query_idx, train_idx;
    float distance;
} vx_match;

/* cv::ORB::create(n_features, scale_factor, n_levels) with OpenCV's remaining defaults
 * (edgeThreshold 31, firstLevel 0, WTA_K 2, HARRIS_SCORE, patchSize 31, fastThreshold 20). */
typedef struct {
    int32_t n_features;      /* 1000 (orb_extractor.h:11) */
    float scale_factor;      /* 1.2f */
    int32_t n_levels;        /* 8   */
    int32_t fast_threshold;  /* 20  */
    int32_t edge_threshold;  /* 31  */
} vx_orb_params;

/* ---------------------------------------------------------------- context */
int vx_version(void);
int vx_create(int device, vx_ctx** out);
/* vx_create with a stream priority (0 normal, 1 the device's greatest) and an optional CU mask
 * (bit i = compute unit i may run this context's workgroups; mask_words 32-bit words, NULL / 0 =
 * every CU).  Disjoint masks keep a latency-critical chain (the LocalBA context of a pipeline)
 * from queueing behind concurrently running bulk work (extraction) — see bench.py --ba-cus. */
int vx_create_ex(int device, int priority, const uint32_t* cu_mask, int mask_words, vx_ctx** out);
/* compute units of a device (the width of a CU mask) */
int vx_device_cus(int device);
void vx_destroy(vx_ctx* ctx);
/* Page-locked, host-cached memory (hipHostMalloc): a vx_map_view whose arrays live in it is uploaded
 * by DMA straight from the caller's arrays (pageable arrays are staged through the runtime's
 * bounce buffers first).  visionx::FlatMap keeps its large arrays in it.  NULL on failure. */
void* vx_host_alloc(size_t bytes);
void vx_host_free(void* p);
const char* vx_last_error(const vx_ctx* ctx);
void* vx_stream(vx_ctx* ctx);          /* the context's hipStream_t */
int vx_synchronize(vx_ctx* ctx);
/* Device-side ordering between two contexts of the same device: work enqueued on `ctx` after
 * this call starts only after everything enqueued on `after` so far has finished (event record on
 * after's stream + stream wait; the host does not block).  This is how a backend context (the
 * LocalBA of keyframe t, which needs tracking(t)) overlaps the frontend context's Extract/Match
 * of frame t+1 — the concurrency ORB-SLAM-style systems get from a separate mapping thread. */
int vx_stream_wait_ctx(vx_ctx* ctx, vx_ctx* after);
/* Device events for finer cross-context ordering (a pipeline that must wait for one specific
 * earlier step of another context, not for everything enqueued on it so far). */
typedef struct vx_event vx_event;
int vx_event_create(vx_ctx* ctx, vx_event** out);
int vx_event_record(vx_ctx* ctx, vx_event* ev); /* marks everything enqueued on ctx so far */
int vx_event_wait(vx_ctx* ctx, vx_event* ev);   /* later work on ctx waits for the marked work */
void vx_event_destroy(vx_event* ev);
/* hipGraph replay: the *_async entry points (and vx_ba_plan_run_async / vx_sba_plan_run_async) run
 * eagerly the first time a launch configuration is seen, capture it into a hipGraph the second
 * time and replay it with one hipGraphLaunch afterwards ($VX_GRAPHS=0 or enable = 0 disables;
 * profiling bypasses it).  Counts of captured graphs and graph launches so far. */
int vx_graph_enable(vx_ctx* ctx, int enable);
int vx_graph_counts(const vx_ctx* ctx, int* captured, int* launched);
/* Fraction (0, 1] of the device's compute units this context's one-round grids (the fused
 * pyramid of vx_orb_extract*) are sized for (default 1).  A frontend context whose extraction
 * runs beside other contexts' work (the LocalBA of the previous keyframe) gets a smaller grid
 * that leaves CUs free: 1/4 in the 3-context pipeline of bench.py.  Results are
 * identical for every share; the call drops the context's captured graphs. */
int vx_set_grid_share(vx_ctx* ctx, float share);
void vx_orb_default_params(vx_orb_params* p);
/* Copies the compiled-in rBRIEF pattern (bit_pattern_31_, 256 x {x1,y1,x2,y2}). */
int vx_orb_pattern(int32_t* out_1024);

/* ---------------------------------------------------------------- ORB extraction
 * img: 8UC1 gray or 8UC3/8UC4 BGR(A) rows of row_stride bytes.  Keypoints are emitted level by
 * level (octave ascending) and, inside a level, in the order OpenCV's KeyPointsFilter::retainBest
 * leaves them when built against libstdc++: std::nth_element + std::partition by FAST score, then
 * again by Harris response (VX_ORDER_STL, the default) — the order ORBExtractor::Extract numbers
 * Frame::Features() in (orb_extractor.cpp:13-24).  VX_ORDER_RASTER (opt-in, vx_orb_set_order)
 * keeps the same keypoint set per level in raster order.  out_desc gets N rows of 32 bytes.
 * Returns VX_ERR_CAPACITY (with *n_out = N) if N > cap. */
#define VX_ORDER_STL 0
#define VX_ORDER_RASTER 1
/* Keypoint order of every later extraction on ctx (drops the context's captured graphs). */
int vx_orb_set_order(vx_ctx* ctx, int order);
int vx_orb_get_order(const vx_ctx* ctx);
/* Test hooks for per-stage parity; single-frame extraction into slot 0
 * (vx_orb_extract) only.  VX_ORB_DEBUG_FAST_NO_BORDER makes k_fast keep every FAST + NMS corner
 * of [3, W-3) x [3, H-3) (the list before runByImageBorder; the later stages are then NOT the
 * reference's); VX_ORB_DEBUG_STAGES records the selection's stages.  vx_orb_debug_read(level,
 * what): 0 the gray / INTER_LINEAR_EXACT level (lw*lh bytes), 1 its GaussianBlur, 2 the level's
 * candidates in raster order (16-byte records {x | y << 16, FAST score, float Harris, 0}),
 * 3 retainBest(2q)'s output order (int32 indices into the candidates), 4 retainBest(q)'s output
 * (16-byte records, the order k_describe emits).  *n_out = elements (bytes for 0/1). */
#define VX_ORB_DEBUG_FAST_NO_BORDER 1
#define VX_ORB_DEBUG_STAGES 2
int vx_orb_set_debug(vx_ctx* ctx, int flags);
int vx_orb_debug_read(vx_ctx* ctx, int level, int what, void* out, int64_t cap_bytes, int64_t* n_out);
/* Test hook: KeyPointsFilter::retainBest(keys, npts) through the device selection code (one
 * workgroup): elements u32 (key <= 255, the FAST-score path) or wide = u64 (the Harris path),
 * in LDS or in global memory; out_idx = kept key indices in output order. */
int vx_test_retain_best(vx_ctx* ctx, const uint32_t* keys, int n, int npts, int wide, int use_lds,
                        int32_t* out_idx, int* n_out);
int vx_orb_extract(vx_ctx* ctx, const vx_orb_params* params, const uint8_t* img, int width,
                   int height, int channels, int64_t row_stride, vx_keypoint* out_kp,
                   uint8_t* out_desc, int cap, int* n_out);
/* Device-resident variant: d_img is device memory; results stay in `slot`. */
int vx_orb_extract_async(vx_ctx* ctx, const vx_orb_params* params, const uint8_t* d_img,
                         int width, int height, int channels, int64_t row_stride, int slot);
int vx_orb_fetch(vx_ctx* ctx, int slot, vx_keypoint* out_kp, uint8_t* out_desc, int cap,
                 int* n_out);
/* Device pointers of a slot's descriptor rows and its device-side count, and its row capacity
 * (for interop and for vx_match_device_async from another context).  Stable until the ORB
 * geometry (image size / params) of the context changes. */
int vx_orb_slot_device(vx_ctx* ctx, int slot, const uint8_t** d_desc, const int32_t** d_count,
                       int32_t* cap);

/* Batched extraction (SURVEY.md 8(d) batched figures; the C5 multi-camera rig): n_frames images
 * of one size, frame f at d_imgs + f * frame_stride (device memory), extracted by ONE launch per
 * kernel (frame = grid z) instead of one extraction per frame — same results as vx_orb_extract
 * for every frame.  Each frame's keypoints / descriptors stay in output bank `bank` (two banks,
 * so a camera's batch t can be matched against its batch t-1) at index f: vx_orb_batch_fetch
 * copies them out, vx_orb_batch_device hands their device rows to vx_match_*_async. */
int vx_orb_extract_batch_async(vx_ctx* ctx, const vx_orb_params* params, const uint8_t* d_imgs,
                               int n_frames, int64_t frame_stride, int width, int height, int channels,
                               int64_t row_stride, int bank);
/* Host-image variant: imgs[f] are host rows of row_stride bytes (all frames one size), uploaded
 * into the context, then extracted as one batch into `bank`. */
int vx_orb_extract_batch(vx_ctx* ctx, const vx_orb_params* params, const uint8_t* const* imgs,
                         int n_frames, int width, int height, int channels, int64_t row_stride,
                         int bank);
int vx_orb_batch_fetch(vx_ctx* ctx, int bank, int frame, vx_keypoint* out_kp, uint8_t* out_desc,
                       int cap, int* n_out);
int vx_orb_batch_device(vx_ctx* ctx, int bank, int frame, const uint8_t** d_desc,
                        const int32_t** d_count, int32_t* cap);

/* ---------------------------------------------------------------- matching
 * knnMatch(query = last frame, train = current frame, k = 2) + ratio test
 * (m1.distance < ratio * m2.distance), matches in ascending query index. */
int vx_match_knn2_ratio(vx_ctx* ctx, const uint8_t* query_desc, int n_query,
                        const uint8_t* train_desc, int n_train, float ratio, vx_match* out,
                        int cap, int* n_out);
/* Device-resident variant matching two extraction slots (counts read on device). */
int vx_match_slots_async(vx_ctx* ctx, int query_slot, int train_slot, float ratio);
/* Device-resident variant over any device descriptor sets whose row counts are device-side
 * (e.g. another context's slots, vx_orb_slot_device); cap_* bound the rows.  Enqueued on ctx's
 * stream: order it after the producer with vx_event_wait / vx_stream_wait_ctx. */
int vx_match_device_async(vx_ctx* ctx, const uint8_t* d_query, const int32_t* d_n_query, int cap_query,
                          const uint8_t* d_train, const int32_t* d_n_train, int cap_train, float ratio);
int vx_match_fetch(vx_ctx* ctx, vx_match* out, int cap, int* n_out);
/* Batched matching: n_pairs (<= VX_MAX_MATCH_PAIRS) independent kNN-2 + ratio problems in one
 * launch pair (pair = grid y), query set i = d_query[i] (d_n_query[i] rows on the device, at most
 * cap_query), train set i likewise — e.g. each camera's frame t against its frame t-1 from two
 * batch banks.  The pointer arrays are host arrays of device pointers.  Results per pair:
 * vx_match_batch_fetch(ctx, i, ...), identical to vx_match_device_async on that pair alone. */
int vx_match_batch_async(vx_ctx* ctx, int n_pairs, const uint8_t* const* d_query,
                         const int32_t* const* d_n_query, int cap_query, const uint8_t* const* d_train,
                         const int32_t* const* d_n_train, int cap_train, float ratio);
/* Host-descriptor variant: pair i = query q[i] (nq[i] rows of 32 B) against train t[i] (nt[i]
 * rows), uploaded in one copy; a pair with an empty side yields 0 matches (orb_matcher.cpp:18-20). */
int vx_match_knn2_ratio_batch(vx_ctx* ctx, int n_pairs, const uint8_t* const* q, const int32_t* nq,
                              const uint8_t* const* t, const int32_t* nt, float ratio);
int vx_match_batch_fetch(vx_ctx* ctx, int pair, vx_match* out, int cap, int* n_out);

/* ---------------------------------------------------------------- local bundle adjustment
 * A flattened snapshot of visionx::Map (map.h:13-34): keyframes with their Feature vectors
 * (frame.h:16-23) and landmarks with their observation maps (landmark.h:12-68).  Keyframes may
 * be in any order (the reference's std::map sorts them by id).  kf_pose and lm_pos are updated
 * in place, exactly as Frame::SetPose / Landmark::SetPosition would be. */
typedef struct {
    int32_t n_kf;
    const uint64_t* kf_id;
    double* kf_pose;             /* 7 per KF: qx qy qz qw tx ty tz (T_cw, world -> camera) */
    const double* kf_intr;       /* 4 per KF: fx fy cx cy */
    const uint8_t* kf_has_cam;   /* Frame::GetCamera() != nullptr */
    const int64_t* kf_feat_ptr;  /* n_kf + 1, CSR into the feature arrays */
    const double* feat_uv;       /* 2 per feature */
    const uint64_t* feat_lm_id;  /* Feature::landmark_id_ */
    const uint8_t* feat_flags;   /* bit0 has_landmark, bit1 is_outlier */
    int32_t n_lm;
    const uint64_t* lm_id;       /* distinct ids in any order (not necessarily sorted: lookups hash them) */
    double* lm_pos;              /* 3 per landmark */
    const uint8_t* lm_bad;
    const int64_t* lm_obs_ptr;   /* n_lm + 1, CSR of (kf id, feature index) observations */
    const uint64_t* obs_kf_id;
    const uint64_t* obs_feat_idx;
} vx_map_view;

typedef struct {                 /* LocalBA::Options, local_ba.h:12-19 */
    int32_t window_size;         /* 5 */
    int32_t max_iterations;      /* 5 */
    int32_t min_pose_observations;   /* 20 */
    int32_t min_point_observations;  /* 2 */
    double huber_delta;          /* 5.0 */
    double max_reproj_error;     /* 5.0 */
} vx_ba_options;

typedef struct {
    int32_t iterations;          /* outer iterations executed (including the one that broke) */
    int32_t n_window_kf, n_landmarks;
    double cost[16];             /* pose-stage total_cost per iteration */
    int32_t obs[16];             /* pose-stage total_obs per iteration */
    double gate_margin;          /* unused by the GPU path (set to -1) */
    int32_t status;              /* 0 optimised, 1 early return (no KF pair / no landmark) */
} vx_ba_stats;

void vx_ba_default_options(vx_ba_options* o);
/* Reproducibility: unsharded windows sum each keyframe's normal-equation row with FP64 float
 * atomics by default (arrival order), so two runs of the same input agree to rounding (~1e-8
 * relative in the positions after five iterations; residuals move < 1e-7 px), not bit for bit.
 * Set $VX_BA_ATOMIC_ROWS=0 before the plan is built for per-workgroup partial slots summed in a fixed
 * order: bitwise-repeatable runs, ~7 % slower LocalBA.  Sharded plans always use
 * the slots. */
int vx_ba_optimize_map(vx_ctx* ctx, vx_map_view* map, uint64_t ref_kf_id, int has_ref,
                       const vx_ba_options* opt, vx_ba_stats* stats);

/* Staged form: plan = window selection + device CSR upload (host work of local_ba.cpp:66-108);
 * run = the iterations on the device from the plan's initial state (repeatable);
 * fetch = download + scatter back into `map` (may be NULL to only read stats).
 * shard_count > 1 keeps only this rank's landmark shard (landmark id hash) and all-reduces the
 * per-keyframe normal equations over the communicator set by vx_comm_init. */
typedef struct vx_ba_plan vx_ba_plan;
int vx_ba_plan_create(vx_ctx* ctx, const vx_map_view* map, uint64_t ref_kf_id, int has_ref,
                      const vx_ba_options* opt, int shard_rank, int shard_count,
                      vx_ba_plan** out);
/* flags: VX_PLAN_HOST_BUILD builds the plan with the host reference restatement of
 * local_ba.cpp:42-108 (hash maps, one core) instead of the device build (default: window join,
 * slot assignment and both CSRs as HIP kernels).  Both give the same plan. */
#define VX_PLAN_HOST_BUILD 1
/* VX_PLAN_GLOBAL_POSES runs the large-window kernels (poses solved once into global memory, one
 * thread per landmark) at any window size; by default they run only beyond 448 keyframes, where
 * the per-workgroup LDS copy of every keyframe's pose no longer fits.  Same results. */
#define VX_PLAN_GLOBAL_POSES 2
int vx_ba_plan_create_ex(vx_ctx* ctx, const vx_map_view* map, uint64_t ref_kf_id, int has_ref,
                         const vx_ba_options* opt, int shard_rank, int shard_count, int flags,
                         vx_ba_plan** out);
int vx_ba_plan_run_async(vx_ctx* ctx, vx_ba_plan* plan);
int vx_ba_plan_fetch(vx_ctx* ctx, vx_ba_plan* plan, vx_map_view* map, vx_ba_stats* stats);
void vx_ba_plan_destroy(vx_ba_plan* plan);
/* sizes of the device problem: out8 = {n_kf, n_lm (local shard), n_pose_obs, n_lm_obs, n_opt,
 * n_split (pose-stage workgroups per keyframe), n_lm_blocks (landmark-stage workgroups),
 * max_lm_obs (most landmark-stage observations of one landmark)} */
int vx_ba_plan_info(const vx_ba_plan* plan, int64_t* out8);
/* kernel layout of the plan: out4 = {1 if it has the fused one-launch-per-iteration layout
 * (k_ba_iter) else 0, threads per fused workgroup, fused workgroups, most partial slots of one
 * keyframe}.  A sharded plan runs the fused kernel only when every rank has the layout (decided by
 * one all-reduce on its first run). */
int vx_ba_plan_layout(const vx_ba_plan* plan, int64_t* out4);
/* 1 when the plan's runs are ONE persistent launch per window (k_ba_win: unsharded float-atomic
 * plans whose workgroups fit on the device at once; $VX_BA_PERSIST=0 disables it), 0 when they are
 * one launch per iteration.  A persistent run whose bounded waits ran out (its workgroups could not
 * all be resident, e.g. another persistent window held the compute units) is re-run by
 * vx_ba_plan_fetch with the per-iteration launches, which the plan keeps from then on. */
int vx_ba_plan_persistent(const vx_ba_plan* plan);
/* Test hook: the fused layout's index tables (workgroup headers, landmark slots and runs,
 * landmark-stage records, keyframe entries, landmark- and pose-stage observation sources, pose
 * codes) copied back to back into dst; *bytes = their total size (dst NULL: the size only).  The
 * device build of the layout must equal the host packing (VX_PLAN_HOST_BUILD) byte for byte. */
int vx_ba_plan_fused_tables(vx_ctx* ctx, const vx_ba_plan* plan, void* dst, size_t cap, size_t* bytes);
/* Test hook: runs the n shard plans plans[r] (shard r of n, built from one window, all on ctx) the
 * way n ranks would run them, on one device: per iteration every shard's pose stage, then the
 * element-wise sum of their partial blocks in rank order written back to every shard in place of
 * the ncclAllReduce, then every shard's landmark stage (the kernel set chosen from the maxima over
 * the shards, as the all-reduced choice of a real sharded run).  Fetch each plan afterwards. */
int vx_ba_shard_emulate_run(vx_ctx* ctx, vx_ba_plan* const* plans, int n);
/* Host-only dry run of vx_ba_plan_create (needs no device): out8 = {status, n_window_kf,
 * n_landmarks (all shards), n_kf, n_opt (local optimisable), n_lm (local table), n_pose_obs,
 * n_lm_obs}; lm_map_idx / kf_map_idx (optional) receive the local tables as map indices. */
int vx_ba_plan_inspect(const vx_map_view* map, uint64_t ref_kf_id, int has_ref,
                       const vx_ba_options* opt, int shard_rank, int shard_count, int64_t* out8,
                       int32_t* lm_map_idx, int cap_lm, int32_t* kf_map_idx, int cap_kf);
/* Landmark -> shard assignment used by sharded plans (splitmix64(id) mod shard_count). */
uint32_t vx_ba_shard_of(uint64_t lm_id, int shard_count);

/* ---------------------------------------------------------------- device-resident map
 * A persistent mirror of visionx::Map on the device: keyframes with their
 * features, landmarks, observations, updated incrementally as Tracking / the Map change them
 * (Map::InsertKeyFrame, Map::InsertLandmark, Landmark::AddObservation, Feature::landmark_id_,
 * Landmark::SetBad, Frame::SetPose), so a LocalBA plan is built from device memory — no map
 * snapshot crosses PCIe per keyframe — and its result is scattered back into the device map
 * without a host round trip.  Keyframes / landmarks keep their insertion order (the map index
 * order of an equivalent vx_map_view); a landmark's observations keep their insertion order.
 * Capacities grow on demand. */
typedef struct vx_dmap vx_dmap;
int vx_dmap_create(vx_ctx* ctx, vx_dmap** out);
void vx_dmap_destroy(vx_dmap* map);
/* Map::InsertKeyFrame: kf_id unique; pose7 T_cw; intr4 fx fy cx cy (ignored unless has_cam);
 * features as in vx_map_view (uv 2 each, landmark ids, flags bit0 has_landmark bit1 is_outlier) */
int vx_dmap_add_keyframe(vx_dmap* map, uint64_t kf_id, const double* pose7, const double* intr4, int has_cam,
                         int n_feat, const double* feat_uv, const uint64_t* feat_lm_id, const uint8_t* feat_flags);
/* Map::InsertLandmark: ids unique; pos 3 each; bad may be NULL (all good) */
int vx_dmap_add_landmarks(vx_dmap* map, int n, const uint64_t* lm_id, const double* pos3, const uint8_t* bad);
/* Landmark::AddObservation(kf_id, feat_idx) on existing landmarks (VX_ERR_INVALID for unknown ids).
 * Like observations_[keyframe_id] = feature_idx (landmark.h:32-35), a (landmark, keyframe) pair
 * already present keeps its place and takes the new feature index; a landmark never holds two
 * observations from one keyframe.  Each new pair takes an observation id for the map's life (8 B of
 * device memory per pair ever added; compaction reclaims rows, not ids). */
int vx_dmap_add_observations(vx_dmap* map, int n, const uint64_t* lm_id, const uint64_t* kf_id,
                             const uint64_t* feat_idx);
/* Landmark::RemoveObservation(kf_id) (landmark.h:37-40): the pair stops counting towards
 * ObservationCount and leaves the landmark's list; an absent pair is a no-op (unordered_map::erase).
 * VX_ERR_INVALID for an unknown landmark id. */
int vx_dmap_remove_observations(vx_dmap* map, int n, const uint64_t* lm_id, const uint64_t* kf_id);
/* Map::RemoveKeyFrame(id) (map.cpp:15-18): the keyframe leaves the map (SelectKeyFrames no longer
 * sees it; observations naming it fail the window check like GetFrame() == nullptr).  Its feature
 * rows stay as dead storage.  The id may be inserted again later.  VX_ERR_INVALID if absent.
 * Tracking::RemoveKeyFrame (tracking.cpp:752-773) = vx_dmap_remove_observations for the frame's
 * landmark features + vx_dmap_set_features (0, no landmark, outlier) + this call. */
int vx_dmap_remove_keyframe(vx_dmap* map, uint64_t kf_id);
/* Map::RemoveLandmark(id) (map.cpp:20-23): GetLandmark() == nullptr afterwards (pose stage and
 * landmark set skip it).  Absent ids are a no-op, as std::unordered_map::erase. */
int vx_dmap_remove_landmarks(vx_dmap* map, int n, const uint64_t* lm_id);
/* Feature::landmark_id_ / has_landmark / is_outlier of features of keyframe kf_id */
int vx_dmap_set_features(vx_dmap* map, uint64_t kf_id, int n, const int32_t* feat_idx, const uint64_t* lm_id,
                         const uint8_t* flags);
int vx_dmap_set_landmark_bad(vx_dmap* map, int n, const uint64_t* lm_id, const uint8_t* bad);
int vx_dmap_set_poses(vx_dmap* map, int n, const uint64_t* kf_id, const double* pose7);
/* out4 = {keyframe rows, feature rows, landmark rows, observation rows}: storage rows in insertion
 * order, removed ones included (vx_dmap_download returns that many) */
int vx_dmap_counts(const vx_dmap* map, int64_t* out4);
/* out4 = {keyframes, landmarks, observations, 0} currently in the map (removed ones excluded) */
int vx_dmap_live_counts(const vx_dmap* map, int64_t* out4);
/* current poses (7 per keyframe row) / positions (3 per landmark row) in insertion order (rows of
 * removed keyframes / landmarks included); either may be NULL */
int vx_dmap_download(vx_dmap* map, double* kf_pose, double* lm_pos);
/* LocalBA plan from the resident map (the plan vx_ba_plan_create builds from the equivalent
 * vx_map_view snapshot); run with vx_ba_plan_run_async as usual */
int vx_ba_plan_create_dmap(vx_ctx* ctx, vx_dmap* map, uint64_t ref_kf_id, int has_ref, const vx_ba_options* opt,
                           int shard_rank, int shard_count, vx_ba_plan** out);
/* enqueue the scatter of a run's window poses and optimised landmark positions into the map (stream
 * ordered after the run; no host synchronisation) */
int vx_ba_plan_apply_dmap(vx_ctx* ctx, vx_ba_plan* plan, vx_dmap* map);
/* LocalBA::Optimize(map, ref_kf) (local_ba.cpp:66-249) on the resident map in ONE call: window
 * selection over the host id mirror, then plan build, iterations and the scatter of the results into
 * the map's rows as one stream-ordered sequence over buffers sized by capacity, with the counts kept
 * on the device — the call synchronises once, at its end, to fill `stats` (ba_lean.hip).  Windows of
 * more than 255 keyframes (or $VX_LEAN=0) take the general build (vx_ba_plan_create_dmap + run +
 * apply) inside the same call.  Same status / iteration / observation counts as vx_ba_optimize_map on
 * the equivalent snapshot; poses and positions within the BA tolerance. */
int vx_ba_optimize_dmap(vx_ctx* ctx, vx_dmap* map, uint64_t ref_kf_id, int has_ref, const vx_ba_options* opt,
                        vx_ba_stats* stats);
/* What the last vx_ba_optimize_dmap changed (for a host Map mirror: Frame::SetPose /
 * Landmark::SetPosition, local_ba.cpp:173,237): *n_kf window keyframe rows (insertion order rows of
 * the map) with their poses (7 each) and *n_lm optimised landmark rows with their positions (3 each);
 * both 0 when nothing was optimised.  Any output pointer may be NULL; VX_ERR_CAPACITY if a count
 * exceeds its cap (the counts are set either way). */
int vx_ba_dmap_results(vx_ctx* ctx, vx_dmap* map, int cap_kf, int64_t* kf_rows, double* kf_pose7, int cap_lm,
                       int64_t* lm_rows, double* lm_pos3, int* n_kf, int* n_lm);
/* on != 0: every following vx_ba_optimize_dmap also copies its results (both pose buffers, the
 * optimised positions and their rows, sized by the call's capacities) into pinned host memory before
 * its one synchronisation, so vx_ba_dmap_results then only copies on the host — no device call, no
 * second synchronisation (what a drop-in that writes every result back wants; default off). */
int vx_dmap_prefetch_results(vx_dmap* map, int on);
/* The same results without a copy, with prefetching on: pointers into the pinned block the last
 * vx_ba_optimize_dmap filled, valid until the next vx_ba_optimize_dmap / vx_dmap_* call on the map —
 * *n_kf keyframe rows (int32) with their poses (8 doubles each: qx qy qz qw tx ty tz, pad), *n_lm
 * landmark rows (int32) with their positions (4 doubles each: x y z, pad); both counts 0 (pointers
 * NULL) when nothing was optimised.  VX_ERR_STATE when the results were not prefetched (prefetching
 * off, or a run that fell back to a built plan): use vx_ba_dmap_results then. */
int vx_ba_dmap_results_view(vx_ctx* ctx, vx_dmap* map, const int32_t** kf_rows, const double** kf_pose8,
                            const int32_t** lm_rows, const double** lm_pos4, int* n_kf, int* n_lm);

/* ---------------------------------------------------------------- Schur-complement joint BA
 * NOT a reference entry point: the reference's LocalBA alternates per-keyframe and per-landmark
 * steps (local_ba.cpp:116-238).  BASELINE.json's north_star (and configs C5) ask for the
 * Schur-complement reduction of the landmark blocks into the dense 6N x 6N pose system and a
 * dense pose solve; this is that solver, on the same window / landmark set / observations /
 * residual / Jacobians / Huber weight / gates as LocalBA (local_ba.cpp:15-108, projection.h:11-31),
 * as one damped Gauss-Newton (Levenberg-Marquardt) system with b = +J^T W e, the oldest
 * `fixed_keyframes` window keyframes held fixed.  Same map snapshot and plan life cycle as
 * vx_ba_plan_*; shard_count > 1 shards landmarks and all-reduces the reduced system over RCCL.
 * Parity is against its CPU restatement (oracle/sba_oracle.cpp), see DESIGN.md §10. */
typedef struct {
    int32_t window_size;             /* keyframes in the window (SelectKeyFrames) */
    int32_t max_iterations;          /* assemblies: initial + accepted + rejected steps, <= 64 */
    int32_t min_point_observations;  /* landmark filter (local_ba.cpp:100-102) */
    int32_t fixed_keyframes;         /* oldest window keyframes held fixed (gauge, 2: also the scale) */
    double huber_delta;              /* 5.0 */
    double max_reproj_error;         /* 5.0 */
    double lambda_init;              /* Marquardt damping H_ii += lambda * H_ii (1e-4) */
    double rel_tol;                  /* stop after an accepted step lowering the cost by < rel_tol */
} vx_sba_options;

typedef struct {
    int32_t iterations;          /* assemblies executed */
    int32_t accepted;            /* accepted steps */
    int32_t n_window_kf, n_landmarks;
    double cost[16];             /* Huber cost at each assembly */
    int32_t obs[16];             /* valid observations at each assembly */
    int32_t step[16];            /* 2 initial, 1 accepted, 0 rejected, 3 re-assembled after a reject */
    double lambda;               /* damping after the last iteration */
    double initial_cost, final_cost;
    int32_t status;              /* 0 optimised, 1 early return (no KF pair / no landmark) */
} vx_sba_stats;

typedef struct vx_sba_plan vx_sba_plan;
void vx_sba_default_options(vx_sba_options* o);
int vx_sba_plan_create(vx_ctx* ctx, const vx_map_view* map, uint64_t ref_kf_id, int has_ref,
                       const vx_sba_options* opt, int shard_rank, int shard_count, vx_sba_plan** out);
int vx_sba_plan_run_async(vx_ctx* ctx, vx_sba_plan* plan);
int vx_sba_plan_fetch(vx_ctx* ctx, vx_sba_plan* plan, vx_map_view* map, vx_sba_stats* stats);
void vx_sba_plan_destroy(vx_sba_plan* plan);
/* out8 = {n_kf, n_opt (local landmarks), n_obs, n_pairs, n_blocks, n (= 6 n_kf), nonzero 16x16
 * tiles of the Cholesky factors (symbolic factorisation, rhs row included), n_components} */
int vx_sba_plan_info(const vx_sba_plan* plan, int64_t* out8);
/* The dense pose solve's symbolic work (all components; the rhs row's tiles left out): out4 =
 * {nonzero tiles of L, trailing-update tile products (16x16x16 each), diagonal tiles (one POTRF
 * each), off-diagonal panel tiles (one TRSM each)} -> algorithmic FP64 flops of one factorisation
 * 2*16^3 * updates + 16^3 * panel + 16^3/3 * diagonal (bench.py's MFMA roofline for config C5). */
int vx_sba_plan_factor_work(const vx_sba_plan* plan, int64_t* out4);
/* The reduced system of the LAST assembly of the last run (S row-major n x n, lower triangle
 * meaningful, damping included; rhs n), for verification against the restatement. */
int vx_sba_plan_system(vx_ctx* ctx, vx_sba_plan* plan, double* S, double* rhs, int n);
/* The same plan from the device-resident map (vx_dmap): window, landmark set and observation set as
 * for the equivalent snapshot, the observation / pair / block tables sorted on the device (two small
 * read-backs: the counts, then the block list for the host's covisibility components and symbolic
 * factorisation).  Unsharded.  Fetch statistics with vx_sba_plan_fetch(map = NULL); the result goes
 * into the map's rows with vx_sba_plan_apply_dmap (stream ordered, no host synchronisation). */
int vx_sba_plan_create_dmap(vx_ctx* ctx, vx_dmap* map, uint64_t ref_kf_id, int has_ref, const vx_sba_options* opt,
                            vx_sba_plan** out);
/* Rebuild a plan made by vx_sba_plan_create_dmap in place for the map's current state and ref_kf_id,
 * with the plan's options: its device buffers and host staging are reused (grown when the window
 * needs more), so a drop-in that keeps one plan per backend pays no allocation or release per
 * Backend::Optimize() (the reference builds its problem per call, core/backend/local_ba.cpp:42-108).
 * The plan's captured run graph is dropped (the next run is eager).  On error the plan is left
 * unusable (status set, no run) until a successful rebuild. */
int vx_sba_plan_rebuild_dmap(vx_ctx* ctx, vx_dmap* map, uint64_t ref_kf_id, int has_ref, vx_sba_plan* plan);
int vx_sba_plan_apply_dmap(vx_ctx* ctx, vx_sba_plan* plan, vx_dmap* map);
/* Test hook, the Schur counterpart of vx_ba_shard_emulate_run: the n shard plans of one window
 * (vx_sba_plan_create with shard_rank r of n, all on ctx; every shard's block structure is the whole
 * window's) run as n ranks would on one device — per iteration every shard's landmark stage and
 * blocks, then their reduced systems summed element-wise in rank order into every shard in place of
 * the ncclAllReduce, then every shard's (identical) factorisation, back-substitution and update.
 * Fetch each plan afterwards. */
int vx_sba_shard_emulate_run(vx_ctx* ctx, vx_sba_plan* const* plans, int n);
int vx_sba_optimize_map(vx_ctx* ctx, vx_map_view* map, uint64_t ref_kf_id, int has_ref,
                        const vx_sba_options* opt, vx_sba_stats* stats);

/* ---------------------------------------------------------------- landmark creation
 * The two loops Tracking::CreateKeyFrame runs on every new keyframe right before LocalBA
 * (core/frontend/tracking.cpp:577-580).  Both return the created landmarks in input order (the
 * order landmark_id_++ numbers them): out_index[i] = rank of item i among the created ones or -1,
 * out_pw[3 * rank ..] = its world position; *n_created = count.  The caller creates the Landmark
 * objects, adds the observations and sets Feature::landmark_id_ / has_landmark / is_outlier
 * exactly as the reference loop body does. */
#define VX_DEPTH_U16 0   /* CV_16U, metres * 5000 (TUM; kDepthScale, tracking.cpp:601) */
#define VX_DEPTH_F32 1   /* CV_32F metres */
#define VX_DEPTH_F64 2   /* CV_64F metres */

/* <- Tracking::CreateLandmarksFromDepth(frame) (tracking.cpp:586-650): features without a
 * landmark, depth at (int)(x + 0.5), (int)(y + 0.5), 0.1 <= d <= 10 m, pw = T_cw^-1 * pixelToCamera.
 * feat_uv: 2 per feature (Feature::position); intr4: fx fy cx cy; pose7: T_cw (qx qy qz qw tx ty tz).
 * depth == NULL (Depth().empty()) creates nothing. */
int vx_depth_landmarks(vx_ctx* ctx, const double* feat_uv, const uint8_t* feat_has_lm, int n_feat,
                       const void* depth, int depth_type, int rows, int cols, int64_t row_stride,
                       const double* intr4, const double* pose7, int32_t* out_index, double* out_pw,
                       int* n_created);
/* <- Tracking::TriangulateWithLastKeyFrame(last, curr) + TriangulatePoint (tracking.cpp:856-945)
 * over the matches Match(last, curr) returned (query = last frame, train = current frame; query
 * indices unique): parallax >= min_angle_deg, 4x4 DLT null vector, reprojection <= max_reproj_error
 * in both views; a train feature triangulated by an earlier match is skipped (the reference sets
 * has_landmark as it goes).  Options: Tracking::Options (tracking.h:43-44), 5.0 px / 1.0 deg. */
int vx_triangulate(vx_ctx* ctx, const double* uv1, const uint8_t* has1, int n1, const double* intr1,
                   const double* pose1, const double* uv2, const uint8_t* has2, int n2,
                   const double* intr2, const double* pose2, const vx_match* matches, int n_matches,
                   double min_angle_deg, double max_reproj_error, int32_t* out_index, double* out_pw,
                   int* n_created);

/* ---------------------------------------------------------------- geometry RANSAC (ransac.hip)
 * <- cv::solvePnPRansac(pts_3d, pts_2d, K, noArray(), rvec, tvec, false, iterations,
 *    max_reproj_error, 0.99, inliers) in Tracking::TrackWithPnP (tracking.cpp:414-423).
 * All hypotheses are generated and scored at once on the device; the sequential RANSAC loop's
 * adaptive stop rule (RANSACUpdateNumIters) is then replayed over them in order, so the selected
 * model is the one a sequential run over the same hypothesis stream keeps.  Minimal solver: P3P
 * (Grunert) on 3 points, the 4th of the sample picks among its up to 4 solutions; hypotheses come
 * from a counter-based splitmix64 stream (OpenCV's cv::RNG stream and its EPnP kernel are not
 * reproduced: parity against OpenCV is unpinned).  Inliers: point in front of the
 * camera and squared reprojection error <= reproj_error^2.  The kept model is refined on its
 * inliers by Levenberg-Marquardt (the SOLVEPNP_ITERATIVE refinement solvePnPRansac runs). */
typedef struct {
    int32_t max_iterations;    /* iterationsCount (tracking.cpp:420: min(100, 2 * n)), <= 4096 */
    int32_t refine_iterations; /* LM iterations on the inliers (0: keep the RANSAC model) */
    double reproj_error;       /* reprojectionError, px (Tracking::Options::max_reproj_error 2.0) */
    double confidence;         /* 0.99 (tracking.cpp:423) */
    uint64_t seed;             /* hypothesis stream */
} vx_pnp_options;
typedef struct {
    int32_t ok;                /* solvePnPRansac's return value */
    int32_t n_inliers;         /* inliers.rows */
    int32_t best_hypothesis;   /* index of the kept hypothesis, -1 when !ok */
    int32_t hypotheses_run;    /* hypotheses the adaptive stop rule let the loop evaluate */
    int32_t refine_iterations; /* LM iterations performed */
    int32_t reserved;
    double rvec[3], tvec[3];   /* T_cw as cv::Rodrigues vector + translation */
    double pose[7];            /* the same T_cw as Sophus storage: qx qy qz qw tx ty tz */
    double cost0, cost;        /* sum of squared reprojection errors over the inliers, before / after LM */
} vx_pnp_result;
/* tracking.cpp:420-423 defaults for n correspondences: min(100, 2n) iterations, 2.0 px, 0.99, 20 LM */
void vx_pnp_default_options(int n_points, vx_pnp_options* out);
/* obj_pts: 3 floats per correspondence (cv::Point3f), img_pts: 2 floats (cv::Point2f), intr4: fx fy
 * cx cy (no distortion, as the reference passes cv::Mat()).  inlier_mask (n bytes) may be NULL. */
int vx_pnp_ransac(vx_ctx* ctx, const float* obj_pts, const float* img_pts, int n, const double* intr4,
                  const vx_pnp_options* opt, uint8_t* inlier_mask, vx_pnp_result* out);
/* Independent problems in one pass (e.g. the C5 rig's 8 camera streams): problem p owns
 * correspondences [offsets[p], offsets[p+1]), intrinsics intr4[4p..], options opt[p]; inlier_mask
 * covers all offsets[n_problems] correspondences; out[p] per problem. */
int vx_pnp_ransac_batch(vx_ctx* ctx, int n_problems, const int32_t* offsets, const float* obj_pts,
                        const float* img_pts, const double* intr4, const vx_pnp_options* opt,
                        uint8_t* inlier_mask, vx_pnp_result* out);

/* <- E = cv::findEssentialMat(pts_last, pts_curr, K, cv::RANSAC, 0.999, 1.0, mask);
 *    inliers = cv::recoverPose(E, pts_last, pts_curr, K, R, t, mask)
 *    in Tracking::EstimatePoseByEssential (tracking.cpp:503-547).
 * Same device strategy as vx_pnp_ransac: every hypothesis (5 correspondences from a splitmix64
 * stream) is solved by the five-point method (up to 10 E, all scored by Sampson error) at once, and
 * the sequential RANSAC loop is replayed over the per-model inlier counts; the kept E is decomposed
 * (E = U diag V^T; R1 = U W V^T, R2 = U W^T V^T, t = U e3) and the four (R, +-t) are scored by DLT
 * triangulation of the RANSAC inliers (positive depth below distance_thresh in both views), OpenCV's
 * tie order.  Parity against OpenCV is unpinned (its cv::RNG stream); DESIGN.md §14. */
typedef struct {
    int32_t max_iterations;    /* findEssentialMat maxIters (OpenCV default 1000), <= 4096 */
    int32_t reserved;
    double threshold;          /* px (tracking.cpp:521: 1.0); divided by (fx + fy) / 2 */
    double confidence;         /* prob (0.999) */
    double distance_thresh;    /* recoverPose's triangulated-depth limit (50) */
    uint64_t seed;             /* hypothesis stream */
} vx_essential_options;
typedef struct {
    int32_t ok;                /* !E.empty() */
    int32_t n_inliers;         /* recoverPose's return value: RANSAC inliers in front of both views */
    int32_t n_ransac_inliers;  /* findEssentialMat's mask count */
    int32_t best_hypothesis, best_model, hypotheses_run;
    int32_t pose_candidate;    /* 0: (R1, t) 1: (R2, t) 2: (R1, -t) 3: (R2, -t) */
    int32_t reserved;
    double E[9];               /* row-major, unit Frobenius norm, x_curr^T E x_last = 0 (normalised) */
    double R[9], t[3];         /* T_cl: x_curr = R x_last + t, |t| = 1 (recoverPose's R, t) */
} vx_essential_result;
void vx_essential_default_options(vx_essential_options* out);
/* pts_last / pts_curr: 2 floats per match (cv::Point2f, tracking.cpp:506-514); mask (n bytes, may
 * be NULL) = recoverPose's output mask. */
int vx_essential_ransac(vx_ctx* ctx, const float* pts_last, const float* pts_curr, int n, const double* intr4,
                        const vx_essential_options* opt, uint8_t* mask, vx_essential_result* out);
int vx_essential_ransac_batch(vx_ctx* ctx, int n_problems, const int32_t* offsets, const float* pts_last,
                              const float* pts_curr, const double* intr4, const vx_essential_options* opt,
                              uint8_t* mask, vx_essential_result* out);

/* ---------------------------------------------------------------- recorded enqueue sequences
 * A list of the async calls above (event waits / records, vx_orb_extract_async,
 * vx_match_device_async, vx_ba_plan_run_async), recorded once with every argument and replayed by
 * vx_seq_run in the recorded order, exactly as the individual calls would run — for a pipelined
 * caller whose per-frame calls would otherwise each cross a language binding (bench.py: one step of
 * F frames = one vx_seq_run).  The recorded pointers (contexts, events, plans, device buffers) must
 * outlive the sequence.  vx_seq_run stops at the first failing call: its status is returned and
 * *failed_op (may be NULL) set to its index (-1 when every call succeeded). */
typedef struct vx_seq vx_seq;
int vx_seq_create(vx_seq** out);
void vx_seq_destroy(vx_seq* seq);
int vx_seq_wait(vx_seq* seq, vx_ctx* ctx, vx_event* ev);
int vx_seq_record(vx_seq* seq, vx_ctx* ctx, vx_event* ev);
int vx_seq_extract(vx_seq* seq, vx_ctx* ctx, const vx_orb_params* params, const uint8_t* d_img, int width,
                   int height, int channels, int64_t row_stride, int slot);
int vx_seq_match(vx_seq* seq, vx_ctx* ctx, const uint8_t* d_query, const int32_t* d_n_query, int cap_query,
                 const uint8_t* d_train, const int32_t* d_n_train, int cap_train, float ratio);
int vx_seq_ba_run(vx_seq* seq, vx_ctx* ctx, vx_ba_plan* plan);
int vx_seq_length(const vx_seq* seq);
int vx_seq_run(vx_seq* seq, int* failed_op);
/* threads > 1: vx_seq_run replays each context's calls on a host thread of its own (persistent
 * workers, one per context after the first), keeping on the host every cross-context order the
 * device semantics depend on (a wait after the record it follows in the sequence; a record after the
 * waits on the event's previous record).  1 (default): one thread, the recorded order. */
int vx_seq_set_threads(vx_seq* seq, int threads);

/* ---------------------------------------------------------------- multi-GPU (RCCL over xGMI) */
int vx_comm_unique_id(uint8_t* out_128);
int vx_comm_init(vx_ctx* ctx, const uint8_t* id_128, int nranks, int rank);
/* What RCCL itself reports for the context's communicator (ncclCommCount / ncclCommUserRank), so a
 * multi-GPU run can check it against WORLD_SIZE / RANK.  VX_ERR_STATE without a communicator. */
int vx_comm_info(vx_ctx* ctx, int* nranks, int* rank);

/* ---------------------------------------------------------------- profiling
 * When enabled, the library brackets its kernels with hipEvents on its own stream; read back
 * accumulated milliseconds and launch counts per stage (names via vx_prof_name).
 * stage_mask: 0 = off, -1 = every stage, otherwise bit s enables stage s only (so a timed run
 * can bracket just the kernel it reports without perturbing the others). */
int vx_prof_enable(vx_ctx* ctx, int stage_mask);
int vx_prof_count(void);
const char* vx_prof_name(int stage);
int vx_prof_read(vx_ctx* ctx, double* ms, int64_t* launches, int reset);

#ifdef __cplusplus
}
#endif
#endif /* VX_SLAM_H */
