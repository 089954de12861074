/*
 * oracle.h — CPU restatement of VisionX-SLAM's hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline.  The product (visionx-slam_amd/) never
 * links or calls it.
 *
 * What it restates (reference = /root/reference, QinZiwen/VisionX-SLAM @ 2026-02-13):
 *   - ORBExtractor::Extract (core/feature/orb_extractor.cpp:9-27), i.e.
 *     cv::ORB::create(n, 1.2f, 8)->detectAndCompute(img, noArray(), kps, desc)
 *     (orb_extractor.cpp:6,13).  The arithmetic lives in OpenCV 4.x (vcpkg port opencv4 at
 *     builtin-baseline 25b458671af03578e6a34edd8f0d1ac85e084df4, vcpkg.json:4,8-11), which is
 *     NOT present in this container.  The restatement follows the published OpenCV 4.x
 *     algorithm.  PARITY VS REAL OPENCV IS UNPINNED: the reference
 *     ships no tests, fixtures or golden vectors for this path.
 *   - ORBMatcher::Match (core/feature/orb_matcher.cpp:11-43): BFMatcher(NORM_HAMMING)
 *     knnMatch(k=2) + ratio test.  Unpinned vs OpenCV for the same reason.
 *   - LocalBA::Optimize (core/backend/local_ba.cpp:66-249) + ProjectToPixel
 *     (core/common/projection.h:11-31), line for line, with Eigen LDLT and Sophus SE3::exp
 *     restated.  Pinned by the reference source itself (fully visible).
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    float x, y;       /* level-0 pixel coordinates (pt *= layerScale, OpenCV computeKeyPoints) */
    float response;   /* Harris response */
    float angle;      /* degrees, fastAtan2 */
    int32_t octave;
} orc_keypoint;

typedef struct {
    int32_t query_idx, train_idx;
    float distance;
} orc_match;

/* Order of keypoints inside one pyramid level.
 *  ORC_ORDER_STL    : the std::nth_element / std::partition permutation of OpenCV's
 *                     KeyPointsFilter::retainBest as compiled against THIS libstdc++ (the order
 *                     ORBExtractor::Extract numbers Frame::Features() in on Linux; the GPU default).
 *  ORC_ORDER_RASTER : the same keypoint set in raster order (y, then x) — the GPU's opt-in
 *                     VX_ORDER_RASTER.                                                        */
enum { ORC_ORDER_STL = 0, ORC_ORDER_RASTER = 1 };

int orc_orb_quotas(int n_features, float scale_factor, int n_levels, int32_t* quotas);
int orc_orb_level_sizes(int w, int h, float scale_factor, int n_levels, int32_t* lw, int32_t* lh,
                        float* scales);
/* gray + INTER_LINEAR_EXACT pyramid; levels packed back to back (level l at offset sum_{k<l} w_k*h_k) */
int orc_orb_pyramid(const uint8_t* img, int w, int h, int channels, int64_t row_stride,
                    float scale_factor, int n_levels, uint8_t* out, int64_t out_cap);
/* FAST-9/16 + 3x3 NMS on one level, raster order; xys = (x,y,score) triples */
int orc_fast_nms(const uint8_t* img, int w, int h, int threshold, int32_t* xys, int cap, int* n_out);
/* FAST score map before NMS (0 = not a corner) */
int orc_fast_scores(const uint8_t* img, int w, int h, int threshold, uint8_t* out);
float orc_harris(const uint8_t* img, int w, int h, int x, int y);
float orc_ic_angle(const uint8_t* img, int w, int h, int x, int y);
float orc_fast_atan2(float y, float x);
/* GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) of one level (float separable path) */
int orc_blur_level(const uint8_t* img, int w, int h, uint8_t* out);

int orc_orb_extract(const uint8_t* img, int w, int h, int channels, int64_t row_stride,
                    int n_features, float scale_factor, int n_levels, int fast_threshold,
                    const int32_t* pattern /* 256*4 ints */, int order,
                    orc_keypoint* kps, uint8_t* desc, int cap, int* n_out);
/* Per-stage lists of one extraction, every level concatenated (level l's
 * counts at counts[4l .. 4l+3], each list's capacity `cap` entries):
 *   fast_xys : FAST + 3x3 NMS (x, y, score) in raster order, before runByImageBorder
 *   cand     : after runByImageBorder, raster order: (x, y, FAST score, Harris response)
 *   keep1    : retainBest(2q) by FAST score, output order, as indices into the level's cand
 *   fin      : retainBest(q) by Harris, output order, as indices into the level's cand      */
int orc_orb_stages(const uint8_t* img, int w, int h, int channels, int64_t row_stride, int n_features,
                   float scale_factor, int n_levels, int fast_threshold, int order, int32_t* counts,
                   int32_t* fast_xys, float* cand, int32_t* keep1, int32_t* fin, int64_t cap);
/* KeyPointsFilter::retainBest over bare keys (std::nth_element + std::partition with
 * comp = key-greater on (key, index) pairs): out_idx = kept indices in the library's order */
int orc_retain_best_keys(const uint32_t* keys, int n, int npts, int32_t* out_idx, int* n_out);
/* McIlroy's antiqsort adversary run against std::nth_element(begin, begin + nth, end, greater):
 * keys that defeat its median-of-3 pivots (reaching the depth limit / heap select). */
int orc_antiqsort(int n, int nth, uint32_t* out_keys);

/* BFMatcher::knnMatch(k=2) raw result per query: (train idx, dist) x 2, -1 when absent */
int orc_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx2, int32_t* dist2);
/* ORBMatcher::Match: returns count, matches in ascending query order */
int orc_match_knn2_ratio(const uint8_t* q, int nq, const uint8_t* t, int nt, float ratio,
                         orc_match* out, int cap, int* n_out);

/* ---- LocalBA on a flattened snapshot of visionx::Map ---- */
typedef struct {
    /* keyframes (any order; the reference's std::map orders them by id) */
    int32_t n_kf;
    const uint64_t* kf_id;
    double* kf_pose;            /* 7 per KF: qx qy qz qw tx ty tz (Sophus SE3d T_cw, world->camera) */
    const double* kf_intr;      /* 4 per KF: fx fy cx cy (Camera getters, camera.h:29-32) */
    const uint8_t* kf_has_cam;  /* Frame::GetCamera() != nullptr */
    const int64_t* kf_feat_ptr; /* n_kf+1 CSR into the feature arrays */
    const double* feat_uv;      /* 2 per feature: Feature::position */
    const uint64_t* feat_lm_id; /* Feature::landmark_id_ */
    const uint8_t* feat_flags;  /* bit0 has_landmark, bit1 is_outlier */
    /* landmarks (Map::landmarks_) */
    int32_t n_lm;
    const uint64_t* lm_id;
    double* lm_pos;             /* 3 per landmark */
    const uint8_t* lm_bad;
    const int64_t* lm_obs_ptr;  /* n_lm+1 CSR: Landmark::observations_ (kf_id -> feature idx) */
    const uint64_t* obs_kf_id;
    const uint64_t* obs_feat_idx;
} orc_map_view;

typedef struct {
    int32_t window_size, max_iterations, min_pose_observations, min_point_observations;
    double huber_delta, max_reproj_error;
} orc_ba_options;

typedef struct {
    int32_t iterations;          /* outer iterations executed (including the breaking one) */
    int32_t n_window_kf, n_landmarks;
    double cost[16];             /* total_cost per iteration */
    int32_t obs[16];             /* total_obs per iteration */
    double gate_margin;          /* min over all evaluations of | |e| - max_reproj_error | */
    int32_t status;              /* 0 ran, 1 early return (no map / <2 KF / no landmarks) */
} orc_ba_stats;

int orc_ba_optimize_map(orc_map_view* map, uint64_t ref_kf_id, int has_ref,
                        const orc_ba_options* opt, orc_ba_stats* stats);
/* wall seconds of the last orc_ba_optimize_map: {window + landmark-set selection, iterations} */
void orc_ba_last_timing(double* out2);

/* ---- Schur-complement joint BA (NOT in the reference: SURVEY.md §8f rank 4, BASELINE.json
 * north_star "Schur-complement marginalisation ... dense pose solve").  Restates the algorithm of
 * visionx-slam_amd/csrc/sba.hip: the LocalBA window and landmark set
 * (local_ba.cpp:42-108), the reference's residual / Jacobians / Huber weight / gates
 * (local_ba.cpp:15-40, projection.h:11-31), but ONE joint Levenberg-Marquardt system over all free
 * keyframe poses and optimised landmarks with the Gauss-Newton sign (b = +J^T W e), the landmarks
 * eliminated by the Schur complement, a dense Cholesky pose solve and back-substitution. */
typedef struct {
    int32_t window_size, max_iterations, min_point_observations;
    int32_t fixed_keyframes;     /* oldest window keyframes held fixed (gauge) */
    double huber_delta, max_reproj_error;
    double lambda_init;          /* Marquardt damping: H_ii += lambda * H_ii (+ 1e-6) */
    double rel_tol;              /* stop after an accepted step with relative decrease < rel_tol */
} orc_sba_options;

typedef struct {
    int32_t iterations;          /* assemblies (accepted, rejected and initial) */
    int32_t accepted;
    int32_t n_window_kf, n_landmarks;
    double cost[16];             /* robust (Huber) cost at each assembly */
    int32_t obs[16];             /* valid observations at each assembly */
    int32_t step[16];            /* 2 initial, 1 accepted, 0 rejected, 3 re-assembled after a reject */
    double lambda;               /* damping after the last iteration */
    double initial_cost, final_cost;
    int32_t status;              /* 0 ran, 1 early return */
} orc_sba_stats;

int orc_sba_optimize_map(orc_map_view* map, uint64_t ref_kf_id, int has_ref,
                         const orc_sba_options* opt, orc_sba_stats* stats);
/* Reduced pose system (Schur complement S, n x n row-major, lower triangle meaningful, and rhs)
 * assembled at the map's current state with damping `lambda`; n = 6 * window keyframes. */
int orc_sba_system(const orc_map_view* map, uint64_t ref_kf_id, int has_ref,
                   const orc_sba_options* opt, double lambda, double* S, double* rhs, int n);
/* One landmark shard's partial reduced system (csrc/sba.hip's sharded run before its ncclAllReduce):
 * the observations of landmarks with splitmix64(id) mod shard_count == shard_rank only, without the
 * pose damping and the fixed-keyframe gauge; HTd (n) = the shard's pose-block diagonals,
 * cost_count = {cost, valid observations}.  Summed over the ranks and finished (damping, gauge) it is
 * orc_sba_system's system. */
int orc_sba_system_shard(const orc_map_view* map, uint64_t ref_kf_id, int has_ref, const orc_sba_options* opt,
                         double lambda, int shard_rank, int shard_count, double* S, double* rhs, double* HTd,
                         double* cost_count, int n);

/* ---- keyframe-insertion landmark creation (landmark_oracle.cpp), same contract as vx_slam.h */
int orc_depth_landmarks(const double* feat_uv, const uint8_t* feat_has_lm, int n_feat, const void* depth,
                        int depth_type /* 0 u16, 1 f32, 2 f64 */, int rows, int cols, int64_t row_stride,
                        const double* intr4, const double* pose7, int32_t* out_index, double* out_pw,
                        int* n_created);
int orc_triangulate(const double* uv1, const uint8_t* has1, int n1, const double* intr1, const double* pose1,
                    const double* uv2, const uint8_t* has2, int n2, const double* intr2, const double* pose2,
                    const orc_match* matches, int n_matches, double min_angle_deg, double max_reproj_error,
                    int32_t* out_index, double* out_pw, int* n_created);

/* ---- PnP RANSAC (ransac_oracle.cpp), same contract and struct layout as vx_slam.h's vx_pnp_* */
#define ORC_PNP_MAX_HYP 4096
typedef struct {
    int32_t max_iterations, refine_iterations;
    double reproj_error, confidence;
    uint64_t seed;
} orc_pnp_options;
typedef struct {
    int32_t ok, n_inliers, best_hypothesis, hypotheses_run, refine_iterations, reserved;
    double rvec[3], tvec[3], pose[7], cost0, cost;
} orc_pnp_result;
int orc_pnp_ransac_batch(int n_problems, const int32_t* offsets, const float* obj, const float* img,
                         const double* intr4, const orc_pnp_options* opt, uint8_t* mask, orc_pnp_result* out);
/* pieces, for the numpy pins: hypothesis h's model (1 = valid), P3P on 3 world points + unit
 * bearings (up to 4 solutions), real roots of a degree <= 4 polynomial, RANSACUpdateNumIters */
int orc_pnp_hypothesis(const float* obj, const float* img, int n, const double* intr4, uint64_t seed, int h,
                       double* R9, double* t3);
int orc_p3p(const double* P9, const double* f9, double* R72, double* t24);  /* up to 8 candidates */
int orc_poly_roots(const double* c, int d, double* out);
int orc_pnp_update_iters(double p, double ep, int max_iters);

/* ---- essential-matrix RANSAC + recoverPose (essential_oracle.cpp), layout = vx_essential_* */
#define ORC_EM_MAX_HYP 4096
typedef struct {
    int32_t max_iterations, reserved;
    double threshold, confidence, distance_thresh;
    uint64_t seed;
} orc_essential_options;
typedef struct {
    int32_t ok, n_inliers, n_ransac_inliers, best_hypothesis, best_model, hypotheses_run, pose_candidate, reserved;
    double E[9], R[9], t[3];
} orc_essential_result;
int orc_essential_ransac_batch(int n_problems, const int32_t* offsets, const float* pts1, const float* pts2,
                               const double* intr4, const orc_essential_options* opt, uint8_t* mask,
                               orc_essential_result* out);
/* five-point solver on 5 normalised correspondences: up to 10 unit-norm E (row-major) */
int orc_five_point(const double* x1, const double* x2, double* Es);

#ifdef __cplusplus
}
#endif
