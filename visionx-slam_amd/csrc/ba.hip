// ba.hip — sliding-window bundle adjustment on gfx950 (LocalBA::Optimize drop-in).
//
// Replaces LocalBA::Optimize (core/backend/local_ba.cpp:66-249).  The reference alternates a
// per-keyframe 6x6 Gauss-Newton step with landmarks fixed (:116-174) and a per-landmark 3x3 step
// with poses fixed (:176-238), up to max_iterations times with a relative-cost stop (:240-247).
// Both stages are embarrassingly parallel, so the device problem is two CSR views of the window:
//
//   host   plan:  SelectKeyFrames (:42-62) + landmark filtering (:93-104) + the per-observation
//                 validity checks that are static during Optimize (:131-138, :186-204) ->
//                 keyframe-major pose observations (uv, landmark slot) and landmark-major
//                 observations (uv, keyframe row); uploaded once, replayed by every run.
//   device run (per iteration it; every kernel early-exits once the stop rule has fired):
//     k_pose_kf        n_split workgroups per keyframe, each over a slice of its observations
//                      (about one per thread): project (ProjectToPixel, projection.h:11-31), gate,
//                      weight, the 21 + 6 + 2 normal-equation terms of the 2x6 PoseJacobian in
//                      registers; a halving-butterfly wave reduction + LDS tree writes the slice's
//                      29-term partial block (fixed order: deterministic)
//     [sharded only]   ncclAllReduce(sum, f64) of the partial blocks over the landmark shards
//                      (one collective per iteration, 32 doubles per keyframe slice)
//     k_landmark_solve every workgroup sums the slice partials in slice order and solves ALL window
//                      keyframes redundantly (one lane per keyframe: H += 1e-6 I, Eigen-style
//                      pivoted LDLT, finite check, T <- exp(dx) T) into LDS — bitwise identical in
//                      every workgroup — while its landmark-stage loads are in flight; then one
//                      thread per landmark OBSERVATION forms its 9 terms (Jp * R), the thread owning
//                      each landmark sums them in CSR order and solves the 3x3 (p += dp).
//                      Workgroup 0 publishes the poses and evaluates the stop rule.
//                      Windows beyond kMaxKfLds keyframes use k_pose_solve_g + k_landmark instead.
// Iterations alternate two pose buffers (no launch reads what another workgroup of it writes);
// iteration 0 reads the initial poses / positions directly, so a run needs no reset launch.
// The step keeps the reference's sign (b = -J^T e, :156 and :224): this is a drop-in, not a fix.
#include <algorithm>
#include <cmath>
#include <type_traits>
#include <cstring>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "vx_internal.hpp"
#include "vx_ktrace.hpp"
#include "ba_common.hpp"
#include "ba_plan.hpp"
#include "dmap.hpp"

namespace vx {
namespace {

using namespace vx::ba;

constexpr int kPoseBlock = kBaPoseBlock;  // threads per pose-stage workgroup
constexpr int kNTerms = 29;      // 21 H (upper) + 6 b + cost + count
constexpr int kStride = 32;      // doubles per keyframe block in global memory
// LDS slot stride of k_landmark_solve: 33, not 32 doubles — a 256-B stride is one full turn of the
// 64 four-byte LDS banks, so lanes reading different keyframes' slots would all hit one bank
constexpr int kLdsStride = 33;
constexpr int kMaxIter = 64;
// keyframes whose LDS slots fit k_landmark_solve: 448 * 33 * 8 B + kLmBlock * (9 * 8 + 4) B =
// 157,184 B of gfx950's 160 KB per workgroup
constexpr int kMaxKfLds = 448;
constexpr int kMaxSplit = kBaMaxSplit;    // pose-stage workgroups per keyframe
constexpr int kCombine = 6;      // (keyframe, term) pairs per thread per combine pass
constexpr int kLmBlock = kBaLmBlock;      // k_landmark_solve: threads = max observations = max landmarks
static_assert(kLmBlock >= kMaxKfLds, "k_landmark_solve solves one keyframe per thread");
static_assert((size_t)kMaxKfLds * kLdsStride * sizeof(double) + (size_t)kLmBlock * (9 * sizeof(double) + sizeof(int)) <=
                  160 * 1024, "k_landmark_solve LDS exceeds gfx950's 160 KB per workgroup");

VX_KT_TABLE();

struct BAState {
    int active[kMaxIter + 1];  // active[it]: iteration it runs
    int iterations;
    int pad;
    double last_cost;
    double cost[16];
    int obs[16];
};

struct BAArgs {
    int n_kf, n_opt, n_lm, pad0;
    int min_pose_obs, min_point_obs, max_iter, n_split;
    double huber, max_err;
    const double* kf_pose0;  // 8 per KF: qx qy qz qw tx ty tz 0
    double* kf_pose;         // 2 x n_kf x 8: ping-pong by iteration parity (see pose_in / pose_out)
    const double* kf_intr;   // 4 per KF
    double* kf_rot;          // 9 per KF (rotation matrix of the current pose)
    const int* kf_flags;     // bit0: keyframe has a camera
    const int* kf_obs_ptr;   // n_kf + 1, CSR into the pose observations
    double* kf_part;         // n_kf * n_split * kStride partial normal-equation blocks (all-reduced when sharded)
    double* kf_cost;         // 2 per KF: pose-stage cost and observation count
    const double* lm_pos0;   // 4 per landmark
    double* lm_pos;
    const double2* pobs_uv;
    const int* pobs_lm;
    const int* lobs_ptr;     // n_opt + 1
    const int* lobs_kf;
    const int* lobs_lm;      // landmark slot of each landmark-stage observation
    const int* lm_blk;       // k_landmark_solve workgroup -> {first landmark, first observation} (n_blocks + 1)
    const double2* lobs_uv;
    BAState* state;
};


// Iteration `it` reads the poses of iteration it-1 (the initial poses at it == 0) and writes the
// other buffer, so no launch ever reads a pose another workgroup of the same launch writes.  The
// landmarks [n_opt, n_lm) are never optimised (other shards' landmarks) and always read initial.
__device__ __forceinline__ const double* pose_in(const BAArgs& a, int it) {
    return it == 0 ? a.kf_pose0 : a.kf_pose + (long long)(it & 1) * a.n_kf * 8;
}
__device__ __forceinline__ double* pose_out(const BAArgs& a, int it) {
    return a.kf_pose + (long long)((it + 1) & 1) * a.n_kf * 8;
}
__device__ __forceinline__ const double* lm_in(const BAArgs& a, int it, int s) {
    return (it == 0 || s >= a.n_opt ? a.lm_pos0 : a.lm_pos) + 4 * (long long)s;
}


// Pose step of one keyframe from its summed terms S (local_ba.cpp:163-173): skipped below
// min_pose_observations or without a camera; T updated in place, R = its rotation (:173, :220).
__device__ __forceinline__ void solve_pose(const BAArgs& a, int flags, const double* S, double* T, double* R) {
    const int obs = (int)S[28];
    if (obs >= a.min_pose_obs && (flags & 1)) {
        double U[21], b[6], dx[6];
#pragma unroll
        for (int t = 0; t < 21; ++t) U[t] = S[t];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            U[hidx(r, r)] += 1e-6;
            b[r] = S[21 + r];
        }
        spd6_block_solve(U, b, dx);
        bool fin = true;
#pragma unroll
        for (int r = 0; r < 6; ++r) fin = fin && isfinite(dx[r]);
        if (fin) se3_left_update(dx, T);
    }
    rot_from_quat(T, R);
}

// Relative-cost stop rule (local_ba.cpp:240-247) -> active[it + 1].  Iteration 0 starts the run's
// state (last_cost = numeric_limits<double>::max(), local_ba.cpp:110); a stop clears every later
// flag, a continue sets the next one (later ones are rewritten before they are read).
__device__ void stop_rule(const BAArgs& a, int it, double total, int tobs) {
    BAState* s = a.state;
    if (it == 0)
        for (int k = 1; k < 16; ++k) {
            s->cost[k] = 0;
            s->obs[k] = 0;
        }
    if (it < 16) {
        s->cost[it] = total;
        s->obs[it] = tobs;
    }
    s->iterations = it + 1;
    const double last = it == 0 ? 1.7976931348623157e308 : s->last_cost;
    const bool stop = tobs == 0 || fabs(last - total) < 1e-6 * last;
    if (!stop) s->last_cost = total;
    if (!stop && it + 1 < a.max_iter)
        s->active[it + 1] = 1;
    else
        for (int k = it + 1; k <= a.max_iter; ++k) s->active[k] = 0;
}

// Ordered (fixed-tree) pose-stage totals over the keyframes; the calling wave must be complete.
__device__ void totals_and_stop(const BAArgs& a, int it, int lane) {
    double total = 0.0;
    int tobs = 0;
    for (int j = lane; j < a.n_kf; j += 64) {
        total += a.kf_cost[2 * j];
        tobs += (int)a.kf_cost[2 * j + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        total += __shfl_xor(total, o, 64);
        tobs += __shfl_xor(tobs, o, 64);
    }
    if (lane == 0) stop_rule(a, it, total, tobs);
}

// Only for max_iterations == 0 (nothing runs): the result is the initial state.  Iteration 0 of
// the kernels below reads the initial arrays directly, so a normal run has no reset launch.
__global__ void k_ba_reset(BAArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n_kf * 8) a.kf_pose[i] = a.kf_pose0[i];
    if (i < a.n_lm * 4) a.lm_pos[i] = a.lm_pos0[i];
    if (i == 0) {
        BAState* s = a.state;
        for (int k = 0; k <= kMaxIter; ++k) s->active[k] = 0;
        s->iterations = 0;
        for (int k = 0; k < 16; ++k) { s->cost[k] = 0; s->obs[k] = 0; }
    }
}

// Pose stage (local_ba.cpp:116-161): n_split workgroups per keyframe, each over a contiguous
// slice of the keyframe's observations.  Each thread accumulates the 29 terms of its observations
// (strided) in registers; a fixed-order wave butterfly + LDS tree reduces them into the slice's
// partial block kf_part[k * n_split + slice].  Partials are summed later in slice order, so the
// result is deterministic (and identical on every rank after the sharded all-reduce).
__global__ __launch_bounds__(kPoseBlock) void k_pose_kf(BAArgs a, int it) {
    if (it > 0 && !a.state->active[it]) return;
    __shared__ double red[kPoseBlock / 64][kNTerms];
    VX_KT(0);
    const int k = blockIdx.x / a.n_split, slice = blockIdx.x - k * a.n_split;
    const int p0 = a.kf_obs_ptr[k], p1 = a.kf_obs_ptr[k + 1];
    const int len = (p1 - p0 + a.n_split - 1) / a.n_split;
    const int i0 = p0 + slice * len, i1 = min(p1, i0 + len);
    // the thread's first observation and its landmark are requested before the pose, so the
    // dependent gather overlaps the pose / intrinsics loads
    const int ifirst = i0 + (int)threadIdx.x;
    D3 P0{0, 0, 0};
    double2 uv0 = make_double2(0.0, 0.0);
    if (ifirst < i1) {
        uv0 = a.pobs_uv[ifirst];
        const double* P = lm_in(a, it, a.pobs_lm[ifirst]);
        P0 = {P[0], P[1], P[2]};
    }
    const double* Tin = pose_in(a, it);
    double T[8], C[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) T[j] = Tin[8 * k + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) C[j] = a.kf_intr[4 * k + j];
    const double fx = C[0], fy = C[1];
    VX_KT(1);
    double v[kNTerms];
#pragma unroll
    for (int t = 0; t < kNTerms; ++t) v[t] = 0.0;
    for (int i = ifirst; i < i1; i += kPoseBlock) {
        D3 Pw = P0;
        double2 uv = uv0;
        if (i != ifirst) {
            uv = a.pobs_uv[i];
            const double* P = lm_in(a, it, a.pobs_lm[i]);
            Pw = {P[0], P[1], P[2]};
        }
        const D3 pc = se3_apply(T, Pw);
        if (!(pc.z > 1e-6)) continue;
        const double inv_z = frcp(pc.z);
        const double x = pc.x * inv_z, y = pc.y * inv_z;
        const double e0 = uv.x - (fx * x + C[2]);
        const double e1 = uv.y - (fy * y + C[3]);
        const double e2 = e0 * e0 + e1 * e1;
        const double re = e2 > 0.0 ? frsq(e2) : 0.0;
        const double en = e2 * re;  // |e| without a sqrt + division on the chain
        if (en > a.max_err) continue;
        const double w = en <= a.huber ? 1.0 : a.huber * re;
        // J = Jp * [I | -hat(pc)] (local_ba.cpp:15-33) with Jp = [[jp0, 0, jp2], [0, jp4, jp5]],
        // written out without its structural zeros (J0[1] = J1[0] = 0)
        const double jp0 = fx * inv_z, jp2 = -jp0 * x, jp4 = fy * inv_z, jp5 = -jp4 * y;
        const double J0[6] = {jp0, 0.0, jp2, jp2 * pc.y, jp0 * pc.z - jp2 * pc.x, -jp0 * pc.y};
        const double J1[6] = {0.0, jp4, jp5, jp5 * pc.y - jp4 * pc.z, -jp5 * pc.x, jp4 * pc.x};
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = r; c < 6; ++c) {
                const bool u0 = r != 1 && c != 1, u1 = r != 0 && c != 0;  // compile-time after unroll
                const double t0 = u0 ? (w * J0[r]) * J0[c] : 0.0;
                const double t1 = u1 ? (w * J1[r]) * J1[c] : 0.0;
                v[hidx(r, c)] += (u0 && u1) ? t0 + t1 : (u0 ? t0 : t1);
            }
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            const double g = r == 0 ? J0[0] * e0 : (r == 1 ? J1[1] * e1 : J0[r] * e0 + J1[r] * e1);
            v[21 + r] -= w * g;
        }
        v[27] += w * (e0 * e0 + e1 * e1);
        v[28] += 1.0;
    }
    VX_KT(2);
    // wave reduction of the 29 terms (halving butterfly, wave_sum32)
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double r[kStride];
#pragma unroll
    for (int t = 0; t < kStride; ++t) r[t] = t < kNTerms ? v[t] : 0.0;
    const double tot = wave_sum32(r);
    VX_KT(3);
    if ((lane & 1) == 0 && (lane >> 1) < kNTerms) red[wv][lane >> 1] = tot;
    __syncthreads();
    VX_KT(4);
    if (threadIdx.x < kStride) {
        double s = 0.0;
        if (threadIdx.x < kNTerms) {
            s = red[0][threadIdx.x];
#pragma unroll
            for (int w2 = 1; w2 < kPoseBlock / 64; ++w2) s += red[w2][threadIdx.x];
        }
        a.kf_part[(long long)blockIdx.x * kStride + threadIdx.x] = s;
    }
    VX_KT(5);
}

// Sum of keyframe k's slice partials for term t, in slice order (absent slices add +0.0).
__device__ __forceinline__ double combine_term(const BAArgs& a, int k, int t) {
    const double* src = a.kf_part + (long long)k * a.n_split * kStride + t;
    double v[kMaxSplit];
#pragma unroll
    for (int c = 0; c < kMaxSplit; ++c) v[c] = c < a.n_split ? src[c * kStride] : 0.0;
    double s = v[0];
#pragma unroll
    for (int c = 1; c < kMaxSplit; ++c) s += v[c];
    return s;
}

// The 9 normal-equation terms {H00 H01 H02 H11 H12 H22 b0 b1 b2} of one landmark observation
// (local_ba.cpp:206-224) against keyframe k of tables T/R/C (strides in doubles), branch-free:
// returns false for a gated-out observation (behind the camera or beyond max_reproj_error),
// whose terms are then exactly +0.0.
__device__ __forceinline__ bool obs_terms(const BAArgs& a, D3 P, int k, double2 uv, const double* T0, int tst,
                                          const double* R0, int rst, const double* C0, int cst, double* h) {
    const double* T = T0 + (long long)tst * k;
    const double* C = C0 + (long long)cst * k;
    const D3 pc = se3_apply(T, P);
    const bool front = pc.z > 1e-6;
    const double inv_z = frcp(pc.z);
    const double x = pc.x * inv_z, y = pc.y * inv_z;
    const double fx = C[0], fy = C[1];
    const double e0 = uv.x - (fx * x + C[2]);
    const double e1 = uv.y - (fy * y + C[3]);
    const double e2 = e0 * e0 + e1 * e1;
    const double re = e2 > 0.0 ? frsq(e2) : 0.0;
    const double en = e2 * re;
    const bool ok = front && !(en > a.max_err);
    const double w = en <= a.huber ? 1.0 : a.huber * re;
    const double jp0 = fx * inv_z, jp2 = -jp0 * x, jp4 = fy * inv_z, jp5 = -jp4 * y;
    const double* R = R0 + (long long)rst * k;
    // J = Jp * R with Jp's structural zeros dropped (local_ba.cpp:219-221)
    double J0[3], J1[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        J0[c] = jp0 * R[c] + jp2 * R[6 + c];
        J1[c] = jp4 * R[3 + c] + jp5 * R[6 + c];
    }
    h[0] = ok ? (w * J0[0]) * J0[0] + (w * J1[0]) * J1[0] : 0.0;
    h[1] = ok ? (w * J0[0]) * J0[1] + (w * J1[0]) * J1[1] : 0.0;
    h[2] = ok ? (w * J0[0]) * J0[2] + (w * J1[0]) * J1[2] : 0.0;
    h[3] = ok ? (w * J0[1]) * J0[1] + (w * J1[1]) * J1[1] : 0.0;
    h[4] = ok ? (w * J0[1]) * J0[2] + (w * J1[1]) * J1[2] : 0.0;
    h[5] = ok ? (w * J0[2]) * J0[2] + (w * J1[2]) * J1[2] : 0.0;
    h[6] = ok ? w * ((-J0[0]) * e0 + (-J1[0]) * e1) : 0.0;
    h[7] = ok ? w * ((-J0[1]) * e0 + (-J1[1]) * e1) : 0.0;
    h[8] = ok ? w * ((-J0[2]) * e0 + (-J1[2]) * e1) : 0.0;
    return ok;
}

// Landmark update from its summed terms (local_ba.cpp:228-237): skipped below min_point_obs or
// for a non-finite step; the position is written either way (iteration 0 reads lm_pos0).
__device__ __forceinline__ void lm_update(const BAArgs& a, int l, D3 P, const double* h, int obs) {
    D3 out = P;
    if (obs >= a.min_point_obs) {
        double H[9] = {h[0] + 1e-6, h[1], h[2], h[1], h[3] + 1e-6, h[4], h[2], h[4], h[5] + 1e-6};
        const double b[3] = {h[6], h[7], h[8]};
        double dp[3];
        ldlt_spd_solve<3>(H, b, dp);
        if (isfinite(dp[0]) && isfinite(dp[1]) && isfinite(dp[2])) out = {P.x + dp[0], P.y + dp[1], P.z + dp[2]};
    }
    double* Pp = a.lm_pos + 4 * l;
    Pp[0] = out.x;
    Pp[1] = out.y;
    Pp[2] = out.z;
}

// Pose solve of every window keyframe (redundantly in each workgroup) + landmark stage, one launch.
// Workgroup b covers the whole landmarks [lm_blk[b], lm_blk[b+1]) (at most kLmBlock landmarks
// and kLmBlock observations, packed on the host).  Thread t projects observation o0 + t and
// leaves its 9 terms in LDS; the thread owning landmark l0 + t then sums its observations' terms
// in CSR order (the order of the per-landmark loop, local_ba.cpp:186) and solves the 3x3.
// Every load of the landmark stage is issued first, so it lands during the combine and solve.
// LDS: one kLdsStride-double slot per keyframe (combined normal equations S, then T 8 | R 9 | C 4) and
// 9 x kLmBlock observation terms.
__global__ __launch_bounds__(kLmBlock) void k_landmark_solve(BAArgs a, int it) {
    if (it > 0 && !a.state->active[it]) return;
    extern __shared__ __attribute__((aligned(16))) double kf_lds[];
    double* terms = kf_lds + (long long)a.n_kf * kLdsStride;  // [9][kLmBlock]
    const int tid = threadIdx.x;
    VX_KT(8);
    const int2 b0 = reinterpret_cast<const int2*>(a.lm_blk)[blockIdx.x];
    const int2 b1 = reinterpret_cast<const int2*>(a.lm_blk)[blockIdx.x + 1];
    const int l0 = b0.x, l1 = b1.x, ob0 = b0.y, ob1 = b1.y;
    // this thread's observation ...
    const int o = ob0 + tid;
    const bool has_o = o < ob1;
    const int ol = has_o ? a.lobs_lm[o] : l0;
    const int ok_kf = has_o ? a.lobs_kf[o] : 0;
    const double2 ouv = has_o ? a.lobs_uv[o] : make_double2(1e300, 1e300);
    const double* Po = lm_in(a, it, ol);
    const D3 PO{Po[0], Po[1], Po[2]};
    // ... and the landmark it owns
    const int l = l0 + tid;
    const bool own = l < l1;
    const int r0 = own ? a.lobs_ptr[l] - ob0 : 0, r1 = own ? a.lobs_ptr[l + 1] - ob0 : 0;
    const double* Pl = lm_in(a, it, own ? l : l0);
    const D3 PL{Pl[0], Pl[1], Pl[2]};
    // ... and the keyframe it solves (pose of the previous iteration, intrinsics, flags): their
    // load latency also passes during the combine instead of after it
    double kT[8] = {0, 0, 0, 0, 0, 0, 0, 0}, kC[4] = {0, 0, 0, 0};
    int kflg = 0;
    if (tid < a.n_kf) {
        const double* Tin = pose_in(a, it);
#pragma unroll
        for (int j = 0; j < 8; ++j) kT[j] = Tin[8 * tid + j];
#pragma unroll
        for (int j = 0; j < 4; ++j) kC[j] = a.kf_intr[4 * tid + j];
        kflg = a.kf_flags[tid];
    }
    VX_KT(9);
    // slice partials -> S: kCombine (keyframe, term) pairs per thread and pass, all their slice
    // loads issued together
    {
        const int ne = a.n_kf * kNTerms;
        for (int e0 = tid; e0 < ne; e0 += kCombine * blockDim.x) {
            double v[kCombine][kMaxSplit];
#pragma unroll
            for (int q = 0; q < kCombine; ++q) {
                const int e = e0 + q * blockDim.x;
                const int k = e / kNTerms, t = e - k * kNTerms;
                const double* src = a.kf_part + (long long)k * a.n_split * kStride + t;
#pragma unroll
                for (int c = 0; c < kMaxSplit; ++c) v[q][c] = (e < ne && c < a.n_split) ? src[c * kStride] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < kCombine; ++q) {
                const int e = e0 + q * blockDim.x;
                if (e >= ne) continue;
                const int k = e / kNTerms, t = e - k * kNTerms;
                double s = v[q][0];
#pragma unroll
                for (int c = 1; c < kMaxSplit; ++c) s += v[q][c];
                kf_lds[k * kLdsStride + t] = s;
            }
        }
    }
    __syncthreads();
    VX_KT(10);
    double* Tout = pose_out(a, it);
    if (tid < a.n_kf) {  // kLmBlock >= kMaxKfLds: one keyframe per thread at most
        const int k = tid;
        double* slot = kf_lds + k * kLdsStride;
        double S[kNTerms];
#pragma unroll
        for (int t = 0; t < kNTerms; ++t) S[t] = slot[t];
        double T[8], R[9];
#pragma unroll
        for (int j = 0; j < 8; ++j) T[j] = kT[j];
        solve_pose(a, kflg, S, T, R);
#pragma unroll
        for (int j = 0; j < 8; ++j) slot[j] = T[j];
#pragma unroll
        for (int j = 0; j < 9; ++j) slot[8 + j] = R[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) slot[17 + j] = kC[j];
        if (blockIdx.x == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) Tout[8 * k + j] = T[j];
#pragma unroll
            for (int j = 0; j < 9; ++j) a.kf_rot[9 * k + j] = R[j];
            a.kf_cost[2 * k] = S[27];
            a.kf_cost[2 * k + 1] = S[28];
        }
    }
    __syncthreads();  // also makes block 0's kf_cost stores visible inside block 0
    VX_KT(11);
    if (blockIdx.x == 0 && tid < 64) totals_and_stop(a, it, tid);
    {
        double h[9];
        const bool ok = obs_terms(a, PO, ok_kf, ouv, kf_lds, kLdsStride, kf_lds + 8, kLdsStride, kf_lds + 17,
                                  kLdsStride, h);
#pragma unroll
        for (int j = 0; j < 9; ++j) terms[j * kLmBlock + tid] = h[j];
        reinterpret_cast<int*>(terms + 9 * kLmBlock)[tid] = (has_o && ok) ? 1 : 0;  // counted observation
    }
    __syncthreads();
    VX_KT(13);
    if (own) {
        double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        int obs = 0;
        const int* okf = reinterpret_cast<const int*>(terms + 9 * kLmBlock);
        for (int r = r0; r < r1; ++r) {
#pragma unroll
            for (int j = 0; j < 9; ++j) h[j] += terms[j * kLmBlock + r];
            obs += okf[r];
        }
        lm_update(a, l, PL, h, obs);
    }
    VX_KT(12);
}

// Large-window fallback (n_kf > kMaxKfLds): one thread per keyframe solves into global memory...
__global__ __launch_bounds__(256) void k_pose_solve_g(BAArgs a, int it) {
    if (it > 0 && !a.state->active[it]) return;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n_kf) return;
    double S[kNTerms];
#pragma unroll
    for (int t = 0; t < kNTerms; ++t) S[t] = combine_term(a, k, t);
    const double* Tin = pose_in(a, it);
    double* Tout = pose_out(a, it);
    double T[8], R[9];
#pragma unroll
    for (int j = 0; j < 8; ++j) T[j] = Tin[8 * k + j];
    solve_pose(a, a.kf_flags[k], S, T, R);
#pragma unroll
    for (int j = 0; j < 8; ++j) Tout[8 * k + j] = T[j];
#pragma unroll
    for (int j = 0; j < 9; ++j) a.kf_rot[9 * k + j] = R[j];
    a.kf_cost[2 * k] = S[27];
    a.kf_cost[2 * k + 1] = S[28];
}

// ... and the landmark stage reads the poses from global memory, one thread per landmark; wave 0
// of block 0 evaluates the stop rule (active[it + 1] is read by no block of this launch).
__global__ __launch_bounds__(256) void k_landmark(BAArgs a, int it) {
    if (it > 0 && !a.state->active[it]) return;
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 64) totals_and_stop(a, it, threadIdx.x);
    if (l >= a.n_opt) return;
    const double* Pin = lm_in(a, it, l);
    const D3 P{Pin[0], Pin[1], Pin[2]};
    double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, t[9];
    int obs = 0;
    const double* T0 = pose_out(a, it);
    for (int o = a.lobs_ptr[l]; o < a.lobs_ptr[l + 1]; ++o) {
        obs += obs_terms(a, P, a.lobs_kf[o], a.lobs_uv[o], T0, 8, a.kf_rot, 9, a.kf_intr, 4, t) ? 1 : 0;
#pragma unroll
        for (int j = 0; j < 9; ++j) h[j] += t[j];
    }
    lm_update(a, l, P, h, obs);
}


}  // namespace
}  // namespace vx


namespace vx {
namespace {

BAArgs make_args(vx_ba_plan* p) {
    BAArgs a{};
    a.n_kf = p->n_kf;
    a.n_opt = p->n_opt;
    a.n_lm = p->n_lm;
    a.min_pose_obs = p->opt.min_pose_observations;
    a.min_point_obs = p->opt.min_point_observations;
    a.max_iter = p->opt.max_iterations;
    a.huber = p->opt.huber_delta;
    a.max_err = p->opt.max_reproj_error;
    a.kf_pose0 = p->kf_pose0.as<double>();
    a.kf_pose = p->kf_pose.as<double>();
    a.kf_intr = p->kf_intr.as<double>();
    a.kf_rot = p->kf_rot.as<double>();
    a.kf_flags = p->kf_flags.as<int>();
    a.kf_obs_ptr = p->kf_obs_ptr.as<int>();
    a.kf_part = p->kf_part.as<double>();
    a.n_split = p->n_split;
    a.kf_cost = p->kf_cost.as<double>();
    a.lm_pos0 = p->lm_pos0.as<double>();
    a.lm_pos = p->lm_pos.as<double>();
    a.pobs_uv = p->pobs_uv.as<double2>();
    a.pobs_lm = p->pobs_lm.as<int>();
    a.lobs_ptr = p->lobs_ptr.as<int>();
    a.lobs_kf = p->lobs_kf.as<int>();
    a.lobs_lm = p->lobs_lm.as<int>();
    a.lm_blk = p->lm_blk.as<int>();
    a.lobs_uv = p->lobs_uv.as<double2>();
    a.state = p->state.as<BAState>();
    return a;
}

template <class T>
int upload(vx_ctx* c, DevBuf& d, const std::vector<T>& h) {
    VX_HIP(c, d.ensure(std::max<size_t>(1, h.size()) * sizeof(T)));
    if (!h.empty()) VX_HIP(c, hipMemcpy(d.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return VX_OK;
}

}  // namespace

// k_landmark_solve workgroups: whole landmarks, at most kLmBlock landmarks and observations each
// (a window of <= kMaxKfLds keyframes gives a landmark <= kMaxKfLds < kLmBlock of them)
// Returned as {first landmark, its first observation} per workgroup (n_blocks + 1 pairs), so a
// workgroup reads both in one load instead of a dependent lobs_ptr load after lm_blk.
// A landmark with more than kLmBlock observations (possible only if a snapshot lists one keyframe
// twice for it) gets a workgroup of its own and *max_cnt reports it: plan_run then takes the
// one-thread-per-landmark kernels, which have no such limit.
std::vector<int> pack_lm_blocks(const std::vector<int>& lptr, int n_opt, int* max_cnt) {
    std::vector<int> blk{0, lptr[0]};
    int n_o = 0, n_l = 0, mx = 0;
    for (int s = 0; s < n_opt; ++s) {
        const int cnt = lptr[s + 1] - lptr[s];
        mx = std::max(mx, cnt);
        if (n_l + 1 > kLmBlock || n_o + cnt > kLmBlock) {
            blk.push_back(s);
            blk.push_back(lptr[s]);
            n_o = n_l = 0;
        }
        n_o += cnt;
        ++n_l;
    }
    blk.push_back(n_opt);
    blk.push_back(lptr[n_opt]);
    if (max_cnt) *max_cnt = mx;
    return blk;
}

// Work buffers of a run (both plan builders end here): ping-pong poses, rotations, pose-stage
// partial blocks, costs, landmark positions and the iteration state.
namespace {
// a finished run's window poses (ping-pong buffer of the last iteration) and optimised landmark
// positions into the resident map's rows
__global__ void k_apply_dmap(const BAState* st, const double* kf_pose, int n_kf, const double* lm_pos, int n_opt,
                             const int* kf_map, const int* lm_map, double* map_pose, double* map_pos) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_kf) {
        const double* src = kf_pose + (size_t)(st->iterations & 1) * n_kf * 8 + (size_t)8 * i;
        for (int j = 0; j < 7; ++j) map_pose[(size_t)7 * kf_map[i] + j] = src[j];
    }
    if (i < n_opt)
        for (int j = 0; j < 3; ++j) map_pos[(size_t)3 * lm_map[i] + j] = lm_pos[(size_t)4 * i + j];
}
}  // namespace

int alloc_run_buffers(vx_ctx* c, vx_ba_plan* p) {
    const size_t nk = (size_t)p->n_kf;
    VX_HIP(c, p->kf_pose.ensure(nk * 2 * 8 * sizeof(double)));
    VX_HIP(c, p->kf_rot.ensure(nk * 9 * sizeof(double)));
    VX_HIP(c, p->kf_part.ensure(nk * p->n_split * kStride * sizeof(double)));
    VX_HIP(c, p->kf_cost.ensure(nk * 2 * sizeof(double)));
    VX_HIP(c, p->lm_pos.ensure((size_t)std::max(p->n_lm, 1) * 4 * sizeof(double)));
    VX_HIP(c, p->state.ensure(sizeof(BAState)));
    return VX_OK;
}

namespace {

int build_plan(vx_ctx* c, const vx_map_view* m, uint64_t ref_kf_id, int has_ref, vx_ba_plan* p,
               bool device = true) {
    const vx_ba_options& o = p->opt;
    p->status = 1;
    if (!m || m->n_kf <= 0) return VX_OK;
    // ---- SelectKeyFrames (local_ba.cpp:42-62) + landmark set (local_ba.cpp:83-108)
    Window W;
    select_window(m, ref_kf_id, has_ref, o.window_size, o.min_point_observations, W);
    const std::vector<int>& win = W.win;
    const auto& win_row = W.win_row;
    const auto& lm_by_id = W.lm_by_id;
    const std::vector<int>& opt_all = W.opt_all;
    p->n_window_kf = (int)win.size();
    p->n_landmarks_global = (int)opt_all.size();
    if (W.status != 0) return VX_OK;
    p->status = 0;

    auto owned = [&](int l) {
        return p->shard_count <= 1 ||
               (int)(splitmix64(m->lm_id[l]) % (uint64_t)p->shard_count) == p->shard_rank;
    };
    // local landmark slots: owned optimisable first, then owned fixed ones met in the pose stage
    std::vector<int> slot_of(m->n_lm, -1);
    p->lm_map_idx.clear();
    for (int l : opt_all)
        if (owned(l)) {
            slot_of[l] = (int)p->lm_map_idx.size();
            p->lm_map_idx.push_back(l);
        }
    p->n_opt = (int)p->lm_map_idx.size();

    // ---- keyframe table + pose-stage CSR (local_ba.cpp:116-161)
    const int nk = (int)win.size();
    p->n_kf = nk;
    p->kf_map_idx = win;
    std::vector<double> pose0((size_t)nk * 8, 0.0), intr((size_t)nk * 4, 0.0);
    std::vector<double2> puv;
    std::vector<int> plm, kf_obs_ptr(nk + 1, 0), kf_flags(nk, 0);
    for (int r = 0; r < nk; ++r) {
        const int k = win[r];
        for (int j = 0; j < 7; ++j) pose0[8 * r + j] = m->kf_pose[7 * k + j];
        for (int j = 0; j < 4; ++j) intr[4 * r + j] = m->kf_intr[4 * k + j];
        kf_flags[r] = m->kf_has_cam[k] ? 1 : 0;
        kf_obs_ptr[r] = (int)puv.size();
        if (!m->kf_has_cam[k]) continue;
        for (int64_t f = m->kf_feat_ptr[k]; f < m->kf_feat_ptr[k + 1]; ++f) {
            const uint8_t fl = m->feat_flags[f];
            if (!(fl & 1) || (fl & 2)) continue;
            const int l_found = lm_by_id.get(m->feat_lm_id[f]);
            if (l_found < 0) continue;
            const int l = l_found;
            if (m->lm_bad[l] || !owned(l)) continue;
            if (slot_of[l] < 0) {
                slot_of[l] = (int)p->lm_map_idx.size();
                p->lm_map_idx.push_back(l);
            }
            puv.push_back(make_double2(m->feat_uv[2 * f], m->feat_uv[2 * f + 1]));
            plm.push_back(slot_of[l]);
        }
    }
    kf_obs_ptr[nk] = (int)puv.size();
    // workgroups per keyframe: about one observation per thread, from counts every shard sees
    // alike (the window's landmark features before sharding), so the all-reduced partial layout
    // is the same on every rank
    {
        int64_t mx = 0;
        for (int k : win)
            if (m->kf_has_cam[k]) {
                int64_t n = 0;
                for (int64_t f = m->kf_feat_ptr[k]; f < m->kf_feat_ptr[k + 1]; ++f) n += m->feat_flags[f] & 1;
                mx = std::max(mx, n);
            }
        p->n_split = ba_split(mx, p->shard_count);
    }
    p->n_lm = (int)p->lm_map_idx.size();
    p->n_pose_obs = (int64_t)puv.size();
    std::vector<double> lm0((size_t)std::max(p->n_lm, 1) * 4, 0.0);
    for (int s = 0; s < p->n_lm; ++s)
        for (int j = 0; j < 3; ++j) lm0[4 * s + j] = m->lm_pos[3 * p->lm_map_idx[s] + j];

    // ---- landmark-stage CSR (local_ba.cpp:186-204)
    std::vector<int> lptr(p->n_opt + 1, 0), lkf, llm;
    std::vector<double2> luv;
    for (int s = 0; s < p->n_opt; ++s) {
        const int l = p->lm_map_idx[s];
        for (int64_t ob = m->lm_obs_ptr[l]; ob < m->lm_obs_ptr[l + 1]; ++ob) {
            auto it = win_row.find(m->obs_kf_id[ob]);
            if (it == win_row.end()) continue;
            const int r = it->second;
            const int k = win[r];
            if (!m->kf_has_cam[k]) continue;
            const uint64_t fi = m->obs_feat_idx[ob];
            const int64_t nf = m->kf_feat_ptr[k + 1] - m->kf_feat_ptr[k];
            if (fi >= (uint64_t)nf) continue;
            const int64_t f = m->kf_feat_ptr[k] + (int64_t)fi;
            const uint8_t fl = m->feat_flags[f];
            if (!(fl & 1) || (fl & 2) || m->feat_lm_id[f] != m->lm_id[l]) continue;
            lkf.push_back(r);
            llm.push_back(s);
            luv.push_back(make_double2(m->feat_uv[2 * f], m->feat_uv[2 * f + 1]));
        }
        lptr[s + 1] = (int)lkf.size();
    }
    p->n_lm_obs = (int64_t)lkf.size();
    const std::vector<int> blk = pack_lm_blocks(lptr, p->n_opt, &p->max_lm_obs);
    p->n_lm_blocks = (int)blk.size() / 2 - 1;
    if (!device) return VX_OK;

    VX_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = upload(c, p->kf_pose0, pose0))) return rc;
    if ((rc = upload(c, p->kf_intr, intr))) return rc;
    if ((rc = upload(c, p->kf_flags, kf_flags))) return rc;
    if ((rc = upload(c, p->kf_obs_ptr, kf_obs_ptr))) return rc;
    if ((rc = upload(c, p->lm_pos0, lm0))) return rc;
    if ((rc = upload(c, p->pobs_uv, puv))) return rc;
    if ((rc = upload(c, p->pobs_lm, plm))) return rc;
    if ((rc = upload(c, p->lobs_ptr, lptr))) return rc;
    if ((rc = upload(c, p->lobs_kf, lkf))) return rc;
    if ((rc = upload(c, p->lobs_lm, llm))) return rc;
    if ((rc = upload(c, p->lm_blk, blk))) return rc;
    if ((rc = upload(c, p->lobs_uv, luv))) return rc;
    return alloc_run_buffers(c, p);
}

// Kernel set of a run.  Every k_landmark_solve workgroup re-solves all window poses, so that
// redundancy grows as n_kf x workgroups: beyond the measured crossover (scripts/ba_window_sweep.py,
// DESIGN.md §6) the large-window kernels (poses solved once, one extra launch per iteration) are
// faster; they are also the only ones for windows beyond kMaxKfLds keyframes and for a landmark
// with more than kLmBlock observations.  `blocks` / `max_obs` are maxima over every shard of the
// window (all-reduced once for a sharded plan), so all ranks take the same kernels.
bool choose_lds_poses(const vx_ba_plan* p, int blocks, int max_obs) {
    return p->n_kf <= kMaxKfLds && !p->global_poses && (int64_t)p->n_kf * blocks <= 80000 && blocks <= 480 &&
           max_obs <= kLmBlock;
}

size_t landmark_solve_lds(const vx_ba_plan* p) {
    return (size_t)p->n_kf * kLdsStride * sizeof(double) + (size_t)kLmBlock * (9 * sizeof(double) + sizeof(int));
}

int pose_stage(vx_ctx* c, const vx_ba_plan* p, const BAArgs& a, int it) {
    VX_HIP(c, launch(c, kStBaPose, k_pose_kf, dim3(p->n_kf * p->n_split), dim3(kPoseBlock), 0, c->stream, a, it));
    return VX_OK;
}

int landmark_stage(vx_ctx* c, const vx_ba_plan* p, const BAArgs& a, int it, bool lds_poses) {
    if (lds_poses) {
        const size_t lds = landmark_solve_lds(p);
        if (lds > 64 * 1024) {  // up to ~154 KB at kMaxKfLds keyframes (gfx950: 160 KB per workgroup)
            static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_landmark_solve),
                                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            VX_HIP(c, attr);
        }
        VX_HIP(c, launch(c, kStBaLandmark, k_landmark_solve, dim3(p->n_lm_blocks), dim3(kLmBlock), (uint32_t)lds,
                         c->stream, a, it));
    } else {
        ProfScope ps(c, kStBaLandmark);
        hipLaunchKernelGGL(k_pose_solve_g, dim3((p->n_kf + 255) / 256), dim3(256), 0, c->stream, a, it);
        VX_LAUNCH_CHECK(c, "k_pose_solve_g");
        hipLaunchKernelGGL(k_landmark, dim3(std::max(1, (p->n_opt + 255) / 256)), dim3(256), 0, c->stream, a, it);
        VX_LAUNCH_CHECK(c, "k_landmark");
    }
    return VX_OK;
}

int reset_if_no_iterations(vx_ctx* c, const vx_ba_plan* p, const BAArgs& a) {
    if (p->opt.max_iterations != 0) return VX_OK;
    ProfScope ps(c, kStBaReset);
    const int n = std::max(p->n_kf * 8, std::max(p->n_lm, 1) * 4);
    hipLaunchKernelGGL(k_ba_reset, dim3((n + 255) / 256), dim3(256), 0, c->stream, a);
    VX_LAUNCH_CHECK(c, "k_ba_reset");
    return VX_OK;
}

#ifndef VX_NO_RCCL
// a sharded plan's kernel choice from the maxima over all ranks (once per plan: one small
// all-reduce and a host synchronisation at its first run)
int shard_kernel_choice(vx_ctx* c, vx_ba_plan* p) {
    if (p->choice_made) return VX_OK;
    const int32_t mine[2] = {p->n_lm_blocks, p->max_lm_obs};
    DevBuf d;
    VX_HIP(c, d.ensure(sizeof mine));
    VX_HIP(c, hipMemcpyAsync(d.p, mine, sizeof mine, hipMemcpyHostToDevice, c->stream));
    ncclResult_t r = ncclAllReduce(d.p, d.p, 2, ncclInt32, ncclMax, c->comm, c->stream);
    if (r != ncclSuccess) return set_error(c, VX_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
    int32_t all[2];
    VX_HIP(c, hipMemcpyAsync(all, d.p, sizeof all, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    p->lds_poses = choose_lds_poses(p, all[0], all[1]);
    p->choice_made = true;
    return VX_OK;
}
#endif

int plan_run(vx_ctx* c, vx_ba_plan* p) {
    if (p->status != 0) {
        p->ran = true;
        return VX_OK;
    }
    const bool sharded = p->shard_count > 1;
    int rc;
    if (sharded) {
#ifndef VX_NO_RCCL
        if (!c->comm || c->nranks != p->shard_count || c->rank != p->shard_rank)
            return set_error(c, VX_ERR_STATE, "sharded plan needs vx_comm_init(%d ranks)", p->shard_count);
        if ((rc = shard_kernel_choice(c, p))) return rc;
#else
        return set_error(c, VX_ERR_COMM, "built without RCCL");
#endif
    } else if (!p->choice_made) {
        p->lds_poses = choose_lds_poses(p, p->n_lm_blocks, p->max_lm_obs);
        p->choice_made = true;
    }
    const BAArgs a = make_args(p);
    if ((rc = reset_if_no_iterations(c, p, a))) return rc;
    for (int it = 0; it < p->opt.max_iterations; ++it) {
        if ((rc = pose_stage(c, p, a, it))) return rc;
#ifndef VX_NO_RCCL
        if (sharded) {
            ProfScope ps(c, kStBaAllreduce);
            ncclResult_t r = ncclAllReduce(p->kf_part.p, p->kf_part.p, (size_t)p->n_kf * p->n_split * kStride, ncclDouble,
                                           ncclSum, c->comm, c->stream);
            if (r != ncclSuccess) return set_error(c, VX_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
        }
#endif
        if ((rc = landmark_stage(c, p, a, it, p->lds_poses))) return rc;
    }
    p->ran = true;
    return VX_OK;
}

// Test hook for the sharded path on one device: the element-wise sum of the shards' partial blocks
// (in rank order) written back to every shard, in place of the per-iteration ncclAllReduce.
constexpr int kMaxEmuShards = 16;
struct PartPtrs {
    double* p[kMaxEmuShards];
};
__global__ void k_sum_parts(PartPtrs parts, int n, long long len) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    double s = parts.p[0][i];
    for (int r = 1; r < n; ++r) s += parts.p[r][i];
    for (int r = 0; r < n; ++r) parts.p[r][i] = s;
}

}  // namespace
}  // namespace vx

using namespace vx;

VX_KT_EXPORT(vx_ktrace_read_ba);

extern "C" {

void vx_ba_default_options(vx_ba_options* o) {
    if (!o) return;
    o->window_size = 5;
    o->max_iterations = 5;
    o->min_pose_observations = 20;
    o->min_point_observations = 2;
    o->huber_delta = 5.0;
    o->max_reproj_error = 5.0;
}

int vx_ba_plan_create(vx_ctx* c, const vx_map_view* m, uint64_t ref, int has_ref, const vx_ba_options* opt,
                      int shard_rank, int shard_count, vx_ba_plan** out) {
    return vx_ba_plan_create_ex(c, m, ref, has_ref, opt, shard_rank, shard_count, 0, out);
}

int vx_ba_plan_create_ex(vx_ctx* c, const vx_map_view* m, uint64_t ref, int has_ref, const vx_ba_options* opt,
                         int shard_rank, int shard_count, int flags, vx_ba_plan** out) {
    if (!c || !out || !opt) return VX_ERR_INVALID;
    *out = nullptr;
    if (opt->max_iterations < 0 || opt->max_iterations > kMaxIter)
        return set_error(c, VX_ERR_INVALID, "max_iterations must be in [0, %d]", kMaxIter);
    if (shard_count < 1 || shard_rank < 0 || shard_rank >= shard_count)
        return set_error(c, VX_ERR_INVALID, "bad shard %d/%d", shard_rank, shard_count);
    auto* p = new vx_ba_plan();
    p->c = c;
    p->opt = *opt;
    p->shard_rank = shard_rank;
    p->shard_count = shard_count;
    p->global_poses = (flags & VX_PLAN_GLOBAL_POSES) != 0;
    const int rc = (flags & VX_PLAN_HOST_BUILD) ? build_plan(c, m, ref, has_ref, p) : build_plan_device(c, m, ref, has_ref, p);
    if (rc) {
        delete p;
        return rc;
    }
    *out = p;
    return VX_OK;
}

int vx_ba_plan_create_dmap(vx_ctx* c, vx_dmap* m, uint64_t ref, int has_ref, const vx_ba_options* opt, int shard_rank,
                           int shard_count, vx_ba_plan** out) {
    if (!c || !out || !opt || !m || m->c != c) return c ? set_error(c, VX_ERR_INVALID, "vx_ba_plan_create_dmap: bad arguments") : VX_ERR_INVALID;
    *out = nullptr;
    if (opt->max_iterations < 0 || opt->max_iterations > kMaxIter)
        return set_error(c, VX_ERR_INVALID, "max_iterations must be in [0, %d]", kMaxIter);
    if (shard_count < 1 || shard_rank < 0 || shard_rank >= shard_count)
        return set_error(c, VX_ERR_INVALID, "bad shard %d/%d", shard_rank, shard_count);
    auto* p = new vx_ba_plan();
    p->c = c;
    p->opt = *opt;
    p->shard_rank = shard_rank;
    p->shard_count = shard_count;
    p->from_dmap = true;
    const int rc = build_plan_dmap(c, m, ref, has_ref, p);
    if (rc) {
        delete p;
        return rc;
    }
    *out = p;
    return VX_OK;
}

int vx_ba_plan_apply_dmap(vx_ctx* c, vx_ba_plan* p, vx_dmap* m) {
    if (!c || !p || !m || p->c != c || m->c != c) return c ? set_error(c, VX_ERR_INVALID, "vx_ba_plan_apply_dmap: bad arguments") : VX_ERR_INVALID;
    if (!p->from_dmap) return set_error(c, VX_ERR_STATE, "plan was not built from a vx_dmap");
    if (!p->ran) return set_error(c, VX_ERR_STATE, "plan not run");
    if (p->status != 0) return VX_OK;
    const int n = std::max(p->n_kf, p->n_opt);
    hipLaunchKernelGGL(k_apply_dmap, dim3((n + 255) / 256), dim3(256), 0, c->stream, (const BAState*)p->state.as<BAState>(),
                       (const double*)p->kf_pose.as<double>(), p->n_kf, (const double*)p->lm_pos.as<double>(), p->n_opt,
                       (const int*)p->kf_map_dev.as<int>(), (const int*)p->lm_map_dev.as<int>(), m->kf_pose.as<double>(),
                       m->lm_pos.as<double>());
    VX_LAUNCH_CHECK(c, "k_apply_dmap");
    return VX_OK;
}

int vx_ba_plan_run_async(vx_ctx* c, vx_ba_plan* p) {
    if (!c || !p || p->c != c) return VX_ERR_INVALID;
    if (p->shard_count > 1 || p->status != 0) return plan_run(c, p);  // (RCCL calls stay outside graphs)
    p->ran = true;
    return graph_run_owned(c, p->graph, [](vx_ctx* cc, void* v) { return plan_run(cc, static_cast<vx_ba_plan*>(v)); }, p);
}

int vx_ba_shard_emulate_run(vx_ctx* c, vx_ba_plan* const* plans, int n) {
    if (!c || !plans || n < 1 || n > kMaxEmuShards) return c ? set_error(c, VX_ERR_INVALID, "vx_ba_shard_emulate_run: bad arguments") : VX_ERR_INVALID;
    vx_ba_plan* p0 = plans[0];
    for (int r = 0; r < n; ++r) {
        const vx_ba_plan* p = plans[r];
        if (!p || p->c != c || p->shard_count != n || p->shard_rank != r)
            return set_error(c, VX_ERR_INVALID, "shard %d: plan of another context or shard layout", r);
        if (p->status != p0->status || p->n_kf != p0->n_kf || p->n_split != p0->n_split ||
            p->opt.max_iterations != p0->opt.max_iterations)
            return set_error(c, VX_ERR_INVALID, "shard %d: plan built from another window", r);
    }
    if (p0->status != 0) {
        for (int r = 0; r < n; ++r) plans[r]->ran = true;
        return VX_OK;
    }
    // the kernel choice every rank would make from the all-reduced maxima
    int blocks = 0, max_obs = 0;
    for (int r = 0; r < n; ++r) {
        blocks = std::max(blocks, plans[r]->n_lm_blocks);
        max_obs = std::max(max_obs, plans[r]->max_lm_obs);
    }
    PartPtrs parts{};
    std::vector<BAArgs> args(n);
    for (int r = 0; r < n; ++r) {
        plans[r]->lds_poses = choose_lds_poses(plans[r], blocks, max_obs);
        plans[r]->choice_made = true;
        parts.p[r] = plans[r]->kf_part.as<double>();
        args[r] = make_args(plans[r]);
    }
    const long long len = (long long)p0->n_kf * p0->n_split * kStride;
    int rc;
    for (int r = 0; r < n; ++r)
        if ((rc = reset_if_no_iterations(c, plans[r], args[r]))) return rc;
    for (int it = 0; it < p0->opt.max_iterations; ++it) {
        for (int r = 0; r < n; ++r)
            if ((rc = pose_stage(c, plans[r], args[r], it))) return rc;
        hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, c->stream, parts, n, len);
        VX_LAUNCH_CHECK(c, "k_sum_parts");
        for (int r = 0; r < n; ++r)
            if ((rc = landmark_stage(c, plans[r], args[r], it, plans[r]->lds_poses))) return rc;
    }
    for (int r = 0; r < n; ++r) plans[r]->ran = true;
    return VX_OK;
}

int vx_ba_plan_fetch(vx_ctx* c, vx_ba_plan* p, vx_map_view* m, vx_ba_stats* st) {
    if (!c || !p || p->c != c) return VX_ERR_INVALID;
    if (!p->ran) return set_error(c, VX_ERR_STATE, "plan not run");
    if (m && p->from_dmap) return set_error(c, VX_ERR_STATE, "dmap plan: scatter with vx_ba_plan_apply_dmap");
    vx_ba_stats s{};
    s.gate_margin = -1.0;
    s.status = p->status;
    s.n_window_kf = p->n_window_kf;
    s.n_landmarks = p->n_landmarks_global;
    if (p->status == 0) {
        BAState hs;
        std::vector<double> pose((size_t)p->n_kf * 8), lm((size_t)std::max(p->n_opt, 1) * 4);
        VX_HIP(c, hipMemcpyAsync(&hs, p->state.p, sizeof hs, hipMemcpyDeviceToHost, c->stream));
        VX_HIP(c, hipStreamSynchronize(c->stream));
        // the poses of the last iteration run are in ping-pong buffer (iterations & 1)
        const double* fin = p->kf_pose.as<double>() + (size_t)(hs.iterations & 1) * p->n_kf * 8;
        VX_HIP(c, hipMemcpyAsync(pose.data(), fin, pose.size() * sizeof(double), hipMemcpyDeviceToHost,
                                 c->stream));
        if (p->n_opt > 0)
            VX_HIP(c, hipMemcpyAsync(lm.data(), p->lm_pos.p, (size_t)p->n_opt * 4 * sizeof(double),
                                     hipMemcpyDeviceToHost, c->stream));
        VX_HIP(c, hipStreamSynchronize(c->stream));
        if (c->prof) prof_collect(c);
        s.iterations = hs.iterations;
        for (int i = 0; i < 16; ++i) {
            s.cost[i] = hs.cost[i];
            s.obs[i] = hs.obs[i];
        }
        if (m) {
            for (int r = 0; r < p->n_kf; ++r)
                for (int j = 0; j < 7; ++j) m->kf_pose[7 * p->kf_map_idx[r] + j] = pose[8 * r + j];
            for (int sl = 0; sl < p->n_opt; ++sl)
                for (int j = 0; j < 3; ++j) m->lm_pos[3 * p->lm_map_idx[sl] + j] = lm[4 * sl + j];
        }
    }
    if (st) *st = s;
    return VX_OK;
}

void vx_ba_plan_destroy(vx_ba_plan* p) {
    delete p;
}

int vx_ba_plan_inspect(const vx_map_view* m, uint64_t ref, int has_ref, const vx_ba_options* opt, int shard_rank,
                       int shard_count, int64_t* out8, int32_t* lm_map_idx, int cap_lm, int32_t* kf_map_idx,
                       int cap_kf) {
    if (!opt || !out8 || shard_count < 1 || shard_rank < 0 || shard_rank >= shard_count) return VX_ERR_INVALID;
    vx_ba_plan p;
    p.opt = *opt;
    p.shard_rank = shard_rank;
    p.shard_count = shard_count;
    const int rc = build_plan(nullptr, m, ref, has_ref, &p, false);
    if (rc) return rc;
    const int64_t v[8] = {p.status, p.n_window_kf, p.n_landmarks_global, p.n_kf, p.n_opt, p.n_lm, p.n_pose_obs,
                          p.n_lm_obs};
    for (int i = 0; i < 8; ++i) out8[i] = v[i];
    if (lm_map_idx) {
        if ((int)p.lm_map_idx.size() > cap_lm) return VX_ERR_CAPACITY;
        for (size_t i = 0; i < p.lm_map_idx.size(); ++i) lm_map_idx[i] = p.lm_map_idx[i];
    }
    if (kf_map_idx) {
        if ((int)p.kf_map_idx.size() > cap_kf) return VX_ERR_CAPACITY;
        for (size_t i = 0; i < p.kf_map_idx.size(); ++i) kf_map_idx[i] = p.kf_map_idx[i];
    }
    return VX_OK;
}

uint32_t vx_ba_shard_of(uint64_t lm_id, int shard_count) {
    return shard_count <= 1 ? 0u : (uint32_t)(vx::ba::splitmix64(lm_id) % (uint64_t)shard_count);
}

int vx_ba_plan_info(const vx_ba_plan* p, int64_t* out8) {
    if (!p || !out8) return VX_ERR_INVALID;
    const int64_t v[8] = {p->n_kf, p->n_lm, p->n_pose_obs, p->n_lm_obs, p->n_opt, p->n_split, p->n_lm_blocks,
                          p->max_lm_obs};
    for (int i = 0; i < 8; ++i) out8[i] = v[i];
    return VX_OK;
}

int vx_ba_optimize_map(vx_ctx* c, vx_map_view* m, uint64_t ref, int has_ref, const vx_ba_options* opt,
                       vx_ba_stats* st) {
    vx_ba_plan* p = nullptr;
    int rc = vx_ba_plan_create(c, m, ref, has_ref, opt, 0, 1, &p);
    if (rc) return rc;
    rc = vx_ba_plan_run_async(c, p);
    if (!rc) rc = vx_ba_plan_fetch(c, p, m, st);
    (void)hipStreamSynchronize(c->stream);
    vx_ba_plan_destroy(p);
    return rc;
}

}  // extern "C"
