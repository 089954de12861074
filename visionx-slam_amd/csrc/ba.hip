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
#include <cstddef>
#include <cstdlib>
#include <chrono>
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
constexpr int kStride = kBaStride;  // doubles per keyframe block in global memory
// LDS slot stride of k_landmark_solve: 33, not 32 doubles — a 256-B stride is one full turn of the
// 64 four-byte LDS banks, so lanes reading different keyframes' slots would all hit one bank
constexpr int kLdsStride = 33;
constexpr int kMaxIter = 64;
// keyframes whose LDS slots fit k_landmark_solve: 448 * 33 * 8 B + kLmBlock * (9 * 8 + 4) B =
// 157,184 B of gfx950's 160 KB per workgroup
constexpr int kMaxKfLds = kBaMaxKfLds;
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
    int fault;                 // k_ba_win: a bounded wait ran out (the run is void; fetch re-runs it)
    double last_cost;
    double cost[16];
    int obs[16];
};

struct BAArgs {
    int n_kf, n_opt, n_lm, pad0;
    int min_pose_obs, min_point_obs, max_iter, n_split;
    double huber, max_err;
    double huber2, max_err2;     // squared thresholds (gates on |e|^2)
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
    // resident one-call build (ba_lean.hip): counts known only on the device — {n_opt, n_lm, landmark
    // workgroups, status (1: no optimisable landmark, nothing runs), ...}; null for built plans
    const int* dyn;
};

// A lean plan's counts from the device (the launch grid is a capacity bound; surplus workgroups of
// the landmark stage exit); false when nothing runs (no optimisable landmark, local_ba.cpp:106-108)
__device__ __forceinline__ bool dyn_counts(BAArgs& a) {
    if (!a.dyn) return true;
    if (a.dyn[kDynStatus]) return false;
    a.n_opt = a.dyn[kDynNOpt];
    a.n_lm = a.dyn[kDynNLm];
    return true;
}


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

__device__ __forceinline__ int mbcnt_lo_hi(unsigned long long m) {  // lanes below this one in m
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// Camera-frame point of pose (R, t) (T_cw * p, projection.h:16): R p + t as three FMA chains (the
// rotation matrix of the pose's quaternion, Eigen toRotationMatrix, instead of Eigen's quaternion
// _transformVector: the same map up to rounding, a third of the dependent depth).
__device__ __forceinline__ D3 rt_apply(const double* R, const double* t, D3 p) {
    return {fma(R[2], p.z, fma(R[1], p.y, fma(R[0], p.x, t[0]))), fma(R[5], p.z, fma(R[4], p.y, fma(R[3], p.x, t[1]))),
            fma(R[8], p.z, fma(R[7], p.y, fma(R[6], p.x, t[2])))};
}

// One pose-stage observation (local_ba.cpp:131-159) against pose T (rotation R) / intrinsics C,
// added to the 29 running terms v (21 H upper, 6 b, cost, count): projection with the z > 1e-6
// check, the gate, the Huber weight and the 2x6 PoseJacobian.  The gate and the Huber switch compare
// |e|^2 with max_reproj_error^2 / huber_delta^2, so 1 / |e| (v_rsq) is only evaluated for
// observations beyond huber_delta; |e| > max_err <=> |e|^2 > max_err^2 up to rounding at the
// boundary (the parity tests keep inputs away from it).
template <bool kFma = true>
__device__ __forceinline__ void pose_obs_accum(const BAArgs& a, const double* T, const double* R, const double* C,
                                               D3 Pw, double2 uv, double* v, bool valid = true) {
    // kFma: branch-free — a rejected observation (invalid lane, behind the camera, beyond the gate)
    // gets weight 0 with finite stand-ins (z = 1), so its terms are exactly +0.0 and the count is not
    // raised (early returns made the running terms a control-flow merge: 27 register moves per
    // observation in the pose-stage loop)
    const double fx = C[0], fy = C[1];
    if constexpr (!kFma) {
        // the round-1 form with early returns, the quaternion rotation, |e| by v_rsq and products
        // then sums: fewer live registers (the 1024-thread kernel's 128-VGPR budget)
        if (!valid) return;
        const D3 pc = se3_apply(T, Pw);
        if (!(pc.z > 1e-6)) return;
        const double inv_z = frcp(pc.z);
        const double x = pc.x * inv_z, y = pc.y * inv_z;
        const double e0 = uv.x - (fx * x + C[2]);
        const double e1 = uv.y - (fy * y + C[3]);
        const double e2 = e0 * e0 + e1 * e1;
        const double re = e2 > 0.0 ? frsq(e2) : 0.0;
        const double en = e2 * re;
        if (en > a.max_err) return;
        const double w = en <= a.huber ? 1.0 : a.huber * re;
        const double jp0 = fx * inv_z, jp2 = -jp0 * x, jp4 = fy * inv_z, jp5 = -jp4 * y;
        const double J0[6] = {jp0, 0.0, jp2, jp2 * pc.y, fma(jp0, pc.z, -jp2 * pc.x), -jp0 * pc.y};
        const double J1[6] = {0.0, jp4, jp5, fma(jp5, pc.y, -jp4 * pc.z), -jp5 * pc.x, jp4 * pc.x};
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
        v[27] += w * e2;
        v[28] += 1.0;
        return;
    }
    const D3 pc = rt_apply(R, T + 4, Pw);
    const bool front = pc.z > 1e-6;
    const double inv_z = frcp(front ? pc.z : 1.0);
    const double x = pc.x * inv_z, y = pc.y * inv_z;
    const double e0 = uv.x - (fx * x + C[2]);
    const double e1 = uv.y - (fy * y + C[3]);
    const double e2 = e0 * e0 + e1 * e1;
    const bool ok = valid && front && !(e2 > a.max_err2);
    const double w = ok ? (e2 > a.huber2 ? a.huber * frsq(e2) : 1.0) : 0.0;
    const double zz = front ? pc.z : 1.0, xx = front ? pc.x : 0.0, yy = front ? pc.y : 0.0;
    // J = Jp * [I | -hat(pc)] (local_ba.cpp:15-33) with Jp = [[jp0, 0, jp2], [0, jp4, jp5]],
    // written out without its structural zeros (J0[1] = J1[0] = 0)
    const double jp0 = fx * inv_z, jp2 = -jp0 * x, jp4 = fy * inv_z, jp5 = -jp4 * y;
    const double J0[6] = {jp0, 0.0, jp2, jp2 * yy, fma(jp0, zz, -jp2 * xx), -jp0 * yy};
    const double J1[6] = {0.0, jp4, jp5, fma(jp5, yy, -jp4 * zz), -jp5 * xx, jp4 * xx};
    // w J^T J, -w J^T e and w |e|^2 accumulated as FMA chains (the FP64 issue rate bounds this loop,
    // ~2 FMAs per term instead of 2 products and 2 sums)
    double wJ0[6], wJ1[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        wJ0[r] = w * J0[r];
        wJ1[r] = w * J1[r];
    }
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) {
            const bool u0 = r != 1 && c != 1, u1 = r != 0 && c != 0;  // compile-time after unroll
            double acc = v[hidx(r, c)];
            if (u0) acc = fma(wJ0[r], J0[c], acc);
            if (u1) acc = fma(wJ1[r], J1[c], acc);
            v[hidx(r, c)] = acc;
        }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        double acc = v[21 + r];
        if (r != 1) acc = fma(-wJ0[r], e0, acc);
        if (r != 0) acc = fma(-wJ1[r], e1, acc);
        v[21 + r] = acc;
    }
    v[27] = fma(w, e2, v[27]);
    v[28] += ok ? 1.0 : 0.0;
}

// Pose stage (local_ba.cpp:116-161): n_split workgroups per keyframe, each over a contiguous
// slice of the keyframe's observations.  Each thread accumulates the 29 terms of its observations
// (strided) in registers; a fixed-order wave butterfly + LDS tree reduces them into the slice's
// partial block kf_part[k * n_split + slice].  Partials are summed later in slice order, so the
// result is deterministic (and identical on every rank after the sharded all-reduce).
__global__ __launch_bounds__(kPoseBlock) void k_pose_kf(BAArgs a0, int it) {
    BAArgs a = a0;
    if (!dyn_counts(a)) return;
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
    double T[8], C[4], R[9];
#pragma unroll
    for (int j = 0; j < 8; ++j) T[j] = Tin[8 * k + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) C[j] = a.kf_intr[4 * k + j];
    rot_from_quat(T, R);
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
        pose_obs_accum(a, T, R, C, Pw, uv, v);
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
template <bool kFma = true>
__device__ __forceinline__ bool obs_terms(const BAArgs& a, D3 P, int k, double2 uv, const double* T0, int tst,
                                          const double* R0, int rst, const double* C0, int cst, double* h) {
    const double* T = T0 + (long long)tst * k;
    const double* C = C0 + (long long)cst * k;
    const double* R = R0 + (long long)rst * k;
    const D3 pc = kFma ? rt_apply(R, T + 4, P) : se3_apply(T, P);
    const bool front = pc.z > 1e-6;
    const double inv_z = frcp(pc.z);
    const double x = pc.x * inv_z, y = pc.y * inv_z;
    const double fx = C[0], fy = C[1];
    const double e0 = uv.x - (fx * x + C[2]);
    const double e1 = uv.y - (fy * y + C[3]);
    const double e2 = e0 * e0 + e1 * e1;
    const bool ok = front && !(e2 > a.max_err2);  // (squared gate, see pose_obs_accum)
    double w = 1.0;
    if (e2 > a.huber2) w = a.huber * frsq(e2);
    const double jp0 = fx * inv_z, jp2 = -jp0 * x, jp4 = fy * inv_z, jp5 = -jp4 * y;
    // J = Jp * R with Jp's structural zeros dropped (local_ba.cpp:219-221); the 9 terms as FMAs with
    // w folded into one factor (a gated-out observation gets w = 0: its terms are exactly +0.0 as
    // long as J and e are finite, and they are selected to 0 below regardless)
    if constexpr (!kFma) {
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
    double J0[3], J1[3], wJ0[3], wJ1[3];
    const double wv = ok ? w : 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        J0[c] = fma(jp0, R[c], jp2 * R[6 + c]);
        J1[c] = fma(jp4, R[3 + c], jp5 * R[6 + c]);
        wJ0[c] = wv * J0[c];
        wJ1[c] = wv * J1[c];
    }
    h[0] = fma(wJ0[0], J0[0], wJ1[0] * J1[0]);
    h[1] = fma(wJ0[0], J0[1], wJ1[0] * J1[1]);
    h[2] = fma(wJ0[0], J0[2], wJ1[0] * J1[2]);
    h[3] = fma(wJ0[1], J0[1], wJ1[1] * J1[1]);
    h[4] = fma(wJ0[1], J0[2], wJ1[1] * J1[2]);
    h[5] = fma(wJ0[2], J0[2], wJ1[2] * J1[2]);
    h[6] = fma(-wJ0[0], e0, -wJ1[0] * e1);
    h[7] = fma(-wJ0[1], e0, -wJ1[1] * e1);
    h[8] = fma(-wJ0[2], e0, -wJ1[2] * e1);
#pragma unroll
    for (int j = 0; j < 9; ++j) h[j] = ok ? h[j] : 0.0;
    return ok;
}

// Landmark update from its summed terms (local_ba.cpp:228-237): skipped below min_point_obs or
// for a non-finite step; the position is written either way (iteration 0 reads lm_pos0).
__device__ __forceinline__ D3 lm_update(const BAArgs& a, int l, D3 P, const double* h, int obs) {
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
    return out;
}

// Pose solve of every window keyframe (redundantly in each workgroup) + landmark stage, one launch.
// Workgroup b covers the whole landmarks [lm_blk[b], lm_blk[b+1]) (at most kLmBlock landmarks
// and kLmBlock observations, packed on the host).  Thread t projects observation o0 + t and
// leaves its 9 terms in LDS; the thread owning landmark l0 + t then sums its observations' terms
// in CSR order (the order of the per-landmark loop, local_ba.cpp:186) and solves the 3x3.
// Every load of the landmark stage is issued first, so it lands during the combine and solve.
// LDS: one kLdsStride-double slot per keyframe (combined normal equations S, then T 8 | R 9 | C 4) and
// 9 x kLmBlock observation terms.
__global__ __launch_bounds__(kLmBlock) void k_landmark_solve(BAArgs a0, int it) {
    BAArgs a = a0;
    if (!dyn_counts(a) || (a.dyn && (int)blockIdx.x >= a.dyn[kDynBlocks])) return;
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

// ------------------------------------------------------------------ fused path: one launch per iteration
// k_ba_iter(it) = combine + pose solve of iteration it, landmark stage of it, pose stage of it + 1.
// Workgroups own whole landmarks in keyframe-locality order (plan: build_fused), so each needs the
// poses of only the few keyframes its observations touch (kent: at most kFK entries).  After its
// landmark stage a workgroup holds the iteration's poses (LDS) and its landmarks' new positions
// (LDS), which is everything the next iteration's pose stage needs for the pose observations of
// those landmarks (local_ba.cpp:131-159 at it + 1): it forms their 29 terms per keyframe (one wave
// per keyframe entry, halving butterfly) into that keyframe's partial slot.  The next launch sums a
// keyframe's slots in slot order — the same sum in every workgroup that needs the pose, so the
// redundant solves agree bitwise — and every keyframe's pose is published by exactly one owner.
// Pose observations of fixed landmarks (not optimised: positions constant) go to the owner of their
// keyframe.  The prologue launch (kPro) forms iteration 0's pose stage from the initial state.
constexpr int kFK = kBaFusedK;
// Threads per fused workgroup (= its landmark-stage observation / landmark capacity): 512, or 1024
// for windows whose 512-thread packing needs more workgroups than the device has CUs (fewer,
// larger workgroups: shorter per-keyframe slot lists; measured).
constexpr int kFTSmall = kBaFTSmall, kFTLarge = kBaFTLarge, kFTNarrow = kBaFTNarrow;

// Fused layout (ba.hip build_fused).  Per workgroup b: landmarks and landmark-stage observations at
// the fixed bases b * kFT (padded), so their loads do not wait for the workgroup table; keyframe
// entries at b * kFK; pose-stage observations in wave-major order — wave w takes entries w, w + kFW,
// ..., each entry's observations start on a 64-aligned index (lane l of round r reads wstart + 64 r
// + l), with fixed landmarks' positions stored in the observation record.
struct FusedArgs {
    const int4* blk;        // 1 + kFW / 2 per workgroup: {landmarks, landmark-stage observations,
                            // keyframe entries, 0}, then {wstart, rounds} per wave
    const int* lm_slot;     // [b * kFT + t] landmark slot (padding: slot 0)
    const int2* lm_run;     // [b * kFT + t] its landmark-stage observations [r0, r1) (workgroup-local)
    const double2* lobs_uv; // [b * kFT + t]
    const int4* lobs_rec;   // [b * kFT + t] {keyframe entry, workgroup-local landmark, slot, 0}
    const int4* kent;       // 2 per entry, kFK entries per workgroup: {row | owner << 30, or -1; slots of
                            // the row; pose observations [start, end)}, {partial slot or -1, 0, 0, 0}
    const double2* pobs_uv;
    const double4* pobs_p;  // {x, y, z, code}: code >= 0 workgroup-local landmark (position from LDS),
                            // code < 0 a fixed landmark at (x, y, z)
    double* part;           // 2 x n_kf x maxl partial blocks of 32 doubles (row-major by keyframe): the
                            // pose stage of iteration i fills buffer i & 1 (a launch reads one buffer
                            // and writes the other, so no workgroup reads what another overwrites)
    int maxl, n_part;
    const double* rowpart;  // sharded plans: per keyframe row the partial slots summed (k_row_sum) and
                            // all-reduced over the ranks; the combine and the stop rule read it instead
    double4* lpos;          // [b * kFT + t] the workgroup's landmark positions in fused order (each read
                            // and rewritten by its owning thread only; the prologue fills them)
    double2* costpart;      // 2 x n_part: each partial slot's {cost, observations} (terms 27, 28) again,
                            // compact, for the stop rule's totals (parity as part)
    int stop_b;             // the workgroup that runs the stop rule (the lightest pose stage, plan time)
    double* epose;          // [(b * kFK + j) * 16] the workgroup's copy of entry j's pose T 8 | C 4 | flags:
                            // every workgroup solving the entry computes the same pose, so each keeps
                            // its own and reads it back at a fixed address (no keyframe-row indirection)
    // Row sums by float atomics (unsharded plans; the default, $VX_BA_ATOMIC_ROWS=0 for slots):
    // launch it >= 0 adds its pose-stage partials (iteration it + 1) straight into per-row sums
    // arow[it % 3] (n_kf x kStride, float atomics executed at the memory side) instead of partial
    // slots, so the next launch combines ONE row per entry instead of re-summing the row's maxl slots
    // (sum order = arrival order: results agree to rounding, not bitwise, run to run; every workgroup
    // of a launch still reads the same row, so the redundant pose solves agree bitwise).  Launch it
    // zeroes arow[(it + 1) % 3], the buffer launch it + 1 accumulates into (last read by launch
    // it - 1).  With apro (plans of >= 2 iterations) the prologue accumulates into arow[3], which
    // launch 0 reads and the run's last launch zeroes for the next run (the plan build zeroes it
    // first); without it the prologue writes slots, which launch 0 combines.
    double* arow;
    int n_kf, apro;
    int drow;  // rows read by the entries' own threads, no combine phase ($VX_BA_DROW=0: the combine)
    int padskip;  // no loads for padding rows / lanes ($VX_BA_PADSKIP=0: every row and lane loads)
};

// the arow buffer launch `it` reads (combine), accumulates into (pose stage of it + 1) and zeroes
__device__ __forceinline__ int arow_rd(int it) { return it == 0 ? 3 : (it - 1) % 3; }
__device__ __forceinline__ int arow_wr(bool pro, int it) { return pro ? 3 : it % 3; }
__device__ __forceinline__ int arow_zero(bool pro, int it) { return pro ? 0 : (it + 1) % 3; }

// LDS layout of k_ba_iter (dynamic): kFK keyframe slots (S, then T 8 | R 9 | C 4), 9 x kFT
// observation terms, kFT counted flags, 3 x kFT landmark positions, the block-0 totals (the entry's
// loaded state stays in its solving thread's registers)
constexpr size_t fused_lds(int ft) {
    return (size_t)kFK * kLdsStride * sizeof(double) + (size_t)9 * ft * sizeof(double) +
           (size_t)ft * sizeof(int) + (size_t)3 * ft * sizeof(double) + (size_t)2 * (ft / 64) * sizeof(double);
}
static_assert(fused_lds(kFTLarge) <= 160 * 1024, "k_ba_iter LDS exceeds gfx950's 160 KB per workgroup");
// compacted pose stage (kCmp): per wave a ring of kQ accepted observations, kQRec doubles each
constexpr int kQ = 128, kQRec = 8;
constexpr size_t fused_lds_cmp(int ft) { return fused_lds(ft) + (size_t)(ft / 64) * kQ * kQRec * sizeof(double); }
static_assert(fused_lds_cmp(kFTSmall) <= 160 * 1024, "k_ba_iter (compacted) LDS exceeds 160 KB");

// The Jacobian / normal-equation half of pose_obs_accum for one accepted observation given its
// camera-frame point (xx, yy, zz), 1 / z, residual and weight (the gate already passed): the same
// FMA chains as the branch-free form (terms 0-26; cost and count are added at the gate).
__device__ __forceinline__ void pose_obs_terms(const double* C, double xx, double yy, double zz, double inv_z,
                                               double e0, double e1, double w, double* v) {
    const double fx = C[0], fy = C[1];
    const double x = xx * inv_z, y = yy * inv_z;
    const double jp0 = fx * inv_z, jp2 = -jp0 * x, jp4 = fy * inv_z, jp5 = -jp4 * y;
    const double J0[6] = {jp0, 0.0, jp2, jp2 * yy, fma(jp0, zz, -jp2 * xx), -jp0 * yy};
    const double J1[6] = {0.0, jp4, jp5, fma(jp5, yy, -jp4 * zz), -jp5 * xx, jp4 * xx};
    double wJ0[6], wJ1[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        wJ0[r] = w * J0[r];
        wJ1[r] = w * J1[r];
    }
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) {
            const bool u0 = r != 1 && c != 1, u1 = r != 0 && c != 0;
            double acc = v[hidx(r, c)];
            if (u0) acc = fma(wJ0[r], J0[c], acc);
            if (u1) acc = fma(wJ1[r], J1[c], acc);
            v[hidx(r, c)] = acc;
        }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        double acc = v[21 + r];
        if (r != 1) acc = fma(-wJ0[r], e0, acc);
        if (r != 0) acc = fma(-wJ1[r], e1, acc);
        v[21 + r] = acc;
    }
}

// trace build: phases of the it == 1 launch only (the last launch of a run has no pose stage)
#define FKT(slot)                              \
    do {                                       \
        if (!kPro && it == 1) VX_KT(slot);     \
    } while (0)

typedef int si4 __attribute__((ext_vector_type(4)));  // (an SGPR quad for the scalar loads below)

template <bool kPro, int kFT, bool kCmp = false>
__global__ __launch_bounds__(kFT) void k_ba_iter(BAArgs a, FusedArgs f, int it) {
    constexpr int kFW = kFT / 64;  // waves per workgroup
    // per-entry pose copies (f.epose) and fused-order landmark positions (f.lpos) in the 512-thread
    // kernel; the 1024-thread one (128 VGPRs) keeps the indirect reads of the published poses and
    // positions, whose longer live ranges it cannot afford
    constexpr bool kEcopy = kFT <= kFTSmall;
    // highest wave priority: in the pipeline, extraction waves share these SIMDs, and the launch's
    // dependent FP64 chains are what the frame waits for (instruction-issue arbitration prefers
    // higher-priority waves; the co-resident waves fill the gaps of the chains)
    __builtin_amdgcn_s_setprio(3);
    // row sums by atomics: the 256 / 512-thread layouts only (the host never enables them for the
    // 1024-thread one, whose 128 VGPRs leave no room: compiled out there)
    double* const arow = kFT <= kFTSmall ? f.arow : nullptr;
    if (!kPro && arow && f.apro && it == a.max_iter - 1) {  // (arow[3] for the next run's prologue)
        double* z = arow + (size_t)3 * f.n_kf * kStride;
        for (int i = blockIdx.x * kFT + threadIdx.x; i < f.n_kf * kStride; i += (int)gridDim.x * kFT) z[i] = 0.0;
    }
    // (an iteration after the stop returns before its first write, below: its loads are issued
    // first so the flag's latency overlaps theirs)
    if (!kEcopy && !kPro && it > 0 && !a.state->active[it]) return;
    // (a relaxed atomic load is issued here with the other loads — a plain one was sunk to its use —
    // and waited for only at its use below)
    const int act = kPro ? 1 : __hip_atomic_load(&a.state->active[it], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    extern __shared__ __attribute__((aligned(16))) double fl[];
    // the workgroup's keyframe entry records, staged once: the combine and the pose stage read them
    // from LDS instead of issuing a dependent global load at the start of each
    __shared__ int4 s_ke[kFK];
    __shared__ int s_kd[kFK];
    double* kslot = fl;                                  // [kFK][kLdsStride]
    double* terms = kslot + kFK * kLdsStride;            // [9][kFT]
    int* tcount = reinterpret_cast<int*>(terms + 9 * kFT);
    double* lpos = terms + 9 * kFT + kFT / 2;            // [kFT][3] (after kFT ints)
    double* red = lpos + 3 * kFT;                        // [2][kFW]
    double* qbuf = red + 2 * kFW;                        // (kCmp) [kFW][kQ][kQRec] accepted observations
    const int tid = threadIdx.x, b = blockIdx.x, wv = tid >> 6, lane = tid & 63;
    const size_t base = (size_t)b * kFT;
    const int4* KE = f.kent + (size_t)b * kFK * 2;
    const double* part_in = f.part + (size_t)(it & 1) * f.n_part * kStride;  // (unused by kPro)
    double* part_out = f.part + (size_t)((it + 1) & 1) * f.n_part * kStride;
    FKT(0);
    // ---- every load the launch needs, issued up front (at most two dependent levels); values
    // needed only after the first barrier are parked in LDS, not held in registers.  Issue order
    // matters: `s_waitcnt vmcnt` retires loads in issue order, so a value is waited for together with
    // every load issued before it.  Wave 0's chain is the block record and its entry records, then
    // the rows those name (drow), then the solve: the entry records and copies go right behind the
    // block record, ahead of the landmark loads, and none of their values is used (no wait) before
    // every independent load is in flight.
    // (the block records by scalar loads — plan data no kernel writes — so that waiting for them
    // (lgkmcnt, below) does not wait for the vector loads issued behind them; the compiler keeps
    // them on the vector path, whose in-order vmcnt made the landmark loads wait for the rows)
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    si4 Bv, WBv;
    asm volatile("s_load_dwordx4 %0, %1, 0x0" : "=s"(Bv) : "s"(f.blk + (size_t)b * (1 + kFW / 2)));
    asm volatile("s_load_dwordx4 %0, %1, 0x0" : "=s"(WBv) : "s"(f.blk + (size_t)b * (1 + kFW / 2) + 1 + (wvu >> 1)));
    // (c) the keyframe entry it solves: previous pose, intrinsics, flags (the prologue
    // gathers them by keyframe row into the workgroup's entry copy; later launches read the copy)
    int4 ke = make_int4(-1, 0, 0, 0);
    int kd = -1;
    double ev[13];
    if (tid < kFK) {
        ke = KE[2 * tid];
        kd = KE[2 * tid + 1].x;
        if (!kPro && kEcopy) {
            // (the copy is read whether or not the entry exists — unused entries are valid memory —
            // so the load does not wait for the entry table)
            const double4* E4 = reinterpret_cast<const double4*>(f.epose + ((size_t)b * kFK + tid) * 16);
            const double4 e0 = E4[0], e1 = E4[1], e2 = E4[2];
            ev[0] = e0.x, ev[1] = e0.y, ev[2] = e0.z, ev[3] = e0.w;
            ev[4] = e1.x, ev[5] = e1.y, ev[6] = e1.z, ev[7] = e1.w;
            ev[8] = e2.x, ev[9] = e2.y, ev[10] = e2.z, ev[11] = e2.w;
            ev[12] = reinterpret_cast<const double*>(E4 + 3)[0];
        }
    }
    // (a) this thread's landmark-stage observation (padding rows are valid memory)
    int4 orec = make_int4(0, 0, 0, 0);
    double2 ouv = make_double2(1e300, 1e300);
    if (!kPro) {
        orec = f.lobs_rec[base + tid];
        ouv = f.lobs_uv[base + tid];
    }
    // (c') with the rows summed by atomics the entry's own thread (wave 0) reads its row as soon as its
    // entry record is in and solves without the combine phase or the first barrier: the other waves
    // meet it at the barrier after the solve (round 5: the combine's LDS round trip and two barriers
    // off the launch's path)
    const bool drow = !kPro && f.drow && arow && (it > 0 || f.apro);
    double Sd[kNTerms];
    if (drow && tid < kFK && ke.x >= 0) {
        const double* rp = arow + ((size_t)arow_rd(it) * f.n_kf + (ke.x & 0x3fffffff)) * kStride;
#pragma unroll
        for (int t = 0; t < kNTerms; ++t) Sd[t] = rp[t];
    }
    // (c) the prologue / 1024-thread layout: the entry's state by keyframe row
    if ((kPro || !kEcopy) && tid < kFK && ke.x >= 0) {
        const int row = ke.x & 0x3fffffff;
        const double* Tin = (kPro ? a.kf_pose0 : pose_in(a, it)) + 8 * (size_t)row;
#pragma unroll
        for (int j = 0; j < 8; ++j) ev[j] = Tin[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) ev[8 + j] = a.kf_intr[4 * row + j];
        ev[12] = (double)a.kf_flags[row];
    }
    // (b) the landmark it owns (its position goes to LDS for the observations of the landmark):
    // fused-order copy at a fixed address (the prologue reads the slot's initial position)
    // (iterations of the 512-thread layout: only the workgroup's B.x landmark threads load — the
    // padding rows of the other ~70 % were ~1.8 MB per launch of HBM traffic; the loads wait for B,
    // which the solving wave's row loads outlast anyway.  The prologue keeps them unconditional: its
    // first barrier waits for them.)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(Bv), "+s"(WBv));  // (the block records, above)
    const int4 B = make_int4(Bv.x, Bv.y, Bv.z, Bv.w), WB = make_int4(WBv.x, WBv.y, WBv.z, WBv.w);
    const int wstart = (wvu & 1) ? WB.z : WB.x, wrounds = (wvu & 1) ? WB.w : WB.y;
    const bool lm_load = kPro || !kEcopy || !f.padskip || tid < B.x;
    int lslot = lm_load ? f.lm_slot[base + tid] : 0;
    int2 run = make_int2(0, 0);
    if (!kPro && lm_load) run = f.lm_run[base + tid];
    D3 PL{0.0, 0.0, 0.0};
    if (kPro || !kEcopy) {
        const double* P = kPro ? a.lm_pos0 + 4 * (size_t)lslot : lm_in(a, it, lslot);
        PL = {P[0], P[1], P[2]};
    } else if (lm_load) {
        const double* P = reinterpret_cast<const double*>(f.lpos + base + tid);
        PL = {P[0], P[1], P[2]};
    }
    // (d) this wave's first pose-stage round (round r + 1 is requested when round r is consumed)
    const bool pose_next = kPro || it + 1 < a.max_iter;
    double2 u0 = make_double2(0, 0);
    double4 p0 = make_double4(0, 0, 0, 0);
    if (pose_next && wrounds > 0) {
        u0 = f.pobs_uv[wstart + lane];
        p0 = f.pobs_p[wstart + lane];
    }
    // (the entry's state stays in the solving thread's registers: an LDS copy here would wait for
    // every load issued so far — the waits merge conservatively over the branches above)
    if (tid < kFK && (ke.x >= 0 || (!kPro && kEcopy))) {
        if (kPro && kEcopy) {
            double* E = f.epose + ((size_t)b * kFK + tid) * 16;
#pragma unroll
            for (int j = 0; j < 13; ++j) E[j] = ev[j];
        }
    }
    const int n_lm = B.x, n_ob = B.y, n_ent = B.z;
    const bool has_o = !kPro && tid < n_ob, own = tid < n_lm;
    if (!kPro && it > 0 && !act) return;  // iteration after the stop: no global write
    if (arow) {  // the buffer the NEXT launch accumulates into (see FusedArgs::arow)
        double* z = arow + (size_t)arow_zero(kPro, it) * f.n_kf * kStride;
        for (int i = b * kFT + tid; i < f.n_kf * kStride; i += (int)gridDim.x * kFT) z[i] = 0.0;
    }
    if (kPro && kEcopy) f.lpos[base + tid] = make_double4(PL.x, PL.y, PL.z, 0.0);
    lpos[3 * tid] = PL.x;
    lpos[3 * tid + 1] = PL.y;
    lpos[3 * tid + 2] = PL.z;
    if (tid < kFK) {
        s_ke[tid] = ke;
        s_kd[tid] = kd;
    }
    FKT(1);
    if (!drow) __syncthreads();  // s_ke / s_kd
    if (!kPro) {
        // ---- combine: S of entry j, term t = the row's partial slots summed in slot order
        for (int pr = tid; !drow && pr < n_ent * kNTerms; pr += kFT) {
            const int j = pr / kNTerms, t = pr - j * kNTerms;
            const int4 e = s_ke[j];
            if (e.x < 0) continue;  // a hole in the entry positions
            if (f.rowpart) {  // sharded: the all-reduced row (identical on every rank)
                kslot[j * kLdsStride + t] = f.rowpart[(size_t)(e.x & 0x3fffffff) * kStride + t];
                continue;
            }
            if (arow && (it > 0 || f.apro)) {  // the row summed by the previous launch's atomics
                kslot[j * kLdsStride + t] = arow[((size_t)arow_rd(it) * f.n_kf + (e.x & 0x3fffffff)) * kStride + t];
                continue;
            }
            const double* src = part_in + ((size_t)(e.x & 0x3fffffff) * f.maxl) * kStride + t;
            constexpr int kCB = kFT <= kFTSmall ? 32 : 16;  // slots per batch of loads (one round at C3)
            double acc = 0.0;
            for (int i0 = 0; i0 < e.y; i0 += kCB) {
                double v[kCB];
#pragma unroll
                for (int q = 0; q < kCB; ++q) v[q] = i0 + q < e.y ? src[(size_t)(i0 + q) * kStride] : 0.0;
#pragma unroll
                for (int q = 0; q < kCB; ++q) acc += v[q];  // (+0.0 past the end: exact)
            }
            kslot[j * kLdsStride + t] = acc;
        }
        // ---- stop rule of iteration it (workgroup 0): totals over every partial slot
        if (b == f.stop_b) {
            double tot = 0.0, cnt = 0.0;
            if (f.rowpart || (arow && (it > 0 || f.apro))) {
                const double* rows = f.rowpart ? f.rowpart : arow + (size_t)arow_rd(it) * f.n_kf * kStride;
                for (int q = tid; q < a.n_kf; q += kFT) {
                    tot += rows[(size_t)q * kStride + 27];
                    cnt += rows[(size_t)q * kStride + 28];
                }
            } else {
                const double2* cp = f.costpart + (size_t)(it & 1) * f.n_part;
                for (int q0 = 0; q0 < f.n_part; q0 += 2 * kFT) {  // (two loads in flight per thread)
                    const int q1 = q0 + tid, q2 = q0 + kFT + tid;
                    const double2 c1 = q1 < f.n_part ? cp[q1] : make_double2(0.0, 0.0);
                    const double2 c2 = q2 < f.n_part ? cp[q2] : make_double2(0.0, 0.0);
                    tot += c1.x;
                    cnt += c1.y;
                    tot += c2.x;
                    cnt += c2.y;
                }
            }
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) {
                tot += __shfl_xor(tot, m, 64);
                cnt += __shfl_xor(cnt, m, 64);
            }
            if (lane == 0) {
                red[wv] = tot;
                red[kFW + wv] = cnt;
            }
        }
    }
    if (!drow) __syncthreads();  // (kslot's combined rows, red[])
    FKT(2);
    // ---- pose solve of the entries (local_ba.cpp:163-173); owners publish
    if (ke.x >= 0) {
        double* sl = kslot + tid * kLdsStride;
        double T[8], R[9], C[4];
#pragma unroll
        for (int j = 0; j < 8; ++j) T[j] = ev[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) C[j] = ev[8 + j];
        if (!kPro) {
            double S[kNTerms];
#pragma unroll
            for (int t = 0; t < kNTerms; ++t) S[t] = drow ? Sd[t] : sl[t];
            solve_pose(a, (int)ev[12], S, T, R);
            if (ke.x & (1 << 30)) {
                double* Tout = pose_out(a, it) + 8 * (size_t)(ke.x & 0x3fffffff);
#pragma unroll
                for (int j = 0; j < 8; ++j) Tout[j] = T[j];
            }
            if (kEcopy) {
                double4* E4 = reinterpret_cast<double4*>(f.epose + ((size_t)b * kFK + tid) * 16);
                E4[0] = make_double4(T[0], T[1], T[2], T[3]);
                E4[1] = make_double4(T[4], T[5], T[6], T[7]);
            }
        } else {
            rot_from_quat(T, R);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) sl[j] = T[j];
#pragma unroll
        for (int j = 0; j < 9; ++j) sl[8 + j] = R[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) sl[17 + j] = C[j];
    }
    auto stop_from_red = [&] {
        double tot = 0.0, cnt = 0.0;
        for (int w2 = 0; w2 < kFW; ++w2) {
            tot += red[w2];
            cnt += red[kFW + w2];
        }
        stop_rule(a, it, tot, (int)cnt);
    };
    if (!kPro && !drow && b == f.stop_b && tid == 0) stop_from_red();
    __syncthreads();
    if (drow && b == f.stop_b && tid == 0) stop_from_red();  // (every wave's red[] is in after the barrier)
    FKT(3);
    // ---- landmark stage of iteration it (local_ba.cpp:176-238)
    if (!kPro) {
        double h[9];
        const D3 PO{lpos[3 * orec.y], lpos[3 * orec.y + 1], lpos[3 * orec.y + 2]};
        const bool ok = obs_terms<kFT <= kFTSmall>(a, PO, orec.x, ouv, kslot, kLdsStride, kslot + 8, kLdsStride,
                                                   kslot + 17, kLdsStride, h);
#pragma unroll
        for (int j = 0; j < 9; ++j) terms[j * kFT + tid] = h[j];
        tcount[tid] = (has_o && ok) ? 1 : 0;
        __syncthreads();
        if (own) {
            double hs[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            int obs = 0;
            for (int r = run.x; r < run.y; ++r) {
#pragma unroll
                for (int j = 0; j < 9; ++j) hs[j] += terms[j * kFT + r];
                obs += tcount[r];
            }
            // (lslot made opaque until here: otherwise its address arithmetic is hoisted next to its
            // load, whose wait — vmcnt, in issue order — then holds wave 0 for the rows behind it)
            asm volatile("" : "+v"(lslot));
            PL = lm_update(a, lslot, PL, hs, obs);
            if (kEcopy) f.lpos[base + tid] = make_double4(PL.x, PL.y, PL.z, 0.0);
            lpos[3 * tid] = PL.x;
            lpos[3 * tid + 1] = PL.y;
            lpos[3 * tid + 2] = PL.z;
        }
        __syncthreads();
    }
    FKT(4);
    // ---- pose stage of iteration it + 1: wave wv takes entries wv, wv + kFW, ...
    if (!pose_next) return;
    int r = 0;
    FKT(6);
    for (int j = wv; j < n_ent; j += kFW) {
        const int4 e = s_ke[j];
        const int dst = s_kd[j];
        const int nr = (e.w - e.z + 63) >> 6;
        if (nr == 0) continue;
        const double* T = kslot + j * kLdsStride;
        const double* R = T + 8;
        const double* C = T + 17;
        double v[kStride];
#pragma unroll
        for (int t = 0; t < kStride; ++t) v[t] = 0.0;
        if constexpr (kCmp) {
            // Projection and gate (local_ba.cpp:131-146) for every observation; the Jacobian and
            // normal-equation half (:148-159) only for the accepted ones, 64 at a time from a per-wave
            // ring in LDS: after the first iterations most observations fail the gate (the
            // reference's step sign grows the residuals), so most rounds skip that half.  Accepted
            // observations keep their order within a lane slot only up to the summation order of
            // the terms (the tolerance-level change documented in DESIGN.md §2).
            double* qw = qbuf + (size_t)wv * kQ * kQRec;
            int qh = 0, qn = 0;  // ring head (next write) and queued count (wave-uniform)
            auto drain = [&](int n) {  // terms of the n oldest queued observations
                const int slot = (qh - qn + lane + kQ) & (kQ - 1);
                const double4 r0 = *reinterpret_cast<const double4*>(qw + (size_t)slot * kQRec);
                const double4 r1 = *reinterpret_cast<const double4*>(qw + (size_t)slot * kQRec + 4);
                // lanes past n read stale ring entries (or never-written LDS): finite stand-ins with
                // weight 0, so their terms are exactly +-0.0
                const bool use = lane < n;
                pose_obs_terms(C, use ? r0.x : 0.0, use ? r0.y : 0.0, use ? r0.z : 1.0, use ? r0.w : 1.0,
                               use ? r1.x : 0.0, use ? r1.y : 0.0, use ? r1.z : 0.0, v);
                qn -= n;
            };
            for (int q = 0; q < nr; ++q, ++r) {
                const double2 uv = u0;
                const double4 P4 = p0;
                if (r + 1 < wrounds) {
                    u0 = f.pobs_uv[wstart + 64 * (r + 1) + lane];
                    p0 = f.pobs_p[wstart + 64 * (r + 1) + lane];
                }
                const bool valid = e.z + 64 * q + lane < e.w;
                const int code = (int)P4.w;
                const D3 P = code >= 0 ? D3{lpos[3 * code], lpos[3 * code + 1], lpos[3 * code + 2]} : D3{P4.x, P4.y, P4.z};
                const D3 pc = rt_apply(R, T + 4, P);
                const bool front = pc.z > 1e-6;
                const double inv_z = frcp(front ? pc.z : 1.0);
                const double e0 = uv.x - (C[0] * (pc.x * inv_z) + C[2]);
                const double e1 = uv.y - (C[1] * (pc.y * inv_z) + C[3]);
                const double e2 = e0 * e0 + e1 * e1;
                const bool ok = valid && front && !(e2 > a.max_err2);
                const double w = ok ? (e2 > a.huber2 ? a.huber * frsq(e2) : 1.0) : 0.0;
                v[27] = fma(w, e2, v[27]);
                v[28] += ok ? 1.0 : 0.0;
                const unsigned long long m = __ballot(ok);
                const int slot = ok ? ((qh + mbcnt_lo_hi(m)) & (kQ - 1)) : -1;
                if (ok) {
                    double4* rec = reinterpret_cast<double4*>(qw + (size_t)slot * kQRec);
                    rec[0] = make_double4(pc.x, pc.y, pc.z, inv_z);
                    rec[1] = make_double4(e0, e1, w, 0.0);
                }
                const int na = __popcll(m);
                qh = (qh + na) & (kQ - 1);
                qn += na;
                if (qn >= 64) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    drain(64);
                }
            }
            if (qn > 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                drain(qn);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the ring is reused by the next entry)
            __builtin_amdgcn_wave_barrier();
        } else {
        for (int q = 0; q < nr; ++q, ++r) {
            const double2 uv = u0;
            const double4 P4 = p0;
            if (r + 1 < wrounds) {
                // only the lanes of the next round that hold an observation load (the entries'
                // 64-aligned padding stays in memory): the next round is this entry's or the first
                // of the wave's next entry with rounds
                int lim = f.padskip ? e.w - (e.z + 64 * (q + 1)) : 64;
                if (f.padskip && q + 1 >= nr) {
                    int jn = j + kFW;
                    int4 en = s_ke[jn < kFK ? jn : j];
                    while (jn < n_ent && ((en.w - en.z + 63) >> 6) == 0) {
                        jn += kFW;
                        en = s_ke[jn < kFK ? jn : j];
                    }
                    lim = en.w - en.z;
                }
                if (lane < lim) {
                    u0 = f.pobs_uv[wstart + 64 * (r + 1) + lane];
                    p0 = f.pobs_p[wstart + 64 * (r + 1) + lane];
                } else {
                    u0 = make_double2(0.0, 0.0);
                    p0 = make_double4(0.0, 0.0, 0.0, 0.0);
                }
            }
            const bool valid = e.z + 64 * q + lane < e.w;
            if (kFT <= kFTSmall || valid) {  // (256 / 512: padding lanes run too, weight 0 — no branch)
                const int code = (int)P4.w;
                const D3 P = code >= 0 ? D3{lpos[3 * code], lpos[3 * code + 1], lpos[3 * code + 2]}
                                       : D3{P4.x, P4.y, P4.z};
                pose_obs_accum<kFT <= kFTSmall>(a, T, R, C, P, uv, v, valid);
            }
        }
        }
        if (j == wv) FKT(7);
        const double tot = wave_sum32(v);
        if (arow && (!kPro || f.apro)) {  // (iteration it + 1's row sums, see FusedArgs::arow)
            if ((lane & 1) == 0 && (lane >> 1) < kNTerms)
                unsafeAtomicAdd(arow + ((size_t)arow_wr(kPro, it) * f.n_kf + (e.x & 0x3fffffff)) * kStride + (lane >> 1),
                                tot);
            continue;
        }
        if ((lane & 1) == 0) part_out[(size_t)dst * kStride + (lane >> 1)] = (lane >> 1) < kNTerms ? tot : 0.0;
        if (lane == 54 || lane == 56)  // terms 27 (cost) and 28 (observations)
            reinterpret_cast<double*>(f.costpart + (size_t)((it + 1) & 1) * f.n_part + dst)[(lane - 54) >> 1] = tot;
    }
    if (!kPro && it == 1) VX_KTW(8, 8);  // (trace build: each wave's pose stage done)
    FKT(5);
}

// ------------------------------------------------------------------ persistent window (k_ba_win)
// The prologue and every iteration of one LocalBA window in ONE launch (round 6, VERDICT r5 #2a).
// k_ba_iter's workgroups already exchange nothing but the keyframe rows: a workgroup solves the poses
// of its own <= kFK keyframe entries from their rows, updates its own landmarks and adds the next
// iteration's pose-stage terms of its landmarks' observations into those rows.  So the launch
// boundary between iterations is replaced by point-to-point hand-offs, not a grid barrier:
//   - iteration i's rows R_i are their own buffer (no reuse inside a run), summed by float atomics
//     (memory side); after its atomics every wave waits for them (vmcnt(0)), the workgroup meets at a
//     barrier, and one lane per entry adds 1 to the entry row's arrival counter cnt[i][row], one lane
//     to done[i] (agent-scope atomics);
//   - a workgroup solves entry row k of iteration i once cnt[i][k] reaches nprod[k] (the number of
//     workgroups with an entry on row k, counted at plan build), polled by the entry's own lane with
//     sc1 loads, and reads the row with sc1 loads (MI355X_MICROARCH.md, hand-off table row 1: atomic
//     producer, sc1-polled counter, sc1 payload loads; no line of R_i is in any cache before it is
//     complete: fresh buffers, kernel-start invalidate);
//   - the stop rule of iteration i - 1 (whether iteration i runs) needs every row of R_(i-1): wave 1
//     polls done[i - 1] == workgroups (one iteration of slack: almost always already true), sums the
//     rows' cost / count terms in a fixed order and decides — every workgroup the same, from the
//     same values; workgroup 0 writes the run's statistics.
// Everything a workgroup loads that no iteration changes (block / entry records, landmark-stage
// observations, the landmarks' slots and runs, the first pose-stage round) is loaded once; the
// entries' poses and the landmark positions stay in registers / LDS.  Buffers by run parity (the
// run's generation, w.gen): a run zeroes the other parity's rows and counters for the next run (plain
// stores, written back at the kernel's end).  Every workgroup must be resident at once (nb <= CUs,
// one 512-thread workgroup per CU); every wait is bounded (kWinSpinTicks): a wait that runs out sets
// the state's fault flag, every workgroup leaves, and vx_ba_plan_fetch re-runs the window with the
// per-iteration launches (plan->win_off) — two persistent windows on one device at once could
// otherwise hold each other's compute units.
struct WinArgs {
    double* rows;      // [2][max_iter][n_kf][kStride]
    int* cnt;          // [2][max_iter][n_kf] arrivals per row
    int* done;         // [2][max_iter][32] workgroups done with iteration i's pose stage (own lines)
    const int* nprod;  // [n_kf] workgroups with an entry on the row
    int* gen;          // run generation (parity = gen & 1), bumped by workgroup 0 at the run's end
    int* fault;        // set when a wait ran out (every workgroup then leaves)
};
constexpr long long kWinSpinTicks = 20'000'000;  // 200 ms of the 100 MHz wall clock
// k_ba_win's LDS: k_ba_iter's plus a second set of pose slots
constexpr size_t win_lds(int ft) {
    return fused_lds(ft) + (size_t)kFK * kLdsStride * sizeof(double) + (size_t)ft * (16 + 16 + 12);
}
static_assert(win_lds(kFTSmall) <= 160 * 1024, "k_ba_win LDS exceeds gfx950's 160 KB per workgroup");

__device__ __forceinline__ int ld_sc1(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add_agent(int* p, int v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lanes with want: spin until *p >= target (each lane its own counter); false when the wait ran out
// or another workgroup reported a fault
#ifndef VX_WIN_POLLS
#define VX_WIN_POLLS 1
#endif
__device__ __forceinline__ bool win_wait(const int* p, int target, bool want, int* fault) {
    const long long t0 = wall_clock64();
    bool ok = true;
    __builtin_amdgcn_s_setprio(0);  // (a polling wave leaves the SIMD to co-resident waves)
    // VX_WIN_POLLS polls in flight: each pass issues the next poll before it checks the oldest (the
    // loads are independent sc1 loads; the compiler waits for the oldest only).  Two or three in
    // flight measured no faster than one (LocalBA alone 0.0508-0.0518 ms with three against
    // 0.0498-0.0509 with one, r06s2 poll A/B): one stays the default
    // (every lane loads — lanes without a wait read the fault word — so no exec-masked branch makes
    // the compiler drain every load at its join)
    const int* const pp = want ? p : fault;
    int q[VX_WIN_POLLS];
#pragma unroll
    for (int i = 0; i + 1 < VX_WIN_POLLS; ++i) q[i] = ld_sc1(pp);
    for (int k = 0;; ++k) {
        q[VX_WIN_POLLS - 1] = ld_sc1(pp);
        const bool pend = want && ok && q[0] < target;
#pragma unroll
        for (int i = 0; i + 1 < VX_WIN_POLLS; ++i) q[i] = q[i + 1];
        if (!__any(pend)) break;
        if ((k & 15) == 15) {
            if (ld_sc1(fault) || wall_clock64() - t0 > kWinSpinTicks) {
                if (pend) ok = false;
                if ((threadIdx.x & 63) == 0) __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_s_sleep(1);  // (longer naps between polls measured the same: r06g)
    }
    __builtin_amdgcn_s_setprio(3);
    return __all(ok);
}

// (232 VGPRs, two waves per SIMD.  Sized for three — 168 VGPRs, so that a third wave of the other
// streams' kernels fits beside it — it spills outside the observation rounds: LocalBA alone 0.067
// against 0.054 ms, the C3 pipeline 0.074 against 0.063 ms/frame, r06i)
template <int kFT>
__global__ __launch_bounds__(kFT) void k_ba_win(BAArgs a, FusedArgs f, WinArgs w) {
    constexpr int kFW = kFT / 64;
    static_assert(kFW >= 2, "k_ba_win: wave 1 runs the stop rule");
    __builtin_amdgcn_s_setprio(3);
    extern __shared__ __attribute__((aligned(16))) double fl[];
    __shared__ int4 s_ke[kFK];
    __shared__ int s_act, s_fault;
    // two pose-slot sets (T 8 | R 9 | C 4 | flags per entry): iteration it solves from set (it - 1) & 1
    // into set it & 1, so a wave still in the previous pose stage (no barrier closes it) reads poses
    // the solve does not overwrite
    double* const ks0 = fl;                              // [2][kFK][kLdsStride]
    double* terms = ks0 + 2 * kFK * kLdsStride;          // [9][kFT]
    int* tcount = reinterpret_cast<int*>(terms + 9 * kFT);
    double* lpos = terms + 9 * kFT + kFT / 2;            // [kFT][3]
    // the landmark stage's per-thread records, loop-invariant: parked in LDS, not in registers
    // (k_ba_win keeps far more state live across its loop than one k_ba_iter launch)
    int4* s_orec = reinterpret_cast<int4*>(lpos + 3 * kFT);      // [kFT]
    double2* s_ouv = reinterpret_cast<double2*>(s_orec + kFT);    // [kFT]
    int* s_run = reinterpret_cast<int*>(s_ouv + kFT);             // [kFT][3]: r0, r1, slot
    const int tid = threadIdx.x, b = blockIdx.x, wv = tid >> 6, lane = tid & 63;
    const size_t base = (size_t)b * kFT;
    const int4* KE = f.kent + (size_t)b * kFK * 2;
    const int M = a.max_iter, nk = a.n_kf, nb = (int)gridDim.x;
    const size_t rows_per = (size_t)M * nk * kStride;
    // ---- loads: the run generation, then everything the window keeps (k_ba_iter's prologue loads
    // plus the landmark-stage records its iteration launches load again and again)
    const int par = w.gen[0] & 1;
    double* const R = w.rows + (size_t)par * rows_per;
    int* const cnt = w.cnt + (size_t)par * M * nk;
    int* const done = w.done + (size_t)par * M * 32;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    const int4 B = f.blk[(size_t)b * (1 + kFW / 2)];
    const int4 WB = f.blk[(size_t)b * (1 + kFW / 2) + 1 + (wvu >> 1)];
    int4 ke = make_int4(-1, 0, 0, 0);
    if (tid < kFK) ke = KE[2 * tid];
    const int4 orec0 = f.lobs_rec[base + tid];
    const double2 ouv0 = f.lobs_uv[base + tid];
    const int lslot0 = f.lm_slot[base + tid];
    const int2 run0 = f.lm_run[base + tid];
    D3 PL;
    {
        const double* P = a.lm_pos0 + 4 * (size_t)lslot0;
        PL = {P[0], P[1], P[2]};
    }
    const int wstart = (wvu & 1) ? WB.z : WB.x, wrounds = (wvu & 1) ? WB.w : WB.y;
    // (each wave's first pose-stage round, requested again before every pose stage: kept in
    // registers across the loop it would cost the registers the landmark stage needs)
    double2 u0 = make_double2(0, 0);
    double4 p0 = make_double4(0, 0, 0, 0);
    auto first_round = [&] {
        if (wrounds > 0) {
            u0 = f.pobs_uv[wstart + lane];
            p0 = f.pobs_p[wstart + lane];
        }
    };
    first_round();
    // the entry's state lives in its LDS slot (T 8 | R 9 | C 4 | flags), not in registers
    double ev[13];
    int np = 0;
    const int row = ke.x & 0x3fffffff;
    if (tid < kFK && ke.x >= 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ev[j] = a.kf_pose0[8 * (size_t)row + j];
#pragma unroll
        for (int j = 0; j < 4; ++j) ev[8 + j] = a.kf_intr[4 * row + j];
        ev[12] = (double)a.kf_flags[row];
        np = w.nprod[row];
    }
    // the next run's buffers (the other parity) zeroed; its rows were last read by the previous run
    {
        double* Ro = w.rows + (size_t)(par ^ 1) * rows_per;
        for (size_t i = (size_t)b * kFT + tid; i < rows_per; i += (size_t)nb * kFT) Ro[i] = 0.0;
        int* co = w.cnt + (size_t)(par ^ 1) * M * nk;
        for (int i = b * kFT + tid; i < M * nk; i += nb * kFT) co[i] = 0;
        int* dn = w.done + (size_t)(par ^ 1) * M * 32;
        for (int i = b * kFT + tid; i < M * 32; i += nb * kFT) dn[i] = 0;
    }
    if (b == 0 && tid < 16) {  // (the statistics of this run, as stop_rule(0) starts them)
        a.state->cost[tid] = 0.0;
        a.state->obs[tid] = 0;
    }
    const int n_lm = B.x, n_ob = B.y, n_ent = B.z;
    const bool has_o = tid < n_ob, own = tid < n_lm;
    lpos[3 * tid] = PL.x;
    lpos[3 * tid + 1] = PL.y;
    lpos[3 * tid + 2] = PL.z;
    s_orec[tid] = orec0;
    s_ouv[tid] = ouv0;
    s_run[3 * tid] = run0.x;
    s_run[3 * tid + 1] = run0.y;
    s_run[3 * tid + 2] = lslot0;
    if (tid < kFK) s_ke[tid] = ke;
    if (tid == 0) s_fault = 0;
    if (tid < kFK && ke.x >= 0) {  // iteration 0's pose stage reads the initial poses (set 1)
        double Rm[9];
        rot_from_quat(ev, Rm);
        double* sl = ks0 + (kFK + tid) * kLdsStride;
        double* sl0 = ks0 + tid * kLdsStride;
#pragma unroll
        for (int j = 0; j < 8; ++j) sl[j] = ev[j];
#pragma unroll
        for (int j = 0; j < 9; ++j) sl[8 + j] = Rm[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) sl[17 + j] = sl0[17 + j] = ev[8 + j];
        sl[21] = sl0[21] = ev[12];
    }
    __syncthreads();

    // ---- pose stage of iteration `itn` from the poses in set (itn - 1) & 1 and the landmarks in lpos,
    // added into R_itn; then the hand-off (every wave's atomics retired, barrier, one arrival per
    // entry row).  (The barrier does not protect the pose slots: the next solve writes the other set.)
    auto pose_stage = [&](int itn) {
        int r = 0;
        double* const Rn = R + (size_t)itn * nk * kStride;
        const double* const kslot = ks0 + ((itn - 1) & 1) * kFK * kLdsStride;
        for (int j = wv; j < n_ent; j += kFW) {
            const int4 e = s_ke[j];
            const int nr = (e.w - e.z + 63) >> 6;
            if (nr == 0) continue;
            const double* T = kslot + j * kLdsStride;
            const double* Rr = T + 8;
            const double* C = T + 17;
            double v[kStride];
#pragma unroll
            for (int t = 0; t < kStride; ++t) v[t] = 0.0;
            for (int q = 0; q < nr; ++q, ++r) {
                const double2 uv = u0;
                const double4 P4 = p0;
                if (r + 1 < wrounds) {
                    int lim = e.w - (e.z + 64 * (q + 1));
                    if (q + 1 >= nr) {  // the wave's next entry with rounds
                        int jn = j + kFW;
                        int4 en = s_ke[jn < kFK ? jn : j];
                        while (jn < n_ent && ((en.w - en.z + 63) >> 6) == 0) {
                            jn += kFW;
                            en = s_ke[jn < kFK ? jn : j];
                        }
                        lim = en.w - en.z;
                    }
                    if (lane < lim) {
                        u0 = f.pobs_uv[wstart + 64 * (r + 1) + lane];
                        p0 = f.pobs_p[wstart + 64 * (r + 1) + lane];
                    } else {
                        u0 = make_double2(0.0, 0.0);
                        p0 = make_double4(0.0, 0.0, 0.0, 0.0);
                    }
                }
                const bool valid = e.z + 64 * q + lane < e.w;
                const int code = (int)P4.w;
                const D3 P = code >= 0 ? D3{lpos[3 * code], lpos[3 * code + 1], lpos[3 * code + 2]} : D3{P4.x, P4.y, P4.z};
                pose_obs_accum<true>(a, T, Rr, C, P, uv, v, valid);
            }
            const double tot = wave_sum32(v);
            if ((lane & 1) == 0 && (lane >> 1) < kNTerms)
                unsafeAtomicAdd(Rn + (size_t)(e.x & 0x3fffffff) * kStride + (lane >> 1), tot);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (this wave's adds are done at the memory side)
        // the hand-off after the workgroup's barrier, one lane per entry row (signalling wave by wave,
        // each wave's entries as soon as its own adds retired, measured 35 % slower: r06e/r06g)
        __syncthreads();
        if (tid < kFK && ke.x >= 0) add_agent(cnt + (size_t)itn * nk + row, 1);
        if (tid == kFK) add_agent(done + (size_t)itn * 32, 1);
    };
    // ---- stop rule of iteration ip (local_ba.cpp:240-247) from every row of R_ip, by wave 1 of every
    // workgroup (the same values summed in the same order: the same decision everywhere)
    double last = 1.7976931348623157e308;
    auto decide = [&](int ip) -> int {
        if (!win_wait(done + (size_t)ip * 32, nb, lane == 0, w.fault)) return -1;
        double tot = 0.0, cn = 0.0;
        for (int q = lane; q < nk; q += 64) {
            tot += ld_sc1(R + ((size_t)ip * nk + q) * kStride + 27);
            cn += ld_sc1(R + ((size_t)ip * nk + q) * kStride + 28);
        }
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) {
            tot += __shfl_xor(tot, m, 64);
            cn += __shfl_xor(cn, m, 64);
        }
        const int tobs = (int)cn;
        const bool stop = tobs == 0 || fabs(last - tot) < 1e-6 * last;
        if (!stop) last = tot;
        if (b == 0 && lane == 0) {
            BAState* s = a.state;
            if (ip < 16) {
                s->cost[ip] = tot;
                s->obs[ip] = tobs;
            }
            s->iterations = ip + 1;
            s->last_cost = last;
            if (!stop && ip + 1 < M)
                s->active[ip + 1] = 1;
            else
                for (int k = ip + 1; k <= M; ++k) s->active[k] = 0;
        }
        return stop ? 0 : 1;
    };

    VX_KT(0);
    pose_stage(0);  // (iteration 0's pose stage: k_ba_iter's prologue)
    if (wv == 0) VX_KT(15);
    for (int it = 0; it < M; ++it) {
        double* const kslot = ks0 + (it & 1) * kFK * kLdsStride;
        const double* const kprev = ks0 + ((it + 1) & 1) * kFK * kLdsStride;
        // ---- A: wave 0 waits for its entries' rows of R_it, reads and solves them; wave 1 decides
        // whether iteration it runs (the stop rule of it - 1)
        if (wv == 0) {
            const bool want = tid < kFK && ke.x >= 0;
            const bool ok = win_wait(cnt + (size_t)it * nk + row, np, want, w.fault);
#ifndef VX_WIN_TRACE_LM
            if (it < 5) VX_KT(1 + 3 * it);
#endif
            if (!ok && lane == 0) s_fault = 1;
            if (want && ok) {
                double S[kNTerms];
                const double* rp = R + ((size_t)it * nk + row) * kStride;
#pragma unroll
                for (int t = 0; t < kNTerms; ++t) S[t] = ld_sc1(rp + t);
                double* sl = kslot + tid * kLdsStride;
                const double* sp = kprev + tid * kLdsStride;
                double T[8], Rm[9];
#pragma unroll
                for (int j = 0; j < 8; ++j) T[j] = sp[j];
                solve_pose(a, (int)sp[21], S, T, Rm);
#pragma unroll
                for (int j = 0; j < 8; ++j) sl[j] = T[j];
#pragma unroll
                for (int j = 0; j < 9; ++j) sl[8 + j] = Rm[j];
            }
        } else if (wv == 1) {
            const int act = it == 0 ? 1 : decide(it - 1);
            if (lane == 0) {
                s_act = act > 0;
                if (act < 0) s_fault = 1;
            }
        }
        __syncthreads();
        if (wv == 0 && it < 5) VX_KT(2 + 3 * it);
        if (s_fault || !s_act) break;
        if (tid < kFK && ke.x >= 0 && (ke.x & (1 << 30))) {  // the owner publishes the pose
            double* Tout = pose_out(a, it) + 8 * (size_t)row;
            const double* sl = kslot + tid * kLdsStride;
#pragma unroll
            for (int j = 0; j < 8; ++j) Tout[j] = sl[j];
        }
        if (it + 1 < M) first_round();
        // ---- landmark stage of iteration it (local_ba.cpp:176-238), as k_ba_iter
        {
            double h[9];
            const int4 orec = s_orec[tid];
            const double2 ouv = s_ouv[tid];
            const D3 PO{lpos[3 * orec.y], lpos[3 * orec.y + 1], lpos[3 * orec.y + 2]};
            const bool ok = obs_terms<true>(a, PO, orec.x, ouv, kslot, kLdsStride, kslot + 8, kLdsStride, kslot + 17,
                                            kLdsStride, h);
#pragma unroll
            for (int j = 0; j < 9; ++j) terms[j * kFT + tid] = h[j];
            tcount[tid] = (has_o && ok) ? 1 : 0;
            __syncthreads();
            if (own) {
                double hs[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                int obs = 0;
                const int r0 = s_run[3 * tid], r1 = s_run[3 * tid + 1];
                int lslot = s_run[3 * tid + 2];
                const D3 P0{lpos[3 * tid], lpos[3 * tid + 1], lpos[3 * tid + 2]};
                for (int q = r0; q < r1; ++q) {
#pragma unroll
                    for (int j = 0; j < 9; ++j) hs[j] += terms[j * kFT + q];
                    obs += tcount[q];
                }
                const D3 P1 = lm_update(a, lslot, P0, hs, obs);
                lpos[3 * tid] = P1.x;
                lpos[3 * tid + 1] = P1.y;
                lpos[3 * tid + 2] = P1.z;
            }
            __syncthreads();
        }
#ifdef VX_WIN_TRACE_LM  // (trace variant: slot 1 + 3 it = the landmark stage done instead of rows ready)
        if (wv == 0 && it < 5) VX_KT(1 + 3 * it);
#endif
        if (it + 1 < M) pose_stage(it + 1);
        if (wv == 0 && it < 4) VX_KT(3 + 3 * it);
    }
    // ---- the last iteration's statistics (a stop inside the loop wrote them), then the next run's
    // parity; workgroup 0 gets here only after every workgroup's first arrival (its waits above), so
    // every workgroup has read the generation
    if (b == 0 && wv == 1 && !s_fault && s_act) {
        const int r = decide(M - 1);
        if (r < 0 && lane == 0) s_fault = 1;
    }
    if (b == 0 && wv == 1 && lane == 0 && !s_fault) w.gen[0] = w.gen[0] + 1;
}

// plan build: nprod[row] = workgroups with an entry on the row (the arrivals k_ba_win waits for)
// (bias: $VX_BA_WIN_TEST_FAULT=1 adds one arrival to row 0 that never comes, so the run's waits run
// out: the test of the fault path, tests/test_gpu_parity.py)
__global__ void k_win_nprod(const int4* kent, int nb, int* nprod, int bias) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nb * kFK) return;
    const int x = kent[2 * (size_t)i].x;
    if (x >= 0) atomicAdd(nprod + (x & 0x3fffffff), 1);
    if (i == 0) atomicAdd(nprod, bias);
}

// sharded plans: each keyframe row's partial slots summed in slot order (the slots of a row no group
// fills are 0) -> rowpart, which the per-iteration all-reduce then sums over the ranks
__global__ void k_row_sum(const double* part, int n_kf, int maxl, double* rowpart) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_kf * kStride) return;
    const int row = i / kStride, t = i - row * kStride;
    const double* src = part + (size_t)row * maxl * kStride + t;
    double s = 0.0;
    for (int q = 0; q < maxl; ++q) s += src[(size_t)q * kStride];
    rowpart[i] = s;
}

// ---- one-shot peer reduction of a sharded window's row sums ($VX_BA_PEER=1, opt-in)
// In place of the per-iteration ncclAllReduce (a ring of 2 (N - 1) dependent steps, latency-bound at
// 100 KB: DESIGN.md §6): every rank publishes its row sums into a block of its own device memory that
// every other rank has mapped (IPC over xGMI) and sets the block's flag to the iteration's
// generation; every rank waits for all N flags and sums the ranks' rows in rank order — the same
// values on every rank, and bitwise what the one-GPU emulation's k_sum_parts gives.  The rows are
// double-buffered by generation parity: a rank rewrites parity p at generation g + 2 only after its
// own wait for every flag >= g + 1, which each rank sets after it has read generation g.  Bounded
// waits: a flag that does not come sets the state's fault (vx_ba_plan_fetch reports VX_ERR_COMM).
constexpr int kMaxPeers = 16;
constexpr long long kPeerSpinTicks = 20'000'000;  // 200 ms of the 100 MHz wall clock
struct PeerPtrs {
    const double* rows[kMaxPeers];
    const unsigned long long* flag[kMaxPeers];
};
// this rank's row sums (k_row_sum's arithmetic: slots in slot order) -> its block (parity), then the flag
__global__ __launch_bounds__(1024) void k_peer_publish(const double* part, int n_kf, int maxl, double* out,
                                                      unsigned long long* flag, unsigned long long gen) {
    const int n = n_kf * kStride;
    for (int i = threadIdx.x; i < n; i += 1024) {
        const int row = i / kStride, t = i - row * kStride;
        const double* src = part + (size_t)row * maxl * kStride + t;
        double s = 0.0;
        for (int q = 0; q < maxl; ++q) s += src[(size_t)q * kStride];
        out[i] = s;
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// every rank's flag >= gen, then the ranks' rows (parity offset off) summed in rank order -> out
__global__ __launch_bounds__(1024) void k_peer_gather(PeerPtrs pp, int n_ranks, int len, int off, unsigned long long gen,
                                                     double* out, int* fault) {
    __shared__ int s_bad;
    if (threadIdx.x == 0) s_bad = 0;
    __syncthreads();
    if (threadIdx.x < n_ranks) {
        const long long t0 = wall_clock64();
        while (__hip_atomic_load(pp.flag[threadIdx.x], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
            if (wall_clock64() - t0 > kPeerSpinTicks) {
                s_bad = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    if (s_bad) {
        if (threadIdx.x == 0) __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    __threadfence_system();
    for (int i = threadIdx.x; i < len; i += 1024) {
        double s = __hip_atomic_load(pp.rows[0] + off + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int r = 1; r < n_ranks; ++r) s += __hip_atomic_load(pp.rows[r] + off + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        out[i] = s;
    }
}

// fused-order observation payloads: uv by plan index (-1: padding), pose records with the fixed
// landmarks' positions
__global__ void k_fused_gather(const int* lsrc, int nl, const double2* luv, double2* out_luv, const int* psrc,
                               const int* pcode, int np, const double2* puv, const double* lm_pos0, double2* out_puv,
                               double4* out_pp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nl) out_luv[i] = lsrc[i] >= 0 ? luv[lsrc[i]] : make_double2(1e300, 1e300);
    if (i < np) {
        const int sidx = psrc[i], c = pcode[i];
        out_puv[i] = sidx >= 0 ? puv[sidx] : make_double2(0.0, 0.0);
        double4 P = make_double4(0.0, 0.0, 0.0, (double)c);
        if (c < 0) {
            const double* q = lm_pos0 + 4 * (size_t)(-1 - c);
            P.x = q[0];
            P.y = q[1];
            P.z = q[2];
        }
        out_pp[i] = P;
    }
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
    a.huber2 = a.huber * a.huber;
    a.max_err2 = a.max_err * a.max_err;
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
    // (the fault word is read by every fetch; a recycled state block may hold anything)
    VX_HIP(c, hipMemsetAsync(p->state.p, 0, sizeof(BAState), c->stream));
    return VX_OK;
}

namespace {
template <class B>
void swap_buf(B& a, B& b) {
    std::swap(a.p, b.p);
    std::swap(a.bytes, b.bytes);
}
// dst takes src's buffers (and src dst's); nothing else of either plan moves
void adopt_buffers(vx_ba_plan* dst, vx_ba_plan* src) {
#define VX_SWAP_BUF(b) swap_buf(dst->b, src->b);
    VX_PLAN_BUFFERS(VX_SWAP_BUF)
#undef VX_SWAP_BUF
}
constexpr size_t kMaxPlanHusks = 4;  // parked buffer sets per context
}  // namespace

vx_ba_plan* plan_new(vx_ctx* c) {
    auto* p = new vx_ba_plan();
    p->c = c;
    if (!c) return p;
    if (!c->plan_husks.empty()) {
        vx_ba_plan* h = c->plan_husks.back();
        c->plan_husks.pop_back();
        adopt_buffers(p, h);
        delete h;
    }
    c->plan_live.push_back(p);
    return p;
}

// Test hook: $VX_TEST_FAIL_PLAN=1 makes every plan build fail after the plan was registered with
// its context (tests/test_gpu_parity.py::test_failed_plan_build_then_destroy).
int plan_fault_injected(vx_ctx* c) {
    const char* e = getenv("VX_TEST_FAIL_PLAN");
    return (e && e[0] == '1') ? set_error(c, VX_ERR_STATE, "plan build failed ($VX_TEST_FAIL_PLAN)") : VX_OK;
}

void plan_pool_release(vx_ctx* c) {
    for (vx_ba_plan* h : c->plan_husks) delete h;
    c->plan_husks.clear();
    for (vx_ba_plan* p : c->plan_live) p->c = nullptr;  // their destroy then just frees
    c->plan_live.clear();
}

bool fused_eligible(const vx_ba_plan* p) {
    if (p->status != 0 || p->global_poses || p->n_kf > kMaxKfLds || p->n_opt <= 0) return false;
    if (const char* e = getenv("VX_BA_FUSED"))
        if (e[0] == '0') return false;
    return true;
}

// $VX_BA_PERSIST=0: the fused LocalBA as one launch per iteration (k_ba_iter) instead of the
// persistent window (k_ba_win; read at plan build)
bool ba_persist() {
    const char* e = getenv("VX_BA_PERSIST");
    return !(e && e[0] == '0');
}

// $VX_BA_ATOMIC_ROWS=0: the fused LocalBA's per-keyframe partial slots (every run bitwise the
// same) instead of row sums by float atomics (FusedArgs::arow; read at plan build)
bool ba_atomic_rows() {
    const char* e = getenv("VX_BA_ATOMIC_ROWS");
    return !(e && e[0] == '0');
}

// 1024 threads when 512-thread workgroups would outnumber the compute units (their count is within a
// few percent of the landmark-stage observations / 512: whole landmarks of <= 5 observations);
// VX_BA_FUSED_THREADS / VX_BA_FUSED_CAP override for sweeps
int fused_threads(vx_ctx* c, int64_t n_lobs, int* cap) {
    if (!c->n_cus) c->n_cus = std::max(vx_device_cus(c->device), 1);
    int ft = n_lobs > (int64_t)c->n_cus * (kFTSmall - 16) ? kFTLarge : kFTSmall;
    if (const char* e = getenv("VX_BA_FUSED_THREADS")) {
        const int v = atoi(e);
        ft = v == kFTLarge ? kFTLarge : v == kFTNarrow ? kFTNarrow : kFTSmall;
    }
    *cap = ft;
    if (const char* e = getenv("VX_BA_FUSED_CAP")) *cap = std::min(ft, std::max(64, atoi(e)));
    return ft;
}

size_t fused_offsets(int nb, int ft, size_t n_pp, FusedOffsets& F) {
    const size_t n_lp = (size_t)nb * ft;
    size_t at = 0;
    auto take = [&](size_t bytes) {
        const size_t o = at;
        at += (bytes + 255) & ~(size_t)255;
        return o;
    };
    F.blk = take((size_t)nb * fused_blk_ints(ft) * 4);
    F.lm_slot = take(n_lp * 4);
    F.lm_run = take(n_lp * 8);
    F.lobs_rec = take(n_lp * 16);
    F.kent = take((size_t)nb * kFK * 32);
    F.lobs_src = take(n_lp * 4);
    F.pobs_src = take(std::max<size_t>(n_pp, 1) * 4);
    F.pobs_code = take(std::max<size_t>(n_pp, 1) * 4);
    return at;
}

int fused_finish(vx_ctx* c, vx_ba_plan* p, int nb, int ft, int maxl, size_t n_pp, int stop_b) {
    const FusedOffsets& F = p->f_off;
    const size_t n_lp = (size_t)nb * ft;
    const uint8_t* T = p->f_tab.as<uint8_t>();
    VX_HIP(c, p->f_lobs_uv.ensure(n_lp * sizeof(double2)));
    VX_HIP(c, p->f_pobs_uv.ensure(std::max<size_t>(n_pp, 1) * sizeof(double2)));
    VX_HIP(c, p->f_pobs_p.ensure(std::max<size_t>(n_pp, 1) * sizeof(double4)));
    hipLaunchKernelGGL(k_fused_gather, dim3((unsigned)((std::max(n_lp, n_pp) + 255) / 256)), dim3(256), 0, c->stream,
                       reinterpret_cast<const int*>(T + F.lobs_src), (int)n_lp, (const double2*)p->lobs_uv.as<double2>(),
                       p->f_lobs_uv.as<double2>(), reinterpret_cast<const int*>(T + F.pobs_src),
                       reinterpret_cast<const int*>(T + F.pobs_code), (int)n_pp, (const double2*)p->pobs_uv.as<double2>(),
                       (const double*)p->lm_pos0.as<double>(), p->f_pobs_uv.as<double2>(), p->f_pobs_p.as<double4>());
    VX_LAUNCH_CHECK(c, "k_fused_gather");
    VX_HIP(c, p->f_lpos.ensure(n_lp * sizeof(double4)));
    VX_HIP(c, p->f_epose.ensure((size_t)nb * kFK * 16 * sizeof(double)));
    const size_t part_bytes = 2 * (size_t)p->n_kf * maxl * kStride * sizeof(double);
    VX_HIP(c, p->f_part.ensure(part_bytes));
    if (p->shard_count > 1) VX_HIP(c, p->f_rowpart.ensure((size_t)p->n_kf * kStride * sizeof(double)));
    VX_HIP(c, hipMemsetAsync(p->f_part.p, 0, part_bytes, c->stream));  // slots no group writes stay 0
    const size_t cost_bytes = 2 * (size_t)p->n_kf * maxl * sizeof(double2);
    VX_HIP(c, p->f_costpart.ensure(cost_bytes));
    VX_HIP(c, hipMemsetAsync(p->f_costpart.p, 0, cost_bytes, c->stream));
    // row sums by float atomics (FusedArgs::arow): unsharded plans, unless $VX_BA_ATOMIC_ROWS=0
    // (partial slots: every run bitwise the same)
    p->f_atomic = p->shard_count <= 1 && ft <= kFTSmall && ba_atomic_rows();
    if (p->f_atomic) {
        const size_t ab = 4 * (size_t)p->n_kf * kStride * sizeof(double);
        VX_HIP(c, p->f_arow.ensure(ab));
        VX_HIP(c, hipMemsetAsync(p->f_arow.p, 0, ab, c->stream));
    }
    // persistent window (k_ba_win): unsharded atomic-row plans of 512-thread workgroups that are all
    // resident at once (one per CU); $VX_BA_PERSIST=0 keeps the per-iteration launches
    p->f_persist = false;
    p->win_off = false;
    if (!c->n_cus) c->n_cus = std::max(vx_device_cus(c->device), 1);
    if (p->f_atomic && ft == kFTSmall && nb <= c->n_cus && p->opt.max_iterations >= 1 &&
        p->opt.max_iterations <= kMaxIter && ba_persist()) {
        const size_t M = (size_t)p->opt.max_iterations, nk = (size_t)p->n_kf;
        size_t at = 0;
        auto take = [&](size_t bytes) {
            const size_t o = at;
            at += (bytes + 255) & ~(size_t)255;
            return o;
        };
        p->win_rows_off = take(2 * M * nk * kStride * sizeof(double));
        p->win_cnt_off = take(2 * M * nk * sizeof(int));
        p->win_done_off = take(2 * M * 32 * sizeof(int));
        p->win_nprod_off = take(nk * sizeof(int));
        p->win_gen_off = take(sizeof(int));
        VX_HIP(c, p->f_win.ensure(at));
        VX_HIP(c, hipMemsetAsync(p->f_win.p, 0, at, c->stream));
        hipLaunchKernelGGL(k_win_nprod, dim3((unsigned)((nb * kFK + 255) / 256)), dim3(256), 0, c->stream,
                           reinterpret_cast<const int4*>(T + F.kent), nb,
                           reinterpret_cast<int*>(p->f_win.as<uint8_t>() + p->win_nprod_off),
                           getenv("VX_BA_WIN_TEST_FAULT") ? 1 : 0);
        VX_LAUNCH_CHECK(c, "k_win_nprod");
        p->f_persist = true;
    }
    p->f_stop_b = stop_b;
    p->f_blocks = nb;
    p->f_maxl = maxl;
    p->f_threads = ft;
    p->f_npp = n_pp;
    p->fused = true;
    return VX_OK;
}

// The fused layout (k_ba_iter) from the plan's CSRs, on the host: both plan builders end here with
// the same arrays, so the layout — and every run — is the same for both.
//   1. optimised landmarks ordered by the first window keyframe that observes them (stable), so a
//      workgroup's landmarks share few keyframes;
//   2. greedy workgroups: at most ft landmarks, ft landmark-stage observations and kFK
//      keyframes (those of its landmark-stage and pose-stage observations);
//   3. each window keyframe owned by the first workgroup that touches it (untouched ones by
//      workgroup 0): the owner publishes its pose and takes the pose observations of fixed
//      landmarks in it;
//   4. a workgroup's pose observations grouped by keyframe (ascending observation index inside,
//      i.e. the plan's keyframe-major order), one partial slot per non-empty (workgroup, keyframe)
//      group, numbered per keyframe in workgroup order.
int build_fused(vx_ctx* c, vx_ba_plan* p, const std::vector<int>& kptr, const std::vector<int>& plm,
                const std::vector<int>& lptr, const std::vector<int>& lkf) {
    p->fused = false;
    if (!fused_eligible(p)) return VX_OK;
    const int nk = p->n_kf, n_opt = p->n_opt, n_pose = kptr[nk];
    // $VX_PLAN_TIMING=1: phase times of this build on stderr (scripts/plan_build_time.py)
    static const bool timing = getenv("VX_PLAN_TIMING") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    double t_ph[16] = {0};
    auto lap = [&](int i) { t_ph[i] = std::chrono::duration<double, std::milli>(clk::now() - t_start).count(); };
    std::vector<int> pkf(n_pose);
    for (int k = 0; k < nk; ++k)
        for (int o = kptr[k]; o < kptr[k + 1]; ++o) pkf[o] = k;
    // pose observations per optimised slot (ascending)
    std::vector<int> pp(n_opt + 1, 0), pidx;
    for (int o = 0; o < n_pose; ++o)
        if (plm[o] < n_opt) ++pp[plm[o] + 1];
    for (int q = 0; q < n_opt; ++q) pp[q + 1] += pp[q];
    pidx.resize(pp[n_opt]);
    {
        std::vector<int> w(pp.begin(), pp.end() - 1);
        for (int o = 0; o < n_pose; ++o)
            if (plm[o] < n_opt) pidx[w[plm[o]]++] = o;
    }
    lap(3);
    // 1. keyframe-locality order (counting sort by first keyframe, stable)
    std::vector<int> key(n_opt, nk), order(n_opt);
    for (int q = 0; q < n_opt; ++q) {
        int k0 = nk;
        for (int o = lptr[q]; o < lptr[q + 1]; ++o) k0 = std::min(k0, lkf[o]);
        for (int i = pp[q]; i < pp[q + 1]; ++i) k0 = std::min(k0, pkf[pidx[i]]);
        key[q] = k0;
    }
    {
        std::vector<int> kc(nk + 2, 0);
        for (int q = 0; q < n_opt; ++q) ++kc[key[q] + 1];
        for (int k = 0; k <= nk; ++k) kc[k + 1] += kc[k];
        for (int q = 0; q < n_opt; ++q) order[kc[key[q]]++] = q;
    }
    lap(4);
    // each optimised landmark's distinct keyframes (landmark-stage and pose-stage observations)
    std::vector<int> uk_ptr(n_opt + 1, 0), uk;
    uk.reserve((size_t)lptr[n_opt] + pidx.size());
    {
        std::vector<int> seen(nk, -1);
        for (int q = 0; q < n_opt; ++q) {
            for (int o = lptr[q]; o < lptr[q + 1]; ++o)
                if (seen[lkf[o]] != q) {
                    seen[lkf[o]] = q;
                    uk.push_back(lkf[o]);
                }
            for (int i = pp[q]; i < pp[q + 1]; ++i)
                if (seen[pkf[pidx[i]]] != q) {
                    seen[pkf[pidx[i]]] = q;
                    uk.push_back(pkf[pidx[i]]);
                }
            uk_ptr[q + 1] = (int)uk.size();
        }
    }
    lap(5);
    // 2. greedy workgroups of ft threads (cap: landmark-stage observations and landmarks per
    // workgroup; VX_BA_FUSED_THREADS / VX_BA_FUSED_CAP override for sweeps).  1024
    // threads when 512-thread workgroups would outnumber the compute units (their count is within a
    // few percent of the landmark-stage observations / 512: whole landmarks of <= 5 observations)
    int cap = 0;
    const int ft = fused_threads(c, lptr[n_opt], &cap);
    std::vector<std::vector<int>> K(1), LM(1);
    std::vector<int> stamp(nk, -1);
    int n_l = 0, n_o = 0;
    for (int idx = 0; idx < n_opt; ++idx) {
        const int q = order[idx], cnt = lptr[q + 1] - lptr[q];
        if (cnt > ft) return VX_OK;
        int cur = (int)K.size() - 1;
        int nn = 0;
        for (int u = uk_ptr[q]; u < uk_ptr[q + 1]; ++u) nn += stamp[uk[u]] != cur;
        if (n_l > 0 && (n_l + 1 > cap || n_o + cnt > cap || (int)K[cur].size() + nn > kFK)) {
            K.emplace_back();
            LM.emplace_back();
            ++cur;
            n_l = n_o = 0;
            nn = uk_ptr[q + 1] - uk_ptr[q];
        }
        if (nn > kFK) return VX_OK;
        for (int u = uk_ptr[q]; u < uk_ptr[q + 1]; ++u)
            if (stamp[uk[u]] != cur) {
                stamp[uk[u]] = cur;
                K[cur].push_back(uk[u]);
            }
        LM[cur].push_back(q);
        ++n_l;
        n_o += cnt;
    }
    const int nb = (int)K.size();
    // the device build's workgroup limit (k_fb_pose_rank's LDS counters, ba_fused_build.hip): beyond
    // it both builds give the plan no fused layout, so host- and device-built plans stay identical
    if (nb > kFusedMaxGroups) return VX_OK;
    const int fw = ft / 64;
    lap(0);
    // 3. owners
    std::vector<int> owner(nk, -1);
    for (int b = 0; b < nb; ++b)
        for (int k : K[b])
            if (owner[k] < 0) owner[k] = b;
    for (int k = 0; k < nk; ++k)
        if (owner[k] < 0) {
            owner[k] = 0;
            K[0].push_back(k);
        }
    if ((int)K[0].size() > kFK) return VX_OK;
    for (auto& v : K) std::sort(v.begin(), v.end());
    lap(6);
    // 4. pose observations per workgroup (ascending observation index = keyframe-major)
    std::vector<int> lm_blk(n_opt), lm_loc(n_opt);
    for (int b = 0; b < nb; ++b)
        for (int i = 0; i < (int)LM[b].size(); ++i) {
            lm_blk[LM[b][i]] = b;
            lm_loc[LM[b][i]] = i;
        }
    // (CSR by workgroup, ascending observation index inside)
    std::vector<int> po_ptr(nb + 1, 0), po(n_pose), po_blk(n_pose);
    for (int o = 0; o < n_pose; ++o) {
        po_blk[o] = plm[o] < n_opt ? lm_blk[plm[o]] : owner[pkf[o]];
        ++po_ptr[po_blk[o] + 1];
    }
    for (int b = 0; b < nb; ++b) po_ptr[b + 1] += po_ptr[b];
    {
        std::vector<int> w(po_ptr.begin(), po_ptr.end() - 1);
        for (int o = 0; o < n_pose; ++o) po[w[po_blk[o]]++] = o;
    }
    // tables: landmarks / landmark-stage observations at b * ft, keyframe entries at b * kFK,
    // pose observations wave-major with 64-aligned entries.  Written straight into one pinned
    // staging block and uploaded with one copy (the build is paid per LocalBA::Optimize call).
    const int kBlkInts = fused_blk_ints(ft);
    lap(7);
    // pass 1: each entry's pose observations, the waves' rounds
    std::vector<int> ent_beg((size_t)nb * kFK, 0), ent_end((size_t)nb * kFK, 0);
    size_t n_pp = 0;
    for (int b = 0; b < nb; ++b) {
        int i = po_ptr[b];
        for (int j = 0; j < (int)K[b].size(); ++j) {
            ent_beg[(size_t)b * kFK + j] = i;
            while (i < po_ptr[b + 1] && pkf[po[i]] == K[b][j]) ++i;
            ent_end[(size_t)b * kFK + j] = i;
            n_pp += (size_t)(i - ent_beg[(size_t)b * kFK + j] + 63) / 64 * 64;
        }
        if (i != po_ptr[b + 1]) return set_error(c, VX_ERR_STATE, "fused layout: pose observations out of keyframe order");
    }
    // entry positions: SIMD-aware LPT over the entries' pose-stage rounds (fused_place_entries)
    std::vector<int> epos((size_t)nb * kFK, -1), n_pos(nb, 0);
    for (int b = 0; b < nb; ++b) {
        int rounds[kFK];
        const int ne = (int)K[b].size();
        for (int j = 0; j < ne; ++j)
            rounds[j] = (ent_end[(size_t)b * kFK + j] - ent_beg[(size_t)b * kFK + j] + 63) / 64;
        n_pos[b] = fused_place_entries(rounds, ne, &epos[(size_t)b * kFK]);
    }
    FusedOffsets& F = p->f_off;
    const size_t at = fused_offsets(nb, ft, n_pp, F);
    lap(8);
    VX_HIP(c, p->f_stage.ensure(at, true));
    lap(9);
    uint8_t* S = static_cast<uint8_t*>(p->f_stage.p);
    int* blk = reinterpret_cast<int*>(S + F.blk);
    int* lm_slot = reinterpret_cast<int*>(S + F.lm_slot);
    int2* lm_run = reinterpret_cast<int2*>(S + F.lm_run);
    int4* lobs_rec = reinterpret_cast<int4*>(S + F.lobs_rec);
    int* kent = reinterpret_cast<int*>(S + F.kent);
    int* lobs_src = reinterpret_cast<int*>(S + F.lobs_src);
    int* pobs_src = reinterpret_cast<int*>(S + F.pobs_src);
    int* pobs_code = reinterpret_cast<int*>(S + F.pobs_code);
    std::memset(blk, 0, (size_t)nb * kBlkInts * 4);
    std::vector<int> loc(nk, -1), rank(nk, 0), ent_rank((size_t)nb * kFK, -1), at_pos(kFK);
    size_t pw = 0;
    long long stop_key = -1;
    for (int b = 0; b < nb; ++b) {
        int max_rounds = 0;
        const int* EP = &epos[(size_t)b * kFK];
        for (int j = 0; j < (int)K[b].size(); ++j) loc[K[b][j]] = EP[j];
        std::fill(at_pos.begin(), at_pos.end(), -1);
        for (int j = 0; j < (int)K[b].size(); ++j) at_pos[EP[j]] = j;
        int* B = blk + (size_t)b * kBlkInts;
        const size_t base = (size_t)b * ft;
        int ob = 0;
        for (int t = 0; t < (int)LM[b].size(); ++t) {
            const int q = LM[b][t];
            lm_slot[base + t] = q;
            lm_run[base + t].x = ob;
            for (int o = lptr[q]; o < lptr[q + 1]; ++o, ++ob) {
                lobs_src[base + ob] = o;
                lobs_rec[base + ob] = make_int4(loc[lkf[o]], t, q, 0);
            }
            lm_run[base + t].y = ob;
        }
        // padding rows (valid loads: slot 0, empty runs, no observation)
        for (int t = (int)LM[b].size(); t < ft; ++t) {
            lm_slot[base + t] = 0;
            lm_run[base + t] = make_int2(0, 0);
        }
        for (int t = ob; t < ft; ++t) {
            lobs_src[base + t] = -1;
            lobs_rec[base + t] = make_int4(0, 0, 0, 0);
        }
        B[0] = (int)LM[b].size();
        B[1] = ob;
        B[2] = n_pos[b];  // (positions: entries and holes)
        int* E = kent + (size_t)b * kFK * 8;
        for (int j = 0; j < kFK; ++j)
            for (int x = 0; x < 8; ++x) E[8 * j + x] = (x == 0 || x == 4) ? -1 : 0;
        for (int w = 0; w < fw; ++w) {
            const size_t wstart = pw;
            for (int P = w; P < n_pos[b]; P += fw) {
                const int j = at_pos[P];
                if (j < 0) continue;  // a hole
                const int k = K[b][j];
                const int e0 = ent_beg[(size_t)b * kFK + j], e1 = ent_end[(size_t)b * kFK + j], n = e1 - e0;
                E[8 * P] = k | (owner[k] == b ? (1 << 30) : 0);
                E[8 * P + 2] = (int)pw;
                E[8 * P + 3] = (int)pw + n;
                for (int x = e0; x < e1; ++x) {
                    const int o = po[x];
                    pobs_src[pw + (x - e0)] = o;
                    pobs_code[pw + (x - e0)] = plm[o] < n_opt ? lm_loc[plm[o]] : -1 - plm[o];
                }
                const size_t padded = (size_t)(n + 63) / 64 * 64;  // pad to the next round
                for (size_t x = n; x < padded; ++x) {
                    pobs_src[pw + x] = -1;
                    pobs_code[pw + x] = 0;
                }
                pw += padded;
                if (n > 0) ent_rank[(size_t)b * kFK + j] = rank[k]++;
            }
            B[4 + 2 * w] = (int)wstart;
            B[4 + 2 * w + 1] = (int)((pw - wstart) / 64);
            max_rounds = std::max(max_rounds, B[4 + 2 * w + 1]);
        }
        const long long key = fused_stop_key(max_rounds, n_pos[b], b);
        if (stop_key < 0 || key < stop_key) stop_key = key;
        for (int k : K[b]) loc[k] = -1;
    }
    lap(10);
    int maxl = 1;
    for (int k = 0; k < nk; ++k) maxl = std::max(maxl, rank[k]);
    for (int b = 0; b < nb; ++b)
        for (int j = 0; j < (int)K[b].size(); ++j) {
            int* E = kent + ((size_t)b * kFK + epos[(size_t)b * kFK + j]) * 8;
            const int k = K[b][j];
            E[1] = rank[k];
            const int r = ent_rank[(size_t)b * kFK + j];
            E[4] = r >= 0 ? k * maxl + r : -1;
        }
    lap(1);
    // one upload, then the observation payloads gathered into the fused order
    VX_HIP(c, p->f_tab.ensure(at));
    VX_HIP(c, hipMemcpyAsync(p->f_tab.p, S, at, hipMemcpyHostToDevice, c->stream));
    int rc;
    if ((rc = fused_finish(c, p, nb, ft, maxl, n_pp, (int)(stop_key & 0xffffffff)))) return rc;
    VX_HIP(c, hipStreamSynchronize(c->stream));  // (the staging block is reused by the next build)
    lap(2);
    if (timing)
    {
        fprintf(stderr, "[vx plan] fused layout: pack %.3f ms, tables %.3f ms, upload + gather %.3f ms (%d workgroups x %d)\n",
                t_ph[0], t_ph[1] - t_ph[0], t_ph[2] - t_ph[1], nb, ft);
        fprintf(stderr, "[vx plan]   laps: pp %.3f order %.3f uk %.3f greedy %.3f owners %.3f po %.3f pass1 %.3f pinned %.3f tables %.3f ranks %.3f\n",
                t_ph[3], t_ph[4] - t_ph[3], t_ph[5] - t_ph[4], t_ph[0] - t_ph[5], t_ph[6] - t_ph[0], t_ph[7] - t_ph[6],
                t_ph[8] - t_ph[7], t_ph[9] - t_ph[8], t_ph[10] - t_ph[9], t_ph[1] - t_ph[10]);
    }
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
    if ((rc = alloc_run_buffers(c, p))) return rc;
    return build_fused(c, p, kf_obs_ptr, plm, lptr, lkf);
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
            static std::atomic<uint64_t> done{0};
            VX_HIP(c, lds_attr_once(c->device, reinterpret_cast<const void*>(&k_landmark_solve), 160 * 1024, done));
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
    // {workgroups, most observations of a landmark, 1 if this rank has no fused layout}: the fused
    // path runs only when every rank has one (their collectives must match)
    const int32_t mine[3] = {p->n_lm_blocks, p->max_lm_obs, p->fused ? 0 : 1};
    DevBuf d;
    VX_HIP(c, d.ensure(sizeof mine));
    VX_HIP(c, hipMemcpyAsync(d.p, mine, sizeof mine, hipMemcpyHostToDevice, c->stream));
    ncclResult_t r = ncclAllReduce(d.p, d.p, 3, ncclInt32, ncclMax, c->comm, c->stream);
    if (r != ncclSuccess) return set_error(c, VX_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
    int32_t all[3];
    VX_HIP(c, hipMemcpyAsync(all, d.p, sizeof all, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    p->lds_poses = choose_lds_poses(p, all[0], all[1]);
    p->fused_all = all[2] == 0;
    p->choice_made = true;
    return VX_OK;
}
#endif

FusedArgs make_fused_args(vx_ba_plan* p) {
    FusedArgs f{};
    const uint8_t* T = p->f_tab.as<uint8_t>();
    f.blk = reinterpret_cast<const int4*>(T + p->f_off.blk);
    f.lm_slot = reinterpret_cast<const int*>(T + p->f_off.lm_slot);
    f.lm_run = reinterpret_cast<const int2*>(T + p->f_off.lm_run);
    f.lobs_uv = p->f_lobs_uv.as<double2>();
    f.lobs_rec = reinterpret_cast<const int4*>(T + p->f_off.lobs_rec);
    f.kent = reinterpret_cast<const int4*>(T + p->f_off.kent);
    f.pobs_uv = p->f_pobs_uv.as<double2>();
    f.pobs_p = p->f_pobs_p.as<double4>();
    f.part = p->f_part.as<double>();
    f.maxl = p->f_maxl;
    f.n_part = p->n_kf * p->f_maxl;
    f.rowpart = p->shard_count > 1 ? p->f_rowpart.as<double>() : nullptr;
    f.costpart = p->f_costpart.as<double2>();
    f.stop_b = p->f_stop_b;
    f.lpos = p->f_lpos.as<double4>();
    f.epose = p->f_epose.as<double>();
    f.arow = p->f_atomic && p->shard_count <= 1 ? p->f_arow.as<double>() : nullptr;
    f.n_kf = p->n_kf;
    f.apro = p->opt.max_iterations >= 2;
    static const int drow_env = [] {
        const char* e = getenv("VX_BA_DROW");
        return e && e[0] == '0' ? 0 : 1;
    }();
    f.drow = drow_env;
    static const int padskip_env = [] {
        const char* e = getenv("VX_BA_PADSKIP");
        return e && e[0] == '0' ? 0 : 1;
    }();
    f.padskip = padskip_env;
    return f;
}

// the fused path's launches: prologue (iteration 0's pose stage, it = -1) or k_ba_iter(it)
// $VX_BA_COMPACT=0: the 512-thread iterations without the compacted pose stage (A/B runs)
bool ba_compact() {
    static const bool on = [] {
        // off by default: measured 0.0559 vs 0.0540 ms per C3 window (profiles/r04), VX_BA_COMPACT=1 on
        const char* e = std::getenv("VX_BA_COMPACT");
        return e && e[0] == '1';
    }();
    return on;
}

template <int kFT>
int fused_launch_t(vx_ctx* c, vx_ba_plan* p, const BAArgs& a, const FusedArgs& f, int it) {
    constexpr int lds = (int)fused_lds(kFT);
    constexpr int lds_c = (int)fused_lds_cmp(kFTSmall);
    static std::atomic<uint64_t> d0{0}, d1{0}, d2{0};  // (per device: ADVICE r4)
    VX_HIP(c, lds_attr_once(c->device, reinterpret_cast<const void*>(&k_ba_iter<true, kFT>), lds, d0));
    VX_HIP(c, lds_attr_once(c->device, reinterpret_cast<const void*>(&k_ba_iter<false, kFT>), lds, d1));
    VX_HIP(c, lds_attr_once(c->device, reinterpret_cast<const void*>(&k_ba_iter<false, kFTSmall, true>), lds_c, d2));
    if (it < 0)
        VX_HIP(c, launch(c, kStBaPrologue, k_ba_iter<true, kFT>, dim3(p->f_blocks), dim3(kFT), (uint32_t)lds, c->stream,
                         a, f, -1));
    else if (kFT == kFTSmall && ba_compact())
        VX_HIP(c, launch(c, kStBaIter, k_ba_iter<false, kFTSmall, true>, dim3(p->f_blocks), dim3(kFTSmall),
                         (uint32_t)lds_c, c->stream, a, f, it));
    else
        VX_HIP(c, launch(c, kStBaIter, k_ba_iter<false, kFT>, dim3(p->f_blocks), dim3(kFT), (uint32_t)lds, c->stream,
                         a, f, it));
    return VX_OK;
}
int fused_launch(vx_ctx* c, vx_ba_plan* p, const BAArgs& a, const FusedArgs& f, int it) {
    if (p->f_threads == kFTLarge) return fused_launch_t<kFTLarge>(c, p, a, f, it);
    if (p->f_threads == kFTNarrow) return fused_launch_t<kFTNarrow>(c, p, a, f, it);
    return fused_launch_t<kFTSmall>(c, p, a, f, it);
}
// sharded fused path: the rows of the partial buffer iteration it reads (parity it & 1) -> f_rowpart
int fused_row_sum(vx_ctx* c, vx_ba_plan* p, int it) {
    const int n = p->n_kf * kStride;
    ProfScope ps(c, kStBaPoseSum);
    hipLaunchKernelGGL(k_row_sum, dim3((n + 255) / 256), dim3(256), 0, c->stream,
                       (const double*)(p->f_part.as<double>() + (size_t)(it & 1) * p->n_kf * p->f_maxl * kStride),
                       p->n_kf, p->f_maxl, p->f_rowpart.as<double>());
    VX_LAUNCH_CHECK(c, "k_row_sum");
    return VX_OK;
}

// the peer reduction of iteration it's row sums into f_rowpart (plans set up by peer_setup or the
// emulation; every rank / shard of the window enqueues the same generations)
size_t peer_len(const vx_ba_plan* p) { return (size_t)p->n_kf * kStride; }
int peer_publish(vx_ctx* c, vx_ba_plan* p, int it, unsigned long long gen) {
    const size_t len = peer_len(p);
    double* blk = static_cast<double*>(p->peer_mem);
    if (!blk) return set_error(c, VX_ERR_STATE, "peer reduction: no block of its own");
    hipLaunchKernelGGL(k_peer_publish, dim3(1), dim3(1024), 0, c->stream,
                       (const double*)(p->f_part.as<double>() + (size_t)(it & 1) * p->n_kf * p->f_maxl * kStride), p->n_kf,
                       p->f_maxl, blk + (gen & 1) * len, reinterpret_cast<unsigned long long*>(blk + 2 * len), gen);
    VX_LAUNCH_CHECK(c, "k_peer_publish");
    return VX_OK;
}
int peer_gather(vx_ctx* c, vx_ba_plan* p, unsigned long long gen) {
    const size_t len = peer_len(p);
    const int n = (int)p->peer_base.size();
    PeerPtrs pp{};
    if (n < 1 || n > kMaxPeers) return set_error(c, VX_ERR_STATE, "peer reduction: %d ranks", n);
    for (int r = 0; r < n; ++r) {
        const double* b = static_cast<const double*>(p->peer_base[r]);
        if (!b) return set_error(c, VX_ERR_STATE, "peer reduction: rank %d's block is not mapped", r);
        pp.rows[r] = b;
        pp.flag[r] = reinterpret_cast<const unsigned long long*>(b + 2 * len);
    }
    hipLaunchKernelGGL(k_peer_gather, dim3(1), dim3(1024), 0, c->stream, pp, n, (int)len, (int)((gen & 1) * len), gen,
                       p->f_rowpart.as<double>(), reinterpret_cast<int*>(p->state.as<uint8_t>() + offsetof(BAState, fault)));
    VX_LAUNCH_CHECK(c, "k_peer_gather");
    return VX_OK;
}
size_t peer_bytes(const vx_ba_plan* p) { return ((2 * peer_len(p) + 8) * sizeof(double) + 4095) & ~(size_t)4095; }

#ifndef VX_NO_RCCL
// this rank's block (uncached device memory: the peers read it over xGMI), its IPC handle gathered
// from every rank over RCCL, the peers' blocks opened; once per plan, at its first sharded run
int peer_setup(vx_ctx* c, vx_ba_plan* p) {
    const int n = p->shard_count, me = p->shard_rank;
    if (n > kMaxPeers) return set_error(c, VX_ERR_INVALID, "$VX_BA_PEER: at most %d ranks", kMaxPeers);
    if (c->nranks != n || c->rank != me)  // (the handle table is indexed by communicator rank)
        return set_error(c, VX_ERR_INVALID, "$VX_BA_PEER: shard %d of %d on communicator rank %d of %d", me, n, c->rank,
                         c->nranks);
    const size_t bytes = peer_bytes(p);
    VX_HIP(c, hipExtMallocWithFlags(&p->peer_mem, bytes, hipDeviceMallocUncached));
    VX_HIP(c, hipMemsetAsync(p->peer_mem, 0, bytes, c->stream));  // (flags 0 before any rank can read them)
    hipIpcMemHandle_t h;
    VX_HIP(c, hipIpcGetMemHandle(&h, p->peer_mem));
    DevBuf d;
    VX_HIP(c, d.ensure((size_t)n * sizeof h));
    VX_HIP(c, hipMemcpyAsync(d.as<uint8_t>() + (size_t)me * sizeof h, &h, sizeof h, hipMemcpyHostToDevice, c->stream));
    ncclResult_t r = ncclAllGather(d.as<uint8_t>() + (size_t)me * sizeof h, d.p, sizeof h, ncclUint8, c->comm, c->stream);
    if (r != ncclSuccess) return set_error(c, VX_ERR_COMM, "ncclAllGather (peer handles): %s", ncclGetErrorString(r));
    std::vector<hipIpcMemHandle_t> all(n);
    VX_HIP(c, hipMemcpyAsync(all.data(), d.p, (size_t)n * sizeof h, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    p->peer_base.assign(n, nullptr);
    for (int q = 0; q < n; ++q) {
        if (q == me) {
            p->peer_base[q] = p->peer_mem;
            continue;
        }
        void* ptr = nullptr;
        VX_HIP(c, hipIpcOpenMemHandle(&ptr, all[q], hipIpcMemLazyEnablePeerAccess));
        p->peer_opened.push_back(ptr);
        p->peer_base[q] = ptr;
    }
    p->peer = true;
    return VX_OK;
}
#endif

bool peer_requested() {
    const char* e = getenv("VX_BA_PEER");
    return e && e[0] == '1';
}

WinArgs make_win_args(vx_ba_plan* p) {
    uint8_t* W = p->f_win.as<uint8_t>();
    WinArgs w{};
    w.rows = reinterpret_cast<double*>(W + p->win_rows_off);
    w.cnt = reinterpret_cast<int*>(W + p->win_cnt_off);
    w.done = reinterpret_cast<int*>(W + p->win_done_off);
    w.nprod = reinterpret_cast<const int*>(W + p->win_nprod_off);
    w.gen = reinterpret_cast<int*>(W + p->win_gen_off);
    w.fault = reinterpret_cast<int*>(p->state.as<uint8_t>() + offsetof(BAState, fault));
    return w;
}

bool win_active(const vx_ba_plan* p) { return p->fused && p->f_persist && !p->win_off && p->shard_count <= 1; }

// the fused path: prologue (iteration 0's pose stage) + one k_ba_iter per iteration (sharded: each
// preceded by the row sums and their all-reduce), or the whole window as one k_ba_win launch
int plan_run_fused(vx_ctx* c, vx_ba_plan* p) {
    const BAArgs a = make_args(p);
    const FusedArgs f = make_fused_args(p);
    int rc;
    if ((rc = reset_if_no_iterations(c, p, a))) return rc;
    if (p->opt.max_iterations == 0) return VX_OK;
    if (win_active(p)) {
        constexpr int lds = (int)win_lds(kFTSmall);
        static std::atomic<uint64_t> dw{0};
        VX_HIP(c, lds_attr_once(c->device, reinterpret_cast<const void*>(&k_ba_win<kFTSmall>), lds, dw));
        VX_HIP(c, launch(c, kStBaWin, k_ba_win<kFTSmall>, dim3(p->f_blocks), dim3(kFTSmall), (uint32_t)lds, c->stream,
                         a, f, make_win_args(p)));
        return VX_OK;
    }
    if ((rc = fused_launch(c, p, a, f, -1))) return rc;
#ifndef VX_NO_RCCL
    if (p->shard_count > 1 && !p->peer && peer_requested() && (rc = peer_setup(c, p))) return rc;
#endif
    for (int it = 0; it < p->opt.max_iterations; ++it) {
        if (p->shard_count > 1 && p->peer) {  // the one-shot peer reduction
            const unsigned long long gen = ++p->peer_gen;
            if ((rc = peer_publish(c, p, it, gen)) || (rc = peer_gather(c, p, gen))) return rc;
        } else if (p->shard_count > 1) {
#ifndef VX_NO_RCCL
            if ((rc = fused_row_sum(c, p, it))) return rc;
            ProfScope ps(c, kStBaAllreduce);
            ncclResult_t r = ncclAllReduce(p->f_rowpart.p, p->f_rowpart.p, (size_t)p->n_kf * kStride, ncclDouble, ncclSum,
                                           c->comm, c->stream);
            if (r != ncclSuccess) return set_error(c, VX_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
#else
            return set_error(c, VX_ERR_COMM, "built without RCCL");
#endif
        }
        if ((rc = fused_launch(c, p, a, f, it))) return rc;
    }
    return VX_OK;
}

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
    }
    if (p->fused && (!sharded || p->fused_all)) {
        rc = plan_run_fused(c, p);
        if (!rc) p->ran = true;
        return rc;
    }
    if (!sharded && !p->choice_made) {
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

}  // namespace

size_t ba_state_bytes() { return sizeof(BAState); }

size_t ba_state_iter_offset() { return offsetof(BAState, iterations); }

void ba_state_to_stats(const void* host_state, vx_ba_stats* s) {
    const BAState& hs = *static_cast<const BAState*>(host_state);
    s->iterations = hs.iterations;
    for (int i = 0; i < 16; ++i) {
        s->cost[i] = hs.cost[i];
        s->obs[i] = hs.obs[i];
    }
}

// The iterations of a lean plan (ba_lean.hip): the two-kernel LDS path (k_pose_kf, k_landmark_solve)
// over capacity grids, the counts read from d.dyn on the device — no host synchronisation.
int ba_run_dyn(vx_ctx* c, const DynPlan& d) {
    BAArgs a{};
    a.n_kf = d.n_kf;
    a.n_opt = 0;  // (from dyn)
    a.n_lm = 0;
    a.min_pose_obs = d.opt.min_pose_observations;
    a.min_point_obs = d.opt.min_point_observations;
    a.max_iter = d.opt.max_iterations;
    a.huber = d.opt.huber_delta;
    a.max_err = d.opt.max_reproj_error;
    a.huber2 = a.huber * a.huber;
    a.max_err2 = a.max_err * a.max_err;
    a.kf_pose0 = d.kf_pose0;
    a.kf_pose = d.kf_pose;
    a.kf_intr = d.kf_intr;
    a.kf_rot = d.kf_rot;
    a.kf_flags = d.kf_flags;
    a.kf_obs_ptr = d.kf_obs_ptr;
    a.kf_part = d.kf_part;
    a.n_split = d.n_split;
    a.kf_cost = d.kf_cost;
    a.lm_pos0 = d.lm_pos0;
    a.lm_pos = d.lm_pos;
    a.pobs_uv = d.pobs_uv;
    a.pobs_lm = d.pobs_lm;
    a.lobs_ptr = d.lobs_ptr;
    a.lobs_kf = d.lobs_kf;
    a.lobs_lm = d.lobs_lm;
    a.lm_blk = d.lm_blk;
    a.lobs_uv = d.lobs_uv;
    a.state = static_cast<BAState*>(d.state);
    a.dyn = d.dyn;
    const size_t lds = (size_t)d.n_kf * kLdsStride * sizeof(double) + (size_t)kLmBlock * (9 * sizeof(double) + sizeof(int));
    if (lds > 64 * 1024) {
        static std::atomic<uint64_t> done{0};
        VX_HIP(c, lds_attr_once(c->device, reinterpret_cast<const void*>(&k_landmark_solve), 160 * 1024, done));
    }
    for (int it = 0; it < d.opt.max_iterations; ++it) {
        VX_HIP(c, launch(c, kStBaPose, k_pose_kf, dim3(d.n_kf * d.n_split), dim3(kPoseBlock), 0, c->stream, a, it));
        VX_HIP(c, launch(c, kStBaLandmark, k_landmark_solve, dim3(d.grid_blocks), dim3(kLmBlock), (uint32_t)lds,
                         c->stream, a, it));
    }
    return VX_OK;
}

namespace {
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

namespace vx {
// ba_lean.hip: vx_ba_optimize_map's one-call path (*fallback: the window needs a plan)
int lean_optimize_view(vx_ctx* c, vx_map_view* v, uint64_t ref, int has_ref, const vx_ba_options& o, vx_ba_stats* st,
                       bool* fallback);
}  // namespace vx

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
    auto* p = plan_new(c);
    p->opt = *opt;
    p->shard_rank = shard_rank;
    p->shard_count = shard_count;
    p->global_poses = (flags & VX_PLAN_GLOBAL_POSES) != 0;
    int rc = plan_fault_injected(c);
    if (!rc) rc = (flags & VX_PLAN_HOST_BUILD) ? build_plan(c, m, ref, has_ref, p) : build_plan_device(c, m, ref, has_ref, p);
    if (rc) {
        vx_ba_plan_destroy(p);  // (also leaves c->plan_live)
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
    auto* p = plan_new(c);
    p->opt = *opt;
    p->shard_rank = shard_rank;
    p->shard_count = shard_count;
    p->from_dmap = true;
    int rc = plan_fault_injected(c);
    if (!rc) rc = build_plan_dmap(c, m, ref, has_ref, p);
    if (rc) {
        vx_ba_plan_destroy(p);  // (also leaves c->plan_live)
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
    if (win_active(p)) {  // (a persistent run whose waits ran out is void: run it again first)
        int fault = 0;
        VX_HIP(c, hipMemcpyAsync(&fault, p->state.as<uint8_t>() + offsetof(BAState, fault), sizeof fault,
                                 hipMemcpyDeviceToHost, c->stream));
        VX_HIP(c, hipStreamSynchronize(c->stream));
        if (fault) {
            p->win_off = true;
            p->graph.reset();
            VX_HIP(c, hipMemsetAsync(p->state.as<uint8_t>() + offsetof(BAState, fault), 0, sizeof(int), c->stream));
            if (int rc = plan_run(c, p)) return rc;
        }
    }
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
    if (p->status != 0) return plan_run(c, p);
    // Sharded plans: the first run is eager (its one small all-reduce fixes the kernel set on every
    // rank and synchronises); later runs replay ONE hipGraph of the whole sequence, the per-iteration
    // k_row_sum -> ncclAllReduce -> k_ba_iter chain included (RCCL collectives are capturable: the
    // graph holds their kernels).  A capture that fails leaves the plan eager; $VX_SHARDED_GRAPHS=0
    // keeps every sharded run eager, and so does the peer reduction ($VX_BA_PEER=1).
    if (p->shard_count > 1) {
        const char* e = std::getenv("VX_SHARDED_GRAPHS");
        // (the peer reduction stays eager: its generations change from run to run)
        if (!p->choice_made || p->graph_eager || p->peer || peer_requested() || (e && e[0] == '0')) return plan_run(c, p);
        const bool capturing = c->use_graphs && !c->prof && p->graph.seen && !p->graph.exec;
        p->ran = true;
        const int rc =
            graph_run_owned(c, p->graph, [](vx_ctx* cc, void* v) { return plan_run(cc, static_cast<vx_ba_plan*>(v)); }, p);
        if (rc != VX_OK && capturing) {
            p->graph_eager = true;
            return plan_run(c, p);
        }
        return rc;
    }
    p->ran = true;
    // the persistent window is ONE kernel: launched directly (a graph launch of one kernel node costs
    // the host more and the stream extra packets, $VX_BA_WIN_GRAPH=1 for it)
    static const bool win_graph = [] {
        const char* e = std::getenv("VX_BA_WIN_GRAPH");
        return e && e[0] == '1';
    }();
    if (win_active(p) && !win_graph && !c->prof) return plan_run(c, p);
    return graph_run_owned(c, p->graph, [](vx_ctx* cc, void* v) { return plan_run(cc, static_cast<vx_ba_plan*>(v)); }, p);
}

namespace {
int shard_emulate_enqueue(vx_ctx* c, vx_ba_plan* const* plans, int n);
struct EmuArgs {
    vx_ba_plan* const* plans;
    int n;
};
}  // namespace

// The emulated sharded run goes through the context's graph cache like a real sharded run's
// sequence: eager on its first sighting, captured on the second, replayed afterwards (keyed by the
// shard plans), so the tests exercise the captured form of the row sum -> reduction -> k_ba_iter chain.
int vx_ba_shard_emulate_run(vx_ctx* c, vx_ba_plan* const* plans, int n) {
    if (!c || !plans || n < 1 || n > kMaxEmuShards) return c ? set_error(c, VX_ERR_INVALID, "vx_ba_shard_emulate_run: bad arguments") : VX_ERR_INVALID;
    for (int r = 0; r < n; ++r)
        if (!plans[r] || plans[r]->c != c) return set_error(c, VX_ERR_INVALID, "shard %d: plan of another context", r);
    std::vector<uint64_t> key{0xE3u, (uint64_t)n};
    for (int r = 0; r < n; ++r) key.push_back((uint64_t)(uintptr_t)plans[r]);
    EmuArgs ea{plans, n};
    // (eager: the first run decides the kernels; the peer reduction's generations change every run)
    if (plans[0]->status != 0 || !plans[0]->choice_made || peer_requested()) return shard_emulate_enqueue(c, plans, n);
    for (int r = 0; r < n; ++r) plans[r]->ran = true;
    return graph_run(c, key, [](vx_ctx* cc, void* v) {
        const EmuArgs* x = static_cast<const EmuArgs*>(v);
        return shard_emulate_enqueue(cc, x->plans, x->n);
    }, &ea);
}

namespace {
int shard_emulate_enqueue(vx_ctx* c, vx_ba_plan* const* plans, int n) {
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
    bool all_fused = true;
    for (int r = 0; r < n; ++r) {
        blocks = std::max(blocks, plans[r]->n_lm_blocks);
        max_obs = std::max(max_obs, plans[r]->max_lm_obs);
        all_fused = all_fused && plans[r]->fused;
    }
    int rc;
    if (all_fused) {  // fused path: row sums of every shard summed in rank order in place of the all-reduce
        PartPtrs rows{};
        std::vector<BAArgs> args(n);
        std::vector<FusedArgs> fargs(n);
        for (int r = 0; r < n; ++r) {
            plans[r]->fused_all = true;
            plans[r]->choice_made = true;
            rows.p[r] = plans[r]->f_rowpart.as<double>();
            args[r] = make_args(plans[r]);
            fargs[r] = make_fused_args(plans[r]);
            if ((rc = reset_if_no_iterations(c, plans[r], args[r]))) return rc;
        }
        const long long len = (long long)p0->n_kf * kStride;
        // $VX_BA_PEER=1: the peer reduction's kernels in place of k_sum_parts, each shard's block in
        // device memory of its own and every shard's base table naming all of them (the IPC mapping
        // of a real multi-GPU run), generations as a real run counts them
        const bool peer = peer_requested();
        if (peer) {
            for (int r = 0; r < n; ++r)
                if (!plans[r]->peer_mem) {
                    VX_HIP(c, hipMalloc(&plans[r]->peer_mem, peer_bytes(plans[r])));
                    VX_HIP(c, hipMemsetAsync(plans[r]->peer_mem, 0, peer_bytes(plans[r]), c->stream));
                }
            for (int r = 0; r < n; ++r) {  // (every block allocated before any table names it)
                plans[r]->peer_base.assign(n, nullptr);
                for (int q = 0; q < n; ++q) plans[r]->peer_base[q] = plans[q]->peer_mem;
            }
        }
        if (p0->opt.max_iterations > 0)
            for (int r = 0; r < n; ++r)
                if ((rc = fused_launch(c, plans[r], args[r], fargs[r], -1))) return rc;
        for (int it = 0; it < p0->opt.max_iterations; ++it) {
            if (peer) {
                const unsigned long long gen = p0->peer_gen + 1;
                for (int r = 0; r < n; ++r) {
                    plans[r]->peer_gen = gen;
                    if ((rc = peer_publish(c, plans[r], it, gen))) return rc;
                }
                for (int r = 0; r < n; ++r)
                    if ((rc = peer_gather(c, plans[r], gen))) return rc;
            } else {
                for (int r = 0; r < n; ++r)
                    if ((rc = fused_row_sum(c, plans[r], it))) return rc;
                hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, c->stream, rows, n, len);
                VX_LAUNCH_CHECK(c, "k_sum_parts");
            }
            for (int r = 0; r < n; ++r)
                if ((rc = fused_launch(c, plans[r], args[r], fargs[r], it))) return rc;
        }
        for (int r = 0; r < n; ++r) plans[r]->ran = true;
        return VX_OK;
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
}  // namespace

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
        // one synchronisation: the state, BOTH pose parities (the last iteration's is known only from
        // the state) and the positions into one host-cached pinned block
        const size_t sb = sizeof(BAState), pb = 2 * (size_t)p->n_kf * 8 * sizeof(double),
                     lb = (size_t)p->n_opt * 4 * sizeof(double);
        const size_t o_pose = (sb + 63) & ~(size_t)63, o_lm = o_pose + ((pb + 63) & ~(size_t)63);
        VX_HIP(c, p->fetch_host.ensure(o_lm + lb + 64, true));
        uint8_t* H = static_cast<uint8_t*>(p->fetch_host.p);
        auto read_back = [&]() -> int {
            VX_HIP(c, hipMemcpyAsync(H, p->state.p, sb, hipMemcpyDeviceToHost, c->stream));
            VX_HIP(c, hipMemcpyAsync(H + o_pose, p->kf_pose.p, pb, hipMemcpyDeviceToHost, c->stream));
            if (lb) VX_HIP(c, hipMemcpyAsync(H + o_lm, p->lm_pos.p, lb, hipMemcpyDeviceToHost, c->stream));
            VX_HIP(c, hipStreamSynchronize(c->stream));
            return VX_OK;
        };
        int rc = read_back();
        if (rc) return rc;
        BAState hs;
        std::memcpy(&hs, H, sb);
        if (hs.fault && !p->peer_base.empty() && p->shard_count > 1)
            return set_error(c, VX_ERR_COMM, "peer reduction: a rank's row sums did not arrive within 200 ms");
        if (hs.fault && win_active(p)) {
            // a persistent window whose wait ran out (its workgroups could not all be resident at
            // once): the run is void; the plan keeps the per-iteration launches from now on and
            // runs the window again
            p->win_off = true;
            p->graph.reset();
            VX_HIP(c, hipMemsetAsync(p->state.as<uint8_t>() + offsetof(BAState, fault), 0, sizeof(int), c->stream));
            if ((rc = plan_run(c, p))) return rc;
            if ((rc = read_back())) return rc;
            std::memcpy(&hs, H, sb);
        }
        // the poses of the last iteration run are in ping-pong buffer (iterations & 1)
        const double* pose = reinterpret_cast<const double*>(H + o_pose) + (size_t)(hs.iterations & 1) * p->n_kf * 8;
        const double* lm = reinterpret_cast<const double*>(H + o_lm);
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
    if (!p) return;
    vx_ctx* c = p->c;
    if (c) {
        auto& live = c->plan_live;
        live.erase(std::remove(live.begin(), live.end(), p), live.end());
        // captured emulated sharded sequences naming this plan (vx_ba_shard_emulate_run's keys
        // {0xE3, n, plans...}) bake its buffers in: drop them before the address can be reused
        auto& ge = c->graphs.entries;
        for (auto it = ge.begin(); it != ge.end();) {
            const bool names = !it->key.empty() && it->key[0] == 0xE3u &&
                               std::find(it->key.begin() + 2, it->key.end(), (uint64_t)(uintptr_t)p) != it->key.end();
            if (names) {
                if (it->exec) (void)hipGraphExecDestroy(it->exec);
                it = ge.erase(it);
            } else {
                ++it;
            }
        }
        if (c->plan_husks.size() < kMaxPlanHusks) {  // park the buffers (no hipFree)
            auto* h = new vx_ba_plan();
            adopt_buffers(h, p);
            c->plan_husks.push_back(h);
        }
    }
    for (void* q : p->peer_opened) (void)hipIpcCloseMemHandle(q);
    if (p->peer_mem) (void)hipFree(p->peer_mem);
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

int vx_ba_plan_layout(const vx_ba_plan* p, int64_t* out4) {
    if (!p || !out4) return VX_ERR_INVALID;
    out4[0] = p->fused ? 1 : 0;
    out4[1] = p->fused ? p->f_threads : 0;
    out4[2] = p->fused ? p->f_blocks : 0;
    out4[3] = p->fused ? p->f_maxl : 0;
    return VX_OK;
}

int vx_ba_plan_persistent(const vx_ba_plan* p) { return p && win_active(p) ? 1 : 0; }

int vx_ba_plan_fused_tables(vx_ctx* c, const vx_ba_plan* p, void* dst, size_t cap, size_t* bytes) {
    if (!c || !p || !bytes || p->c != c) return VX_ERR_INVALID;
    if (!p->fused) return set_error(c, VX_ERR_STATE, "plan has no fused layout");
    const FusedOffsets& F = p->f_off;
    const size_t n_lp = (size_t)p->f_blocks * p->f_threads;
    const std::pair<size_t, size_t> part[] = {
        {F.blk, (size_t)p->f_blocks * fused_blk_ints(p->f_threads) * 4},
        {F.lm_slot, n_lp * 4},
        {F.lm_run, n_lp * 8},
        {F.lobs_rec, n_lp * 16},
        {F.kent, (size_t)p->f_blocks * kFK * 32},
        {F.lobs_src, n_lp * 4},
        {F.pobs_src, p->f_npp * 4},
        {F.pobs_code, p->f_npp * 4}};
    size_t total = 0;
    for (const auto& x : part) total += x.second;
    *bytes = total;
    if (!dst) return VX_OK;
    if (cap < total) return VX_ERR_CAPACITY;
    VX_HIP(c, hipSetDevice(c->device));
    size_t at = 0;
    for (const auto& x : part) {
        if (x.second)
            VX_HIP(c, hipMemcpyAsync(static_cast<uint8_t*>(dst) + at, p->f_tab.as<uint8_t>() + x.first, x.second,
                                     hipMemcpyDeviceToHost, c->stream));
        at += x.second;
    }
    VX_HIP(c, hipStreamSynchronize(c->stream));
    return VX_OK;
}

int vx_ba_optimize_map(vx_ctx* c, vx_map_view* m, uint64_t ref, int has_ref, const vx_ba_options* opt,
                       vx_ba_stats* st) {
    if (!c) return VX_ERR_INVALID;
    // ($VX_OPT_TIMING=1: the call's phases on stderr, scripts/adapter_timing.py)
    static const bool timing = getenv("VX_OPT_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (timing)
            std::fprintf(stderr, "[vx optmap] %s %.1f us\n", what,
                         std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    };
    // the lean one-call build on the view loaded into the context's scratch map for windows of up to
    // 64 keyframes; the plan below for larger ones (C3, 50: 0.37 against 0.62 ms; C4, 100: the plan's
    // fused window wins, 0.93 against 1.20 ms, profiles/r06/bench_c4_r06.json) and for a window the
    // lean build does not take.  $VX_OPTMAP_LEAN=0 / 1: always the plan / the lean build (A/B runs)
    static const int lean_env = [] {
        const char* e = getenv("VX_OPTMAP_LEAN");
        return e ? (e[0] == '0' ? 0 : 1) : -1;
    }();
    const bool lean = m && opt && opt->max_iterations >= 0 && opt->max_iterations <= 64 &&
                      (lean_env == 1 || (lean_env < 0 && std::min(opt->window_size, m->n_kf) <= 64));
    if (lean) {
        bool fb = false;
        const int rc = lean_optimize_view(c, m, ref, has_ref, *opt, st, &fb);
        lap("lean");
        if (!fb) return rc;
    }
    vx_ba_plan* p = nullptr;
    int rc = vx_ba_plan_create(c, m, ref, has_ref, opt, 0, 1, &p);
    lap("plan_create");
    if (rc) return rc;
    rc = vx_ba_plan_run_async(c, p);
    if (timing) (void)hipStreamSynchronize(c->stream);
    lap("run");
    if (!rc) rc = vx_ba_plan_fetch(c, p, m, st);
    lap("fetch");
    (void)hipStreamSynchronize(c->stream);
    vx_ba_plan_destroy(p);
    lap("destroy");
    return rc;
}

}  // extern "C"
