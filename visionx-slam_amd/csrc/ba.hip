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
//     k_pose_kf        one workgroup per keyframe: each thread projects its observations
//                      (ProjectToPixel, projection.h:11-31), gates, weights and accumulates the
//                      21 + 6 + 2 normal-equation terms of the 2x6 PoseJacobian in registers; one
//                      fixed-order workgroup reduction writes the keyframe's 29-term block
//     [sharded only]   ncclAllReduce(sum, f64) of the per-keyframe blocks over the landmark
//                      shards (one collective per iteration, 32 doubles per keyframe)
//     k_landmark_solve every workgroup first solves ALL window keyframes redundantly (one lane per
//                      keyframe: H += 1e-6 I, Eigen-style pivoted LDLT, finite check, T <- exp(dx) T)
//                      into LDS — bitwise identical in every workgroup — then runs one landmark
//                      per thread (2x3 Jacobian Jp*R, 3x3 normal equations, LDLT, p += dp) against
//                      those poses; workgroup 0 publishes the poses and evaluates the stop rule.
//                      Windows beyond kMaxKfLds keyframes use k_pose_solve_g + k_landmark instead.
// The step keeps the reference's sign (b = -J^T e, :156 and :224): this is a drop-in, not a fix.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "vx_internal.hpp"

namespace vx {
namespace {

constexpr int kPoseBlock = 256;  // threads per keyframe workgroup
constexpr int kNTerms = 29;      // 21 H (upper) + 6 b + cost + count
constexpr int kStride = 32;      // doubles per keyframe block
constexpr int kMaxIter = 64;
constexpr int kMaxKfLds = 512;   // keyframes whose poses fit the LDS of k_landmark_solve

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
    int min_pose_obs, min_point_obs, max_iter, pad1;
    double huber, max_err;
    const double* kf_pose0;  // 8 per KF: qx qy qz qw tx ty tz 0
    double* kf_pose;         // 2 x n_kf x 8: ping-pong by iteration parity (see pose_in / pose_out)
    const double* kf_intr;   // 4 per KF
    double* kf_rot;          // 9 per KF (rotation matrix of the current pose)
    const int* kf_flags;     // bit0: keyframe has a camera
    const int* kf_obs_ptr;   // n_kf + 1, CSR into the pose observations
    double* kf_sums;         // n_kf * kStride normal-equation blocks (all-reduced when sharded)
    double* kf_cost;         // 2 per KF: pose-stage cost and observation count
    const double* lm_pos0;   // 4 per landmark
    double* lm_pos;
    const double2* pobs_uv;
    const int* pobs_lm;
    const int* lobs_ptr;     // n_opt + 1
    const int* lobs_kf;
    const double2* lobs_uv;
    BAState* state;
};

struct D3 { double x, y, z; };

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

__device__ __forceinline__ D3 cross3(D3 a, D3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// Eigen _transformVector + translation (Sophus SE3 * point)
__device__ __forceinline__ D3 se3_apply(const double* T, D3 p) {
    const D3 qv{T[0], T[1], T[2]};
    D3 uv = cross3(qv, p);
    uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
    const D3 c = cross3(qv, uv);
    const double w = T[3];
    return {p.x + w * uv.x + c.x + T[4], p.y + w * uv.y + c.y + T[5], p.z + w * uv.z + c.z + T[6]};
}

// Eigen Quaternion::toRotationMatrix
__device__ __forceinline__ void rot_from_quat(const double* q, double* R) {
    const double tx = 2.0 * q[0], ty = 2.0 * q[1], tz = 2.0 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

// Eigen::LDLT (lower, diagonal pivoting) compute + solve, row-major N x N in registers.  The
// pivot permutation is data dependent; every swap is written with compile-time indices under a
// runtime predicate so the matrix stays in VGPRs (no scratch).
template <int N>
__device__ __forceinline__ void ldlt_solve(double* A, const double* b, double* x) {
    int tr[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        int big = k;
        double bv = fabs(A[k * N + k]);
#pragma unroll
        for (int i = k + 1; i < N; ++i) {
            const double v = fabs(A[i * N + i]);
            if (v > bv) { bv = v; big = i; }
        }
        tr[k] = big;
#pragma unroll
        for (int bi = k + 1; bi < N; ++bi) {
            if (bi == big) {
#pragma unroll
                for (int j = 0; j < k; ++j) { const double t = A[k * N + j]; A[k * N + j] = A[bi * N + j]; A[bi * N + j] = t; }
#pragma unroll
                for (int i = bi + 1; i < N; ++i) { const double t = A[i * N + k]; A[i * N + k] = A[i * N + bi]; A[i * N + bi] = t; }
                { const double t = A[k * N + k]; A[k * N + k] = A[bi * N + bi]; A[bi * N + bi] = t; }
#pragma unroll
                for (int i = k + 1; i < bi; ++i) { const double t = A[i * N + k]; A[i * N + k] = A[bi * N + i]; A[bi * N + i] = t; }
            }
        }
        if (k > 0) {
            double temp[N];
#pragma unroll
            for (int j = 0; j < k; ++j) temp[j] = A[j * N + j] * A[k * N + j];
            double s = 0;
#pragma unroll
            for (int j = 0; j < k; ++j) s += A[k * N + j] * temp[j];
            A[k * N + k] -= s;
#pragma unroll
            for (int i = k + 1; i < N; ++i) {
                double t = 0;
#pragma unroll
                for (int j = 0; j < k; ++j) t += A[i * N + j] * temp[j];
                A[i * N + k] -= t;
            }
        }
        const double akk = A[k * N + k];
        if (fabs(akk) > 0.0) {
#pragma unroll
            for (int i = k + 1; i < N; ++i) A[i * N + k] /= akk;
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = b[i];
#pragma unroll
    for (int k = 0; k < N; ++k)
#pragma unroll
        for (int bi = k + 1; bi < N; ++bi)
            if (tr[k] == bi) { const double t = x[k]; x[k] = x[bi]; x[bi] = t; }
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int r = i + 1; r < N; ++r) x[r] -= x[i] * A[r * N + i];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double d = A[i * N + i];
        x[i] = fabs(d) > 2.2250738585072014e-308 ? x[i] / d : 0.0;
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        double s = 0;
#pragma unroll
        for (int j = i + 1; j < N; ++j) s += A[j * N + i] * x[j];
        x[i] -= s;
    }
#pragma unroll
    for (int k = N - 1; k >= 0; --k)
#pragma unroll
        for (int bi = k + 1; bi < N; ++bi)
            if (tr[k] == bi) { const double t = x[k]; x[k] = x[bi]; x[bi] = t; }
}

// upper-triangle index of the 6x6 pose Hessian
__device__ __forceinline__ int hidx(int i, int j) {  // i <= j
    return i * 6 - (i * (i - 1)) / 2 + (j - i);
}

// Sophus SE3::exp(dx) * T, written into T (8 doubles)
__device__ void se3_left_update(const double* dx, double* T) {
    const double eps = 1e-10;  // Sophus::Constants<double>::epsilon()
    const double wx = dx[3], wy = dx[4], wz = dx[5];
    const double theta_sq = wx * wx + wy * wy + wz * wz;
    double theta, imag, real;
    if (theta_sq < eps * eps) {
        theta = 0.0;
        const double t4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * t4;
        real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * t4;
    } else {
        theta = sqrt(theta_sq);
        const double half = 0.5 * theta;
        imag = sin(half) / theta;
        real = cos(half);
    }
    const double eq[4] = {imag * wx, imag * wy, imag * wz, real};
    const double O[9] = {0, -wz, wy, wz, 0, -wx, -wy, wx, 0};
    double V[9];
    if (theta < eps) {
        rot_from_quat(eq, V);
    } else {
        double O2[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                O2[3 * r + c] = O[3 * r] * O[c] + O[3 * r + 1] * O[3 + c] + O[3 * r + 2] * O[6 + c];
        const double c1 = (1.0 - cos(theta)) / theta_sq;
        const double c2 = (theta - sin(theta)) / (theta_sq * theta);
#pragma unroll
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c1 * O[i] + c2 * O2[i];
    }
    const double et[3] = {V[0] * dx[0] + V[1] * dx[1] + V[2] * dx[2], V[3] * dx[0] + V[4] * dx[1] + V[5] * dx[2],
                          V[6] * dx[0] + V[7] * dx[1] + V[8] * dx[2]};
    // q <- normalize(eq * q)   (Sophus SO3 product + normalize)
    const double ax = eq[0], ay = eq[1], az = eq[2], aw = eq[3];
    const double bx = T[0], by = T[1], bz = T[2], bw = T[3];
    const double q[4] = {aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                         aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz};
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    // t <- et + rotate(eq, t)
    const double rt[8] = {eq[0], eq[1], eq[2], eq[3], 0, 0, 0, 0};
    const D3 r = se3_apply(rt, {T[4], T[5], T[6]});
    T[0] = q[0] / n; T[1] = q[1] / n; T[2] = q[2] / n; T[3] = q[3] / n;
    T[4] = et[0] + r.x; T[5] = et[1] + r.y; T[6] = et[2] + r.z;
}

// Pose step of one keyframe from its summed terms S (local_ba.cpp:163-173): skipped below
// min_pose_observations or without a camera; T updated in place, R = its rotation (:173, :220).
__device__ __forceinline__ void solve_pose(const BAArgs& a, int k, const double* S, double* T, double* R) {
    const int obs = (int)S[28];
    if (obs >= a.min_pose_obs && (a.kf_flags[k] & 1)) {
        double H[36], b[6], dx[6];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = 0; c < 6; ++c) H[6 * r + c] = r <= c ? S[hidx(r, c)] : S[hidx(c, r)];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            H[7 * r] += 1e-6;
            b[r] = S[21 + r];
        }
        ldlt_solve<6>(H, b, dx);
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

// Pose stage (local_ba.cpp:116-161): one workgroup per keyframe.  Each thread accumulates the 29
// terms of its observations (strided) in registers; a fixed-order wave butterfly + LDS tree
// reduces them into kf_sums[k].
__global__ __launch_bounds__(kPoseBlock) void k_pose_kf(BAArgs a, int it) {
    if (it > 0 && !a.state->active[it]) return;
    __shared__ double red[kPoseBlock / 64][kNTerms];
    const int k = blockIdx.x;
    const int i0 = a.kf_obs_ptr[k], i1 = a.kf_obs_ptr[k + 1];
    const double* Tin = pose_in(a, it);
    double T[8], C[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) T[j] = Tin[8 * k + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) C[j] = a.kf_intr[4 * k + j];
    const double fx = C[0], fy = C[1];
    double v[kNTerms];
#pragma unroll
    for (int t = 0; t < kNTerms; ++t) v[t] = 0.0;
#pragma unroll 2
    for (int i = i0 + (int)threadIdx.x; i < i1; i += kPoseBlock) {
        const int s = a.pobs_lm[i];
        const double2 uv = a.pobs_uv[i];
        const double* P = lm_in(a, it, s);
        const D3 pc = se3_apply(T, {P[0], P[1], P[2]});
        if (!(pc.z > 1e-6)) continue;
        const double inv_z = 1.0 / pc.z;
        const double x = pc.x * inv_z, y = pc.y * inv_z;
        const double e0 = uv.x - (fx * x + C[2]);
        const double e1 = uv.y - (fy * y + C[3]);
        const double en = sqrt(e0 * e0 + e1 * e1);
        if (en > a.max_err) continue;
        const double w = en <= a.huber ? 1.0 : a.huber / en;
        const double z = pc.z, z2 = z * z;
        const double jp0 = fx / z, jp2 = -fx * pc.x / z2, jp4 = fy / z, jp5 = -fy * pc.y / z2;
        // J = Jp * [I | -hat(pc)] (local_ba.cpp:26-33), formed as the 2x3 * 3x6 product
        const double Jp[6] = {jp0, 0.0, jp2, 0.0, jp4, jp5};
        const double S[18] = {1, 0, 0, 0, pc.z, -pc.y, 0, 1, 0, -pc.z, 0, pc.x, 0, 0, 1, pc.y, -pc.x, 0};
        double J0[6], J1[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            J0[c] = Jp[0] * S[c] + Jp[1] * S[6 + c] + Jp[2] * S[12 + c];
            J1[c] = Jp[3] * S[c] + Jp[4] * S[6 + c] + Jp[5] * S[12 + c];
        }
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = r; c < 6; ++c) v[hidx(r, c)] += (w * J0[r]) * J0[c] + (w * J1[r]) * J1[c];
#pragma unroll
        for (int r = 0; r < 6; ++r) v[21 + r] += w * ((-J0[r]) * e0 + (-J1[r]) * e1);
        v[27] += w * (e0 * e0 + e1 * e1);
        v[28] += 1.0;
    }
#pragma unroll
    for (int t = 0; t < kNTerms; ++t) {
        double x = v[t];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        v[t] = x;
    }
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
#pragma unroll
        for (int t = 0; t < kNTerms; ++t) red[wv][t] = v[t];
    }
    __syncthreads();
    if (threadIdx.x < kStride) {
        double s = 0.0;
        if (threadIdx.x < kNTerms) {
            s = red[0][threadIdx.x];
#pragma unroll
            for (int w2 = 1; w2 < kPoseBlock / 64; ++w2) s += red[w2][threadIdx.x];
        }
        a.kf_sums[(long long)k * kStride + threadIdx.x] = s;
    }
}

// Landmark step of landmark l (local_ba.cpp:176-238) against keyframe tables T/R/C (LDS or
// global memory).
__device__ __forceinline__ void landmark_step(const BAArgs& a, int it, int l, const double* sT,
                                              const double* sR, const double* sC) {
    const double* Pin = lm_in(a, it, l);
    double* Pp = a.lm_pos + 4 * l;
    const D3 P{Pin[0], Pin[1], Pin[2]};
    double h00 = 0, h01 = 0, h02 = 0, h11 = 0, h12 = 0, h22 = 0, b0 = 0, b1 = 0, b2 = 0;
    int obs = 0;
    for (int o = a.lobs_ptr[l]; o < a.lobs_ptr[l + 1]; ++o) {
        const int k = a.lobs_kf[o];
        const double2 uv = a.lobs_uv[o];
        const double* T = sT + 8 * k;
        const double* C = sC + 4 * k;
        const D3 pc = se3_apply(T, P);
        if (!(pc.z > 1e-6)) continue;
        const double inv_z = 1.0 / pc.z;
        const double x = pc.x * inv_z, y = pc.y * inv_z;
        const double fx = C[0], fy = C[1];
        const double e0 = uv.x - (fx * x + C[2]);
        const double e1 = uv.y - (fy * y + C[3]);
        const double en = sqrt(e0 * e0 + e1 * e1);
        if (en > a.max_err) continue;
        const double w = en <= a.huber ? 1.0 : a.huber / en;
        const double z = pc.z, z2 = z * z;
        const double jp0 = fx / z, jp2 = -fx * pc.x / z2, jp4 = fy / z, jp5 = -fy * pc.y / z2;
        const double* R = sR + 9 * k;
        double J0[3], J1[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            J0[c] = jp0 * R[c] + 0.0 * R[3 + c] + jp2 * R[6 + c];
            J1[c] = 0.0 * R[c] + jp4 * R[3 + c] + jp5 * R[6 + c];
        }
        h00 += (w * J0[0]) * J0[0] + (w * J1[0]) * J1[0];
        h01 += (w * J0[0]) * J0[1] + (w * J1[0]) * J1[1];
        h02 += (w * J0[0]) * J0[2] + (w * J1[0]) * J1[2];
        h11 += (w * J0[1]) * J0[1] + (w * J1[1]) * J1[1];
        h12 += (w * J0[1]) * J0[2] + (w * J1[1]) * J1[2];
        h22 += (w * J0[2]) * J0[2] + (w * J1[2]) * J1[2];
        b0 += w * ((-J0[0]) * e0 + (-J1[0]) * e1);
        b1 += w * ((-J0[1]) * e0 + (-J1[1]) * e1);
        b2 += w * ((-J0[2]) * e0 + (-J1[2]) * e1);
        ++obs;
    }
    D3 out = P;  // skipped landmarks keep their position (written anyway: iteration 0 reads lm_pos0)
    if (obs >= a.min_point_obs) {
        double H[9] = {h00 + 1e-6, h01, h02, h01, h11 + 1e-6, h12, h02, h12, h22 + 1e-6};
        const double b[3] = {b0, b1, b2};
        double dp[3];
        ldlt_solve<3>(H, b, dp);
        if (isfinite(dp[0]) && isfinite(dp[1]) && isfinite(dp[2])) out = {P.x + dp[0], P.y + dp[1], P.z + dp[2]};
    }
    Pp[0] = out.x;
    Pp[1] = out.y;
    Pp[2] = out.z;
}

// Pose solve of every window keyframe (redundantly in each workgroup) + landmark stage, one launch.
__global__ __launch_bounds__(256) void k_landmark_solve(BAArgs a, int it) {
    if (it > 0 && !a.state->active[it]) return;
    extern __shared__ __attribute__((aligned(16))) double kf_lds[];  // n_kf x (8 T + 9 R + 4 C)
    double* sT = kf_lds;
    double* sR = kf_lds + 8 * a.n_kf;
    double* sC = sR + 9 * a.n_kf;
    const int tid = threadIdx.x;
    const double* Tin = pose_in(a, it);
    double* Tout = pose_out(a, it);
    for (int k = tid; k < a.n_kf; k += blockDim.x) {
        double S[kStride];
#pragma unroll
        for (int t = 0; t < kNTerms; ++t) S[t] = a.kf_sums[(long long)k * kStride + t];
        double T[8], R[9];
#pragma unroll
        for (int j = 0; j < 8; ++j) T[j] = Tin[8 * k + j];
        solve_pose(a, k, S, T, R);
#pragma unroll
        for (int j = 0; j < 8; ++j) sT[8 * k + j] = T[j];
#pragma unroll
        for (int j = 0; j < 9; ++j) sR[9 * k + j] = R[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) sC[4 * k + j] = a.kf_intr[4 * k + j];
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
    if (blockIdx.x == 0 && tid < 64) totals_and_stop(a, it, tid);
    const int l = blockIdx.x * blockDim.x + tid;
    if (l < a.n_opt) landmark_step(a, it, l, sT, sR, sC);
}

// Large-window fallback (n_kf > kMaxKfLds): one thread per keyframe solves into global memory...
__global__ __launch_bounds__(256) void k_pose_solve_g(BAArgs a, int it) {
    if (it > 0 && !a.state->active[it]) return;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n_kf) return;
    double S[kStride];
#pragma unroll
    for (int t = 0; t < kNTerms; ++t) S[t] = a.kf_sums[(long long)k * kStride + t];
    const double* Tin = pose_in(a, it);
    double* Tout = pose_out(a, it);
    double T[8], R[9];
#pragma unroll
    for (int j = 0; j < 8; ++j) T[j] = Tin[8 * k + j];
    solve_pose(a, k, S, T, R);
#pragma unroll
    for (int j = 0; j < 8; ++j) Tout[8 * k + j] = T[j];
#pragma unroll
    for (int j = 0; j < 9; ++j) a.kf_rot[9 * k + j] = R[j];
    a.kf_cost[2 * k] = S[27];
    a.kf_cost[2 * k + 1] = S[28];
}

// ... and the landmark stage reads the poses from global memory; wave 0 of block 0 evaluates
// the stop rule (active[it + 1] is read by no block of this launch).
__global__ __launch_bounds__(256) void k_landmark(BAArgs a, int it) {
    if (it > 0 && !a.state->active[it]) return;
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 64) totals_and_stop(a, it, threadIdx.x);
    if (l < a.n_opt) landmark_step(a, it, l, pose_out(a, it), a.kf_rot, a.kf_intr);
}

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

}  // namespace
}  // namespace vx

struct vx_ba_plan {
    vx_ctx* c = nullptr;
    vx_ba_options opt{};
    int status = 1;
    int shard_rank = 0, shard_count = 1;
    int n_window_kf = 0, n_landmarks_global = 0;
    int n_kf = 0, n_opt = 0, n_lm = 0;
    int64_t n_pose_obs = 0, n_lm_obs = 0;
    std::vector<int> kf_map_idx, lm_map_idx;
    vx::DevBuf kf_pose0, kf_pose, kf_intr, kf_rot, kf_flags, kf_obs_ptr, kf_sums, kf_cost, lm_pos0, lm_pos,
        pobs_uv, pobs_lm, lobs_ptr, lobs_kf, lobs_uv, state;
    bool ran = false;
};

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
    a.kf_sums = p->kf_sums.as<double>();
    a.kf_cost = p->kf_cost.as<double>();
    a.lm_pos0 = p->lm_pos0.as<double>();
    a.lm_pos = p->lm_pos.as<double>();
    a.pobs_uv = p->pobs_uv.as<double2>();
    a.pobs_lm = p->pobs_lm.as<int>();
    a.lobs_ptr = p->lobs_ptr.as<int>();
    a.lobs_kf = p->lobs_kf.as<int>();
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

int build_plan(vx_ctx* c, const vx_map_view* m, uint64_t ref_kf_id, int has_ref, vx_ba_plan* p,
               bool device = true) {
    const vx_ba_options& o = p->opt;
    p->status = 1;
    if (!m || m->n_kf <= 0) return VX_OK;
    // ---- SelectKeyFrames (local_ba.cpp:42-62): std::map order = ascending id
    std::vector<int> order(m->n_kf);
    for (int i = 0; i < m->n_kf; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int x, int y) { return m->kf_id[x] < m->kf_id[y]; });
    const int window = std::max(1, (int)o.window_size);
    const uint64_t max_id = has_ref ? ref_kf_id : m->kf_id[order.back()];
    std::vector<int> win;
    for (int i = m->n_kf - 1; i >= 0 && (int)win.size() < window; --i) {
        if (m->kf_id[order[i]] > max_id) continue;
        win.push_back(order[i]);
    }
    std::reverse(win.begin(), win.end());
    p->n_window_kf = (int)win.size();
    if (win.size() < 2) return VX_OK;
    std::unordered_map<uint64_t, int> win_row;  // kf id -> device row
    for (int r = 0; r < (int)win.size(); ++r) win_row[m->kf_id[win[r]]] = r;

    // ---- landmark set (local_ba.cpp:83-108)
    std::unordered_map<uint64_t, int> lm_by_id;
    lm_by_id.reserve((size_t)m->n_lm * 2);
    for (int i = 0; i < m->n_lm; ++i) lm_by_id[m->lm_id[i]] = i;
    std::unordered_set<uint64_t> lm_ids;
    for (int k : win)
        for (int64_t f = m->kf_feat_ptr[k]; f < m->kf_feat_ptr[k + 1]; ++f)
            if (m->feat_flags[f] & 1) lm_ids.insert(m->feat_lm_id[f]);
    std::vector<int> opt_all;
    for (uint64_t id : lm_ids) {
        auto it = lm_by_id.find(id);
        if (it == lm_by_id.end()) continue;
        const int l = it->second;
        if (m->lm_bad[l]) continue;
        if (m->lm_obs_ptr[l + 1] - m->lm_obs_ptr[l] < (int64_t)o.min_point_observations) continue;
        opt_all.push_back(l);
    }
    std::sort(opt_all.begin(), opt_all.end());
    p->n_landmarks_global = (int)opt_all.size();
    if (opt_all.empty()) return VX_OK;
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
            auto it = lm_by_id.find(m->feat_lm_id[f]);
            if (it == lm_by_id.end()) continue;
            const int l = it->second;
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
    p->n_lm = (int)p->lm_map_idx.size();
    p->n_pose_obs = (int64_t)puv.size();
    std::vector<double> lm0((size_t)std::max(p->n_lm, 1) * 4, 0.0);
    for (int s = 0; s < p->n_lm; ++s)
        for (int j = 0; j < 3; ++j) lm0[4 * s + j] = m->lm_pos[3 * p->lm_map_idx[s] + j];

    // ---- landmark-stage CSR (local_ba.cpp:186-204)
    std::vector<int> lptr(p->n_opt + 1, 0), lkf;
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
            luv.push_back(make_double2(m->feat_uv[2 * f], m->feat_uv[2 * f + 1]));
        }
        lptr[s + 1] = (int)lkf.size();
    }
    p->n_lm_obs = (int64_t)lkf.size();
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
    if ((rc = upload(c, p->lobs_uv, luv))) return rc;
    VX_HIP(c, p->kf_pose.ensure((size_t)nk * 2 * 8 * sizeof(double)));
    VX_HIP(c, p->kf_rot.ensure((size_t)nk * 9 * sizeof(double)));
    VX_HIP(c, p->kf_sums.ensure((size_t)nk * kStride * sizeof(double)));
    VX_HIP(c, p->kf_cost.ensure((size_t)nk * 2 * sizeof(double)));
    VX_HIP(c, p->lm_pos.ensure(lm0.size() * sizeof(double)));
    VX_HIP(c, p->state.ensure(sizeof(BAState)));
    return VX_OK;
}

int plan_run(vx_ctx* c, vx_ba_plan* p) {
    if (p->status != 0) {
        p->ran = true;
        return VX_OK;
    }
    const bool sharded = p->shard_count > 1;
    if (sharded) {
#ifndef VX_NO_RCCL
        if (!c->comm || c->nranks != p->shard_count || c->rank != p->shard_rank)
            return set_error(c, VX_ERR_STATE, "sharded plan needs vx_comm_init(%d ranks)", p->shard_count);
#else
        return set_error(c, VX_ERR_COMM, "built without RCCL");
#endif
    }
    const BAArgs a = make_args(p);
    if (p->opt.max_iterations == 0) {
        ProfScope ps(c, kStBaReset);
        const int n = std::max(p->n_kf * 8, std::max(p->n_lm, 1) * 4);
        hipLaunchKernelGGL(k_ba_reset, dim3((n + 255) / 256), dim3(256), 0, c->stream, a);
        VX_LAUNCH_CHECK(c, "k_ba_reset");
    }
    const bool lds_poses = p->n_kf <= kMaxKfLds;
    const size_t lds = (size_t)p->n_kf * 21 * sizeof(double);
    const int lm_blocks = std::max(1, (p->n_opt + 255) / 256);
    for (int it = 0; it < p->opt.max_iterations; ++it) {
        {
            ProfScope ps(c, kStBaPose);
            hipLaunchKernelGGL(k_pose_kf, dim3(p->n_kf), dim3(kPoseBlock), 0, c->stream, a, it);
            VX_LAUNCH_CHECK(c, "k_pose_kf");
        }
#ifndef VX_NO_RCCL
        if (sharded) {
            ProfScope ps(c, kStBaAllreduce);
            ncclResult_t r = ncclAllReduce(p->kf_sums.p, p->kf_sums.p, (size_t)p->n_kf * kStride, ncclDouble,
                                           ncclSum, c->comm, c->stream);
            if (r != ncclSuccess) return set_error(c, VX_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
        }
#endif
        ProfScope ps(c, kStBaLandmark);
        if (lds_poses) {
            hipLaunchKernelGGL(k_landmark_solve, dim3(lm_blocks), dim3(256), lds, c->stream, a, it);
            VX_LAUNCH_CHECK(c, "k_landmark_solve");
        } else {
            hipLaunchKernelGGL(k_pose_solve_g, dim3((p->n_kf + 255) / 256), dim3(256), 0, c->stream, a, it);
            VX_LAUNCH_CHECK(c, "k_pose_solve_g");
            hipLaunchKernelGGL(k_landmark, dim3(lm_blocks), dim3(256), 0, c->stream, a, it);
            VX_LAUNCH_CHECK(c, "k_landmark");
        }
    }
    p->ran = true;
    return VX_OK;
}

}  // namespace
}  // namespace vx

using namespace vx;

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
    const int rc = build_plan(c, m, ref, has_ref, p);
    if (rc) {
        delete p;
        return rc;
    }
    *out = p;
    return VX_OK;
}

int vx_ba_plan_run_async(vx_ctx* c, vx_ba_plan* p) {
    if (!c || !p || p->c != c) return VX_ERR_INVALID;
    return plan_run(c, p);
}

int vx_ba_plan_fetch(vx_ctx* c, vx_ba_plan* p, vx_map_view* m, vx_ba_stats* st) {
    if (!c || !p || p->c != c) return VX_ERR_INVALID;
    if (!p->ran) return set_error(c, VX_ERR_STATE, "plan not run");
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

void vx_ba_plan_destroy(vx_ba_plan* p) { delete p; }

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
    return shard_count <= 1 ? 0u : (uint32_t)(vx::splitmix64(lm_id) % (uint64_t)shard_count);
}

int vx_ba_plan_info(const vx_ba_plan* p, int64_t* out4) {
    if (!p || !out4) return VX_ERR_INVALID;
    out4[0] = p->n_kf;
    out4[1] = p->n_lm;
    out4[2] = p->n_pose_obs;
    out4[3] = p->n_lm_obs;
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
