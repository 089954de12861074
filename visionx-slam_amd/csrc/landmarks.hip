// landmarks.hip — landmark creation on keyframe insertion.
//
// Replaces the two per-feature / per-match loops Tracking::CreateKeyFrame runs right before
// LocalBA (core/frontend/tracking.cpp:577-580):
//   CreateLandmarksFromDepth (tracking.cpp:586-650)  one thread per feature: rounding to the depth
//        pixel (static_cast<int>(x + 0.5)), TUM depth scale 5000 (u16) / metres (f32, f64),
//        0.1 <= d <= 10, Camera::pixelToCamera (camera.cpp:30-34), T_cw.inverse() * pc (Sophus).
//   TriangulateWithLastKeyFrame + TriangulatePoint (tracking.cpp:856-945)  one thread per match:
//        parallax angle of the two bearing rays (>= triangulation_min_angle_deg), the 4x4 DLT
//        system of ProjectionMatrix (K [R | t] with the CURRENT frame's camera for both views,
//        tracking.cpp:864-867), its right singular vector of the smallest singular value
//        (Eigen::JacobiSVD in the reference; here a one-sided Jacobi SVD in registers — the null
//        vector is unique up to sign for a rank-3 system, so the point is the same to rounding),
//        ProjectToPixel in both views (projection.h:11-31) and the reprojection gate.
// The reference marks features as it goes, so a later match whose train feature an earlier match
// already triangulated is skipped: the first passing match per train feature wins (atomicMin),
// which is the sequential outcome because the matcher's query indices are unique.  Created
// landmarks are numbered in input order (an order-preserving scan), as landmark_id_++ numbers them.
#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

#include "vx_internal.hpp"
#include "ba_common.hpp"

namespace vx {
namespace {

using namespace vx::ba;

constexpr int kThreads = 256;
constexpr int kScanThreads = 1024;

struct Pose {  // Sophus SE3d: unit quaternion (x y z w) + translation, T_cw
    double q[4], t[3];
};

// Eigen _transformVector: q * v
__device__ __forceinline__ D3 qrot(const double* q, D3 v) {
    const D3 qv{q[0], q[1], q[2]};
    D3 uv{qv.y * v.z - qv.z * v.y, qv.z * v.x - qv.x * v.z, qv.x * v.y - qv.y * v.x};
    uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
    const D3 c{qv.y * uv.z - qv.z * uv.y, qv.z * uv.x - qv.x * uv.z, qv.x * uv.y - qv.y * uv.x};
    return {v.x + q[3] * uv.x + c.x, v.y + q[3] * uv.y + c.y, v.z + q[3] * uv.z + c.z};
}

// Sophus T.inverse() * p: inverse = (conj(q), conj(q) * (-t)), then rotate + translate
__device__ __forceinline__ D3 inv_apply(const Pose& T, D3 p) {
    const double qc[4] = {-T.q[0], -T.q[1], -T.q[2], T.q[3]};
    const D3 ti = qrot(qc, {T.t[0] * -1.0, T.t[1] * -1.0, T.t[2] * -1.0});
    const D3 r = qrot(qc, p);
    return {r.x + ti.x, r.y + ti.y, r.z + ti.z};
}

// ---------------------------------------------------------------- CreateLandmarksFromDepth
struct DepthArgs {
    const double* uv;        // 2 per feature (Feature::position)
    const uint8_t* has;      // Feature::has_landmark
    int n;
    const uint8_t* depth;
    int type, rows, cols;
    long long stride;        // bytes per depth row
    double fx, fy, cx, cy;
    Pose T;
    int* valid;
    double* pw;              // 3 per feature (uncompacted)
};

__global__ __launch_bounds__(kThreads) void k_depth_lm(DepthArgs a) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= a.n) return;
    int ok = 0;
    if (!a.has[i]) {
        const double x = a.uv[2 * i], y = a.uv[2 * i + 1];
        const int u = (int)(x + 0.5), v = (int)(y + 0.5);  // static_cast<int>: truncation
        if (u >= 0 && u < a.cols && v >= 0 && v < a.rows) {
            const uint8_t* row = a.depth + (long long)v * a.stride;
            double d = 0.0;
            bool have = true;
            if (a.type == VX_DEPTH_U16) {
                const uint16_t raw = reinterpret_cast<const uint16_t*>(row)[u];
                have = raw != 0;
                d = (double)raw / 5000.0;  // kDepthScale (tracking.cpp:601)
            } else if (a.type == VX_DEPTH_F32) {
                d = (double)reinterpret_cast<const float*>(row)[u];
            } else {
                d = reinterpret_cast<const double*>(row)[u];
            }
            if (have && !(d < 0.1 || d > 10.0)) {  // kMinDepth / kMaxDepth (tracking.cpp:602-603)
                const double xn = (x - a.cx) / a.fx, yn = (y - a.cy) / a.fy;
                const D3 p = inv_apply(a.T, {xn * d, yn * d, d});
                a.pw[3 * i] = p.x;
                a.pw[3 * i + 1] = p.y;
                a.pw[3 * i + 2] = p.z;
                ok = 1;
            }
        }
    }
    a.valid[i] = ok;
}

// ---------------------------------------------------------------- TriangulateWithLastKeyFrame
struct TriArgs {
    const double* uv1;
    const uint8_t* has1;
    int n1;
    const double* uv2;
    const uint8_t* has2;
    int n2;
    const vx_match* m;
    int n;
    double c1[4], c2[4];     // fx fy cx cy of the last / current frame camera
    Pose T1, T2;
    double min_angle_rad, max_err;
    int* valid;
    double* pw;
    int* winner;             // n2: first passing match per train feature
    int* qseen;              // n1: duplicate query detection
    int* err;
};

// rotation matrix of a unit quaternion (Eigen toRotationMatrix)
__device__ __forceinline__ void qmat(const double* q, double* R) { rot_from_quat(q, R); }

// ProjectToPixel (projection.h:11-31)
__device__ __forceinline__ bool project(const double* c, const Pose& T, D3 pw, double& u, double& v) {
    const D3 r = qrot(T.q, pw);
    const D3 pc{r.x + T.t[0], r.y + T.t[1], r.z + T.t[2]};
    if (pc.z <= 1e-6) return false;
    const double inv_z = 1.0 / pc.z;
    u = c[0] * (pc.x * inv_z) + c[2];
    v = c[1] * (pc.y * inv_z) + c[3];
    return true;
}

// Right singular vector of the smallest singular value of the 4x4 A (row-major) by one-sided
// Jacobi (Hestenes): rotate column pairs of A V until they are orthogonal, V accumulates the
// rotations; the column of least norm of A V gives the singular vector.
__device__ void null_vector4(double* A, double* X) {
    double V[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    for (int sweep = 0; sweep < 12; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double al = 0.0, be = 0.0, ga = 0.0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    al += A[4 * r + p] * A[4 * r + p];
                    be += A[4 * r + q] * A[4 * r + q];
                    ga += A[4 * r + p] * A[4 * r + q];
                }
                if (!(fabs(ga) > 1e-15 * sqrt(al * be))) continue;
                rotated = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double ap = A[4 * r + p], aq = A[4 * r + q];
                    A[4 * r + p] = cs * ap - sn * aq;
                    A[4 * r + q] = sn * ap + cs * aq;
                    const double vp = V[4 * r + p], vq = V[4 * r + q];
                    V[4 * r + p] = cs * vp - sn * vq;
                    V[4 * r + q] = sn * vp + cs * vq;
                }
            }
        if (!rotated) break;
    }
    int best = 0;
    double bn = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) s += A[4 * r + c] * A[4 * r + c];
        if (c == 0 || s < bn) {
            bn = s;
            best = c;
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) X[r] = best == 0 ? V[4 * r] : best == 1 ? V[4 * r + 1] : best == 2 ? V[4 * r + 2] : V[4 * r + 3];
}

__global__ __launch_bounds__(kThreads) void k_triangulate(TriArgs a) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= a.n) return;
    a.valid[k] = 0;
    const vx_match mt = a.m[k];
    const int qi = mt.query_idx, ti = mt.train_idx;
    if (qi < 0 || qi >= a.n1 || ti < 0 || ti >= a.n2) {
        atomicOr(a.err, 1);
        return;
    }
    if (atomicAdd(&a.qseen[qi], 1) != 0) atomicOr(a.err, 2);
    if (a.has1[qi] || a.has2[ti]) return;
    const double x1 = a.uv1[2 * qi], y1 = a.uv1[2 * qi + 1];
    const double x2 = a.uv2[2 * ti], y2 = a.uv2[2 * ti + 1];
    // parallax (tracking.cpp:878-890): bearings of pixelToCamera(px, 1), normalized, rotated by
    // T_cw.inverse().rotationMatrix()
    double f1[3] = {(x1 - a.c1[2]) / a.c1[0], (y1 - a.c1[3]) / a.c1[1], 1.0};
    double f2[3] = {(x2 - a.c2[2]) / a.c2[0], (y2 - a.c2[3]) / a.c2[1], 1.0};
    {
        const double n1 = sqrt(f1[0] * f1[0] + f1[1] * f1[1] + f1[2] * f1[2]);
        const double n2 = sqrt(f2[0] * f2[0] + f2[1] * f2[1] + f2[2] * f2[2]);
        for (int j = 0; j < 3; ++j) {
            f1[j] = f1[j] / n1;
            f2[j] = f2[j] / n2;
        }
    }
    double R1[9], R2[9];
    {
        const double q1c[4] = {-a.T1.q[0], -a.T1.q[1], -a.T1.q[2], a.T1.q[3]};
        const double q2c[4] = {-a.T2.q[0], -a.T2.q[1], -a.T2.q[2], a.T2.q[3]};
        qmat(q1c, R1);
        qmat(q2c, R2);
    }
    double g1[3], g2[3];
    for (int r = 0; r < 3; ++r) {
        g1[r] = R1[3 * r] * f1[0] + R1[3 * r + 1] * f1[1] + R1[3 * r + 2] * f1[2];
        g2[r] = R2[3 * r] * f2[0] + R2[3 * r + 1] * f2[1] + R2[3 * r + 2] * f2[2];
    }
    const double dot = g1[0] * g2[0] + g1[1] * g2[1] + g1[2] * g2[2];
    const double m1 = sqrt(g1[0] * g1[0] + g1[1] * g1[1] + g1[2] * g1[2]);
    const double m2 = sqrt(g2[0] * g2[0] + g2[1] * g2[1] + g2[2] * g2[2]);
    const double cosa = fmin(fmax(dot / (m1 * m2), -1.0), 1.0);
    if (acos(cosa) < a.min_angle_rad) return;
    // DLT (tracking.cpp:931-945): P = K [R | t] with the current frame's camera for both views
    double P1[12], P2[12];
    {
        double Ra[9], Rb[9];
        qmat(a.T1.q, Ra);
        qmat(a.T2.q, Rb);
        const double* K = a.c2;
        for (int c = 0; c < 4; ++c) {
            const double r0a = c < 3 ? Ra[c] : a.T1.t[0], r1a = c < 3 ? Ra[3 + c] : a.T1.t[1], r2a = c < 3 ? Ra[6 + c] : a.T1.t[2];
            const double r0b = c < 3 ? Rb[c] : a.T2.t[0], r1b = c < 3 ? Rb[3 + c] : a.T2.t[1], r2b = c < 3 ? Rb[6 + c] : a.T2.t[2];
            P1[c] = K[0] * r0a + K[2] * r2a;
            P1[4 + c] = K[1] * r1a + K[3] * r2a;
            P1[8 + c] = r2a;
            P2[c] = K[0] * r0b + K[2] * r2b;
            P2[4 + c] = K[1] * r1b + K[3] * r2b;
            P2[8 + c] = r2b;
        }
    }
    double A[16];
    for (int c = 0; c < 4; ++c) {
        A[c] = x1 * P1[8 + c] - P1[c];
        A[4 + c] = y1 * P1[8 + c] - P1[4 + c];
        A[8 + c] = x2 * P2[8 + c] - P2[c];
        A[12 + c] = y2 * P2[8 + c] - P2[4 + c];
    }
    double X[4];
    null_vector4(A, X);
    const D3 pw{X[0] / X[3], X[1] / X[3], X[2] / X[3]};
    if (!(isfinite(pw.x) && isfinite(pw.y) && isfinite(pw.z))) return;
    double u1, v1, u2, v2;
    if (!project(a.c1, a.T1, pw, u1, v1)) return;
    if (!project(a.c2, a.T2, pw, u2, v2)) return;
    const double e1 = sqrt((u1 - x1) * (u1 - x1) + (v1 - y1) * (v1 - y1));
    const double e2 = sqrt((u2 - x2) * (u2 - x2) + (v2 - y2) * (v2 - y2));
    if (e1 > a.max_err || e2 > a.max_err) return;
    a.valid[k] = 1;
    a.pw[3 * k] = pw.x;
    a.pw[3 * k + 1] = pw.y;
    a.pw[3 * k + 2] = pw.z;
    atomicMin(&a.winner[ti], k);
}

__global__ __launch_bounds__(kThreads) void k_tri_resolve(int* valid, const vx_match* m, const int* winner, int n) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k < n && valid[k] && winner[m[k].train_idx] != k) valid[k] = 0;
}

// Order-preserving compaction: index[i] = rank of i among the valid entries (-1 otherwise), the
// valid points packed in that order; one workgroup, each thread owns a contiguous chunk.
__global__ __launch_bounds__(kScanThreads) void k_compact(const int* valid, const double* pw, int n, int* index,
                                                          double* out, int* count) {
    __shared__ int part[kScanThreads];
    const int t = threadIdx.x;
    const int chunk = (n + kScanThreads - 1) / kScanThreads;
    const int b = min(n, t * chunk), e = min(n, b + chunk);
    int c = 0;
    for (int i = b; i < e; ++i) c += valid[i];
    part[t] = c;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {  // inclusive Hillis-Steele scan
        const int v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int r = part[t] - c;
    for (int i = b; i < e; ++i) {
        if (valid[i]) {
            index[i] = r;
            out[3 * r] = pw[3 * i];
            out[3 * r + 1] = pw[3 * i + 1];
            out[3 * r + 2] = pw[3 * i + 2];
            ++r;
        } else {
            index[i] = -1;
        }
    }
    if (t == kScanThreads - 1) *count = part[t];
}

template <class T>
int to_dev(vx_ctx* c, DevBuf& d, const T* h, size_t n) {
    VX_HIP(c, d.ensure(std::max<size_t>(1, n) * sizeof(T)));
    if (n) VX_HIP(c, hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return VX_OK;
}

Pose host_pose(const double* p) {
    Pose T;
    for (int j = 0; j < 4; ++j) T.q[j] = p[j];
    for (int j = 0; j < 3; ++j) T.t[j] = p[4 + j];
    return T;
}

int fetch_compacted(vx_ctx* c, int n, int32_t* out_index, double* out_pw, int* n_created) {
    int cnt = 0;
    VX_HIP(c, hipMemcpyAsync(&cnt, c->lm_count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    if (out_index) VX_HIP(c, hipMemcpy(out_index, c->lm_index.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
    if (out_pw && cnt) VX_HIP(c, hipMemcpy(out_pw, c->lm_out.p, (size_t)cnt * 3 * sizeof(double), hipMemcpyDeviceToHost));
    *n_created = cnt;
    return VX_OK;
}

int compact(vx_ctx* c, int n) {
    VX_HIP(c, c->lm_index.ensure((size_t)std::max(n, 1) * sizeof(int)));
    VX_HIP(c, c->lm_out.ensure((size_t)std::max(n, 1) * 3 * sizeof(double)));
    VX_HIP(c, c->lm_count.ensure(4 * sizeof(int)));
    ProfScope ps(c, kStLmCompact);
    hipLaunchKernelGGL(k_compact, dim3(1), dim3(kScanThreads), 0, c->stream, c->lm_valid.as<int>(),
                       c->lm_pw.as<double>(), n, c->lm_index.as<int>(), c->lm_out.as<double>(), c->lm_count.as<int>());
    VX_LAUNCH_CHECK(c, "k_compact");
    return VX_OK;
}

}  // namespace
}  // namespace vx

using namespace vx;

extern "C" {

int vx_depth_landmarks(vx_ctx* c, const double* feat_uv, const uint8_t* feat_has_lm, int n_feat, const void* depth,
                       int depth_type, int rows, int cols, int64_t row_stride, const double* intr4,
                       const double* pose7, int32_t* out_index, double* out_pw, int* n_created) {
    if (!c || !n_created || n_feat < 0 || (n_feat > 0 && (!feat_uv || !feat_has_lm)) || !intr4 || !pose7)
        return c ? set_error(c, VX_ERR_INVALID, "vx_depth_landmarks: bad arguments") : VX_ERR_INVALID;
    *n_created = 0;
    if (depth_type < VX_DEPTH_U16 || depth_type > VX_DEPTH_F64)
        return set_error(c, VX_ERR_INVALID, "unknown depth type %d", depth_type);
    const int esz = depth_type == VX_DEPTH_U16 ? 2 : (depth_type == VX_DEPTH_F32 ? 4 : 8);
    if (n_feat == 0 || !depth || rows <= 0 || cols <= 0) {  // depth.empty() (tracking.cpp:591-594)
        for (int i = 0; out_index && i < n_feat; ++i) out_index[i] = -1;
        return VX_OK;
    }
    if (row_stride < (int64_t)cols * esz) return set_error(c, VX_ERR_INVALID, "row_stride < cols * element size");
    VX_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = to_dev(c, c->lm_in0, feat_uv, (size_t)n_feat * 2))) return rc;
    if ((rc = to_dev(c, c->lm_in1, feat_has_lm, (size_t)n_feat))) return rc;
    if ((rc = to_dev(c, c->lm_depth, static_cast<const uint8_t*>(depth), (size_t)row_stride * rows))) return rc;
    VX_HIP(c, c->lm_valid.ensure((size_t)n_feat * sizeof(int)));
    VX_HIP(c, c->lm_pw.ensure((size_t)n_feat * 3 * sizeof(double)));
    DepthArgs a{};
    a.uv = c->lm_in0.as<double>();
    a.has = c->lm_in1.as<uint8_t>();
    a.n = n_feat;
    a.depth = c->lm_depth.as<uint8_t>();
    a.type = depth_type;
    a.rows = rows;
    a.cols = cols;
    a.stride = row_stride;
    a.fx = intr4[0];
    a.fy = intr4[1];
    a.cx = intr4[2];
    a.cy = intr4[3];
    a.T = host_pose(pose7);
    a.valid = c->lm_valid.as<int>();
    a.pw = c->lm_pw.as<double>();
    VX_HIP(c, launch(c, kStLmDepth, k_depth_lm, dim3((n_feat + kThreads - 1) / kThreads), dim3(kThreads), 0,
                     c->stream, a));
    if ((rc = compact(c, n_feat))) return rc;
    return fetch_compacted(c, n_feat, out_index, out_pw, n_created);
}

int vx_triangulate(vx_ctx* c, const double* uv1, const uint8_t* has1, int n1, const double* intr1, const double* pose1,
                   const double* uv2, const uint8_t* has2, int n2, const double* intr2, const double* pose2,
                   const vx_match* matches, int n_matches, double min_angle_deg, double max_reproj_error,
                   int32_t* out_index, double* out_pw, int* n_created) {
    if (!c || !n_created || n_matches < 0 || n1 < 0 || n2 < 0 || !intr1 || !intr2 || !pose1 || !pose2 ||
        (n_matches > 0 && (!matches || !uv1 || !uv2 || !has1 || !has2)))
        return c ? set_error(c, VX_ERR_INVALID, "vx_triangulate: bad arguments") : VX_ERR_INVALID;
    *n_created = 0;
    if (n_matches == 0) return VX_OK;
    VX_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = to_dev(c, c->lm_in0, uv1, (size_t)n1 * 2))) return rc;
    if ((rc = to_dev(c, c->lm_in1, has1, (size_t)n1))) return rc;
    if ((rc = to_dev(c, c->lm_in2, uv2, (size_t)n2 * 2))) return rc;
    if ((rc = to_dev(c, c->lm_in3, has2, (size_t)n2))) return rc;
    if ((rc = to_dev(c, c->lm_in4, matches, (size_t)n_matches))) return rc;
    VX_HIP(c, c->lm_valid.ensure((size_t)n_matches * sizeof(int)));
    VX_HIP(c, c->lm_pw.ensure((size_t)n_matches * 3 * sizeof(double)));
    VX_HIP(c, c->lm_aux.ensure(((size_t)n2 + n1 + 4) * sizeof(int)));
    int* winner = c->lm_aux.as<int>();
    int* qseen = winner + n2;
    int* err = qseen + n1;
    VX_HIP(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(winner), INT_MAX, (size_t)std::max(n2, 0), c->stream));
    VX_HIP(c, hipMemsetAsync(qseen, 0, ((size_t)n1 + 1) * sizeof(int), c->stream));
    TriArgs a{};
    a.uv1 = c->lm_in0.as<double>();
    a.has1 = c->lm_in1.as<uint8_t>();
    a.n1 = n1;
    a.uv2 = c->lm_in2.as<double>();
    a.has2 = c->lm_in3.as<uint8_t>();
    a.n2 = n2;
    a.m = c->lm_in4.as<vx_match>();
    a.n = n_matches;
    for (int j = 0; j < 4; ++j) {
        a.c1[j] = intr1[j];
        a.c2[j] = intr2[j];
    }
    a.T1 = host_pose(pose1);
    a.T2 = host_pose(pose2);
    a.min_angle_rad = min_angle_deg * M_PI / 180.0;  // tracking.cpp:870-871
    a.max_err = max_reproj_error;
    a.valid = c->lm_valid.as<int>();
    a.pw = c->lm_pw.as<double>();
    a.winner = winner;
    a.qseen = qseen;
    a.err = err;
    const dim3 grid((n_matches + kThreads - 1) / kThreads);
    VX_HIP(c, launch(c, kStLmTriangulate, k_triangulate, grid, dim3(kThreads), 0, c->stream, a));
    hipLaunchKernelGGL(k_tri_resolve, grid, dim3(kThreads), 0, c->stream, a.valid, a.m, winner, n_matches);
    VX_LAUNCH_CHECK(c, "k_tri_resolve");
    if ((rc = compact(c, n_matches))) return rc;
    int herr = 0;
    VX_HIP(c, hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if ((rc = fetch_compacted(c, n_matches, out_index, out_pw, n_created))) return rc;
    if (herr & 1) return set_error(c, VX_ERR_INVALID, "match index out of range");
    if (herr & 2) return set_error(c, VX_ERR_INVALID, "duplicate query index (matches must come from one knnMatch)");
    return VX_OK;
}

}  // extern "C"
