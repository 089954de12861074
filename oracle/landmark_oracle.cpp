// landmark_oracle.cpp — CPU restatement of the keyframe-insertion loops.  TEST INFRASTRUCTURE ONLY.
//
//   orc_depth_landmarks  <- Tracking::CreateLandmarksFromDepth (core/frontend/tracking.cpp:586-650)
//   orc_triangulate      <- Tracking::TriangulateWithLastKeyFrame (tracking.cpp:856-929) with
//                           ProjectionMatrix (:843-854) and TriangulatePoint (:931-945)
// Both are restated as the reference loops: in feature / match order, marking has_landmark as
// they go (so a later match on an already triangulated feature is skipped), Camera::pixelToCamera
// (core/camera/camera.cpp:30-34), Sophus SE3 inverse / action and ProjectToPixel
// (core/common/projection.h:11-31).  Third-party: TriangulatePoint takes column 3 of
// Eigen::JacobiSVD(A, ComputeFullV).matrixV() (Eigen 3, unpinned, not installed here); this file
// computes the same right singular vector (smallest singular value) with a one-sided Jacobi SVD.
// For a rank-3 A that vector is unique up to sign and X / X(3) removes the sign, so any accurate
// SVD gives the point to rounding; tests/test_landmarks_cpu.py pins it against numpy's LAPACK SVD.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "ba_math.h"
#include "oracle.h"

using namespace orc_ba;

namespace {

SE3 pose_of(const double* p) { return SE3{{p[0], p[1], p[2], p[3]}, {p[4], p[5], p[6]}}; }

// Sophus SE3::inverse(): (conj(q), conj(q) * (-t))
SE3 inverse(const SE3& T) {
    SE3 I;
    I.q = {-T.q.x, -T.q.y, -T.q.z, T.q.w};
    I.t = rotate(I.q, {T.t.x * -1.0, T.t.y * -1.0, T.t.z * -1.0});
    return I;
}

void null_vector4(double A[16], double X[4]) {
    double V[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    for (int sweep = 0; sweep < 12; ++sweep) {
        bool rotated = false;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                double al = 0.0, be = 0.0, ga = 0.0;
                for (int r = 0; r < 4; ++r) {
                    al += A[4 * r + p] * A[4 * r + p];
                    be += A[4 * r + q] * A[4 * r + q];
                    ga += A[4 * r + p] * A[4 * r + q];
                }
                if (!(std::fabs(ga) > 1e-15 * std::sqrt(al * be))) continue;
                rotated = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double cs = 1.0 / std::sqrt(1.0 + t * t), sn = cs * t;
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
    for (int c = 0; c < 4; ++c) {
        double s = 0.0;
        for (int r = 0; r < 4; ++r) s += A[4 * r + c] * A[4 * r + c];
        if (c == 0 || s < bn) {
            bn = s;
            best = c;
        }
    }
    for (int r = 0; r < 4; ++r) X[r] = V[4 * r + best];
}

// ProjectionMatrix (tracking.cpp:843-854): K [R | t]
void projection_matrix(const SE3& T, const double* K, double P[12]) {
    double R[9];
    rotation_matrix(T.q, R);
    const double t[3] = {T.t.x, T.t.y, T.t.z};
    for (int c = 0; c < 4; ++c) {
        const double r0 = c < 3 ? R[c] : t[0], r1 = c < 3 ? R[3 + c] : t[1], r2 = c < 3 ? R[6 + c] : t[2];
        P[c] = K[0] * r0 + K[2] * r2;
        P[4 + c] = K[1] * r1 + K[3] * r2;
        P[8 + c] = r2;
    }
}

}  // namespace

extern "C" int orc_depth_landmarks(const double* uv, const uint8_t* has, int n, const void* depth, int type,
                                   int rows, int cols, int64_t stride, const double* intr4, const double* pose7,
                                   int32_t* out_index, double* out_pw, int* n_created) {
    *n_created = 0;
    for (int i = 0; i < n; ++i) out_index[i] = -1;
    if (!depth || rows <= 0 || cols <= 0) return 0;
    const SE3 Tinv = inverse(pose_of(pose7));
    const double kDepthScale = 5000.0, kMinDepth = 0.1, kMaxDepth = 10.0;
    for (int i = 0; i < n; ++i) {
        if (has[i]) continue;
        const int u = static_cast<int>(uv[2 * i] + 0.5);
        const int v = static_cast<int>(uv[2 * i + 1] + 0.5);
        if (u < 0 || u >= cols || v < 0 || v >= rows) continue;
        const uint8_t* row = static_cast<const uint8_t*>(depth) + (int64_t)v * stride;
        double depth_m = 0.0;
        if (type == 0) {
            uint16_t d;
            std::memcpy(&d, row + 2 * u, 2);
            if (d == 0) continue;
            depth_m = static_cast<double>(d) / kDepthScale;
        } else if (type == 1) {
            float d;
            std::memcpy(&d, row + 4 * u, 4);
            depth_m = static_cast<double>(d);
        } else {
            std::memcpy(&depth_m, row + 8 * u, 8);
        }
        if (depth_m < kMinDepth || depth_m > kMaxDepth) continue;
        const double x = (uv[2 * i] - intr4[2]) / intr4[0];
        const double y = (uv[2 * i + 1] - intr4[3]) / intr4[1];
        const Vec3 pc{x * depth_m, y * depth_m, depth_m};
        const Vec3 pw = transform(Tinv, pc);
        out_index[i] = *n_created;
        out_pw[3 * *n_created] = pw.x;
        out_pw[3 * *n_created + 1] = pw.y;
        out_pw[3 * *n_created + 2] = pw.z;
        ++*n_created;
    }
    return 0;
}

extern "C" int orc_triangulate(const double* uv1, const uint8_t* has1_in, int n1, const double* intr1,
                               const double* pose1, const double* uv2, const uint8_t* has2_in, int n2,
                               const double* intr2, const double* pose2, const orc_match* m, int nm,
                               double min_angle_deg, double max_err, int32_t* out_index, double* out_pw,
                               int* n_created) {
    *n_created = 0;
    std::vector<uint8_t> has1(has1_in, has1_in + n1), has2(has2_in, has2_in + n2);
    const SE3 T1 = pose_of(pose1), T2 = pose_of(pose2);
    double P1[12], P2[12];
    projection_matrix(T1, intr2, P1);  // both with the current frame's camera (tracking.cpp:864-867)
    projection_matrix(T2, intr2, P2);
    const double min_angle_rad = min_angle_deg * M_PI / 180.0;
    double R1[9], R2[9];
    rotation_matrix(inverse(T1).q, R1);
    rotation_matrix(inverse(T2).q, R2);
    const Cam c1{intr1[0], intr1[1], intr1[2], intr1[3]}, c2{intr2[0], intr2[1], intr2[2], intr2[3]};
    for (int k = 0; k < nm; ++k) {
        out_index[k] = -1;
        const int qi = m[k].query_idx, ti = m[k].train_idx;
        if (qi < 0 || qi >= n1 || ti < 0 || ti >= n2) return -1;
        const double x1 = uv1[2 * qi], y1 = uv1[2 * qi + 1], x2 = uv2[2 * ti], y2 = uv2[2 * ti + 1];
        if (has1[qi] || has2[ti]) continue;
        double f1[3] = {(x1 - intr1[2]) / intr1[0], (y1 - intr1[3]) / intr1[1], 1.0};
        double f2[3] = {(x2 - intr2[2]) / intr2[0], (y2 - intr2[3]) / intr2[1], 1.0};
        const double n1n = std::sqrt(f1[0] * f1[0] + f1[1] * f1[1] + f1[2] * f1[2]);
        const double n2n = std::sqrt(f2[0] * f2[0] + f2[1] * f2[1] + f2[2] * f2[2]);
        for (int j = 0; j < 3; ++j) {
            f1[j] = f1[j] / n1n;
            f2[j] = f2[j] / n2n;
        }
        double g1[3], g2[3];
        for (int r = 0; r < 3; ++r) {
            g1[r] = R1[3 * r] * f1[0] + R1[3 * r + 1] * f1[1] + R1[3 * r + 2] * f1[2];
            g2[r] = R2[3 * r] * f2[0] + R2[3 * r + 1] * f2[1] + R2[3 * r + 2] * f2[2];
        }
        const double dot = g1[0] * g2[0] + g1[1] * g2[1] + g1[2] * g2[2];
        const double m1 = std::sqrt(g1[0] * g1[0] + g1[1] * g1[1] + g1[2] * g1[2]);
        const double m2 = std::sqrt(g2[0] * g2[0] + g2[1] * g2[1] + g2[2] * g2[2]);
        const double cosa = std::clamp(dot / (m1 * m2), -1.0, 1.0);
        if (std::acos(cosa) < min_angle_rad) continue;
        double A[16];
        for (int c = 0; c < 4; ++c) {
            A[c] = x1 * P1[8 + c] - P1[c];
            A[4 + c] = y1 * P1[8 + c] - P1[4 + c];
            A[8 + c] = x2 * P2[8 + c] - P2[c];
            A[12 + c] = y2 * P2[8 + c] - P2[4 + c];
        }
        double X[4];
        null_vector4(A, X);
        const Vec3 pw{X[0] / X[3], X[1] / X[3], X[2] / X[3]};
        if (!(std::isfinite(pw.x) && std::isfinite(pw.y) && std::isfinite(pw.z))) continue;
        double r1[2], r2[2];
        Vec3 pc;
        if (!project(c1, T1, pw, r1, pc)) continue;
        if (!project(c2, T2, pw, r2, pc)) continue;
        const double e1 = std::sqrt((r1[0] - x1) * (r1[0] - x1) + (r1[1] - y1) * (r1[1] - y1));
        const double e2 = std::sqrt((r2[0] - x2) * (r2[0] - x2) + (r2[1] - y2) * (r2[1] - y2));
        if (e1 > max_err || e2 > max_err) continue;
        out_index[k] = *n_created;
        out_pw[3 * *n_created] = pw.x;
        out_pw[3 * *n_created + 1] = pw.y;
        out_pw[3 * *n_created + 2] = pw.z;
        ++*n_created;
        has1[qi] = 1;
        has2[ti] = 1;
    }
    return 0;
}
