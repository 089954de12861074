// ba_math.h — SE(3), projection and small dense solves shared by the LocalBA restatement
// (ba_oracle.cpp) and the Schur-complement BA restatement (sba_oracle.cpp).  TEST INFRASTRUCTURE
// ONLY.  Sources restated: Eigen QuaternionBase / LDLT, Sophus SE3d::exp (unpinned versions,
// vcpkg.json), ProjectToPixel (core/common/projection.h:11-31), ProjectionJacobian / PoseJacobian /
// HuberWeight (core/backend/local_ba.cpp:15-40).
#pragma once
#include <algorithm>
#include <cmath>
#include <limits>

namespace orc_ba {

struct Vec3 { double x, y, z; };
struct Quat { double x, y, z, w; };
struct SE3 { Quat q; Vec3 t; };

static inline Vec3 cross(const Vec3& a, const Vec3& b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// Eigen QuaternionBase::_transformVector (Sophus SO3 * point)
static inline Vec3 rotate(const Quat& q, const Vec3& v) {
    const Vec3 qv{q.x, q.y, q.z};
    Vec3 uv = cross(qv, v);
    uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
    const Vec3 c = cross(qv, uv);
    return {v.x + q.w * uv.x + c.x, v.y + q.w * uv.y + c.y, v.z + q.w * uv.z + c.z};
}

static inline Vec3 transform(const SE3& T, const Vec3& p) {
    const Vec3 r = rotate(T.q, p);
    return {r.x + T.t.x, r.y + T.t.y, r.z + T.t.z};
}

// Eigen Quaternion::toRotationMatrix
static inline void rotation_matrix(const Quat& q, double R[9]) {
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

// Sophus SO3 product + normalize()
static inline Quat quat_mul_normalized(const Quat& a, const Quat& b) {
    Quat r{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
           a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
           a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x,
           a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
    const double n = std::sqrt(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w);
    r.x /= n; r.y /= n; r.z /= n; r.w /= n;
    return r;
}

// Sophus::SE3d::exp(a), a = (upsilon, omega)
static inline SE3 se3_exp(const double a[6]) {
    const double eps = 1e-10;  // Sophus::Constants<double>::epsilon()
    const Vec3 w{a[3], a[4], a[5]};
    const double theta_sq = w.x * w.x + w.y * w.y + w.z * w.z;
    double theta, imag, real;
    if (theta_sq < eps * eps) {
        theta = 0.0;
        const double t4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * t4;
        real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * t4;
    } else {
        theta = std::sqrt(theta_sq);
        const double half = 0.5 * theta;
        imag = std::sin(half) / theta;
        real = std::cos(half);
    }
    SE3 T;
    T.q = {imag * w.x, imag * w.y, imag * w.z, real};
    const double O[9] = {0, -w.z, w.y, w.z, 0, -w.x, -w.y, w.x, 0};  // hat(omega)
    double V[9];
    if (theta < eps) {
        rotation_matrix(T.q, V);
    } else {
        double O2[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                O2[3 * r + c] = O[3 * r] * O[c] + O[3 * r + 1] * O[3 + c] + O[3 * r + 2] * O[6 + c];
        const double c1 = (1.0 - std::cos(theta)) / theta_sq;
        const double c2 = (theta - std::sin(theta)) / (theta_sq * theta);
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c1 * O[i] + c2 * O2[i];
    }
    T.t = {V[0] * a[0] + V[1] * a[1] + V[2] * a[2], V[3] * a[0] + V[4] * a[1] + V[5] * a[2],
           V[6] * a[0] + V[7] * a[1] + V[8] * a[2]};
    return T;
}

// exp(dx) * T   (local_ba.cpp:173)
static inline SE3 left_update(const double dx[6], const SE3& T) {
    const SE3 E = se3_exp(dx);
    SE3 R;
    R.q = quat_mul_normalized(E.q, T.q);
    const Vec3 rt = rotate(E.q, T.t);
    R.t = {E.t.x + rt.x, E.t.y + rt.y, E.t.z + rt.z};
    return R;
}

// Eigen::LDLT<Matrix<double,N,N>> (Lower) compute + solve.  A is row-major N x N (lower used).
template <int N>
static inline void ldlt_solve(double A[N * N], const double b[N], double x[N]) {
    int tr[N];
    for (int k = 0; k < N; ++k) {
        int big = k;
        double bv = std::fabs(A[k * N + k]);
        for (int i = k + 1; i < N; ++i)
            if (std::fabs(A[i * N + i]) > bv) { bv = std::fabs(A[i * N + i]); big = i; }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; ++j) std::swap(A[k * N + j], A[big * N + j]);
            for (int i = big + 1; i < N; ++i) std::swap(A[i * N + k], A[i * N + big]);
            std::swap(A[k * N + k], A[big * N + big]);
            for (int i = k + 1; i < big; ++i) {
                const double tmp = A[i * N + k];
                A[i * N + k] = A[big * N + i];
                A[big * N + i] = tmp;
            }
        }
        double temp[N];
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = A[j * N + j] * A[k * N + j];
            double s = 0;
            for (int j = 0; j < k; ++j) s += A[k * N + j] * temp[j];
            A[k * N + k] -= s;
            for (int i = k + 1; i < N; ++i) {
                double t = 0;
                for (int j = 0; j < k; ++j) t += A[i * N + j] * temp[j];
                A[i * N + k] -= t;
            }
        }
        const double akk = A[k * N + k];
        if (std::fabs(akk) > 0.0)
            for (int i = k + 1; i < N; ++i) A[i * N + k] /= akk;
    }
    for (int i = 0; i < N; ++i) x[i] = b[i];
    for (int k = 0; k < N; ++k) std::swap(x[k], x[tr[k]]);
    for (int i = 0; i < N; ++i)
        for (int r = i + 1; r < N; ++r) x[r] -= x[i] * A[r * N + i];
    for (int i = 0; i < N; ++i) {
        const double d = A[i * N + i];
        x[i] = std::fabs(d) > std::numeric_limits<double>::min() ? x[i] / d : 0.0;
    }
    for (int i = N - 1; i >= 0; --i) {
        double s = 0;
        for (int j = i + 1; j < N; ++j) s += A[j * N + i] * x[j];
        x[i] -= s;
    }
    for (int k = N - 1; k >= 0; --k) std::swap(x[k], x[tr[k]]);
}

static inline bool all_finite(const double* v, int n) {
    for (int i = 0; i < n; ++i)
        if (!std::isfinite(v[i])) return false;
    return true;
}

struct Cam { double fx, fy, cx, cy; };

// ProjectToPixel (projection.h:11-31)
static inline bool project(const Cam& c, const SE3& T, const Vec3& pw, double uv[2], Vec3& pc) {
    pc = transform(T, pw);
    if (pc.z <= 1e-6) return false;
    const double inv_z = 1.0 / pc.z;
    const double x = pc.x * inv_z, y = pc.y * inv_z;
    uv[0] = c.fx * x + c.cx;
    uv[1] = c.fy * y + c.cy;
    return true;
}

// ProjectionJacobian (local_ba.cpp:15-24), row-major 2x3
static inline void proj_jac(const Cam& c, const Vec3& pc, double J[6]) {
    const double x = pc.x, y = pc.y, z = pc.z, z2 = z * z;
    J[0] = c.fx / z; J[1] = 0.0;        J[2] = -c.fx * x / z2;
    J[3] = 0.0;      J[4] = c.fy / z;   J[5] = -c.fy * y / z2;
}

// PoseJacobian (local_ba.cpp:26-33): Jp * [I | -hat(pc)], row-major 2x6
static inline void pose_jac(const Cam& c, const Vec3& pc, double J[12]) {
    double Jp[6];
    proj_jac(c, pc, Jp);
    const double S[18] = {1, 0, 0, 0, pc.z, -pc.y,   // J_se3 (3x6)
                          0, 1, 0, -pc.z, 0, pc.x,
                          0, 0, 1, pc.y, -pc.x, 0};
    for (int r = 0; r < 2; ++r)
        for (int col = 0; col < 6; ++col)
            J[6 * r + col] = Jp[3 * r] * S[col] + Jp[3 * r + 1] * S[6 + col] + Jp[3 * r + 2] * S[12 + col];
}

static inline double huber(double e, double d) { return e <= d ? 1.0 : d / e; }  // local_ba.cpp:35-40

}  // namespace orc_ba
