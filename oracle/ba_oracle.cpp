// ba_oracle.cpp — CPU restatement of LocalBA::Optimize.  TEST INFRASTRUCTURE ONLY.
//
// Line-for-line restatement of /root/reference/core/backend/local_ba.cpp:66-249 (alternating
// pose / landmark Gauss-Newton, including the reference's b = -J^T e step sign :185,:253, the
// 5 px gate :177,:243 and the relative-cost stop :269-276), ProjectToPixel
// (core/common/projection.h:11-31), ProjectionJacobian / PoseJacobian / HuberWeight
// (local_ba.cpp:15-40) and SelectKeyFrames (:42-62).  Third-party pieces restated from their
// published algorithms (Eigen 3 / Sophus, unpinned versions, vcpkg.json):
//   - Eigen::LDLT (diagonal pivoting, ldlt_inplace::unblocked + _solve_impl),
//   - Sophus::SE3d::exp / SO3::expAndTheta, SO3 product with renormalisation,
//     quaternion point rotation (Eigen _transformVector), Quaternion::toRotationMatrix.
// The landmark-observation iteration order of the reference is std::unordered_map order
// (landmark.h:47-48,65) and therefore implementation-defined; this oracle uses the snapshot
// order.  Build: -O2 -ffp-contract=off.
#include "oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <limits>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

struct Vec3 { double x, y, z; };
struct Quat { double x, y, z, w; };
struct SE3 { Quat q; Vec3 t; };

inline Vec3 cross(const Vec3& a, const Vec3& b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// Eigen QuaternionBase::_transformVector (Sophus SO3 * point)
inline Vec3 rotate(const Quat& q, const Vec3& v) {
    const Vec3 qv{q.x, q.y, q.z};
    Vec3 uv = cross(qv, v);
    uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
    const Vec3 c = cross(qv, uv);
    return {v.x + q.w * uv.x + c.x, v.y + q.w * uv.y + c.y, v.z + q.w * uv.z + c.z};
}

inline Vec3 transform(const SE3& T, const Vec3& p) {
    const Vec3 r = rotate(T.q, p);
    return {r.x + T.t.x, r.y + T.t.y, r.z + T.t.z};
}

// Eigen Quaternion::toRotationMatrix
void rotation_matrix(const Quat& q, double R[9]) {
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

// Sophus SO3 product + normalize()
Quat quat_mul_normalized(const Quat& a, const Quat& b) {
    Quat r{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
           a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
           a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x,
           a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
    const double n = std::sqrt(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w);
    r.x /= n; r.y /= n; r.z /= n; r.w /= n;
    return r;
}

// Sophus::SE3d::exp(a), a = (upsilon, omega)
SE3 se3_exp(const double a[6]) {
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
SE3 left_update(const double dx[6], const SE3& T) {
    const SE3 E = se3_exp(dx);
    SE3 R;
    R.q = quat_mul_normalized(E.q, T.q);
    const Vec3 rt = rotate(E.q, T.t);
    R.t = {E.t.x + rt.x, E.t.y + rt.y, E.t.z + rt.z};
    return R;
}

// Eigen::LDLT<Matrix<double,N,N>> (Lower) compute + solve.  A is row-major N x N (lower used).
template <int N>
void ldlt_solve(double A[N * N], const double b[N], double x[N]) {
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

inline bool all_finite(const double* v, int n) {
    for (int i = 0; i < n; ++i)
        if (!std::isfinite(v[i])) return false;
    return true;
}

struct Cam { double fx, fy, cx, cy; };

// ProjectToPixel (projection.h:11-31)
inline bool project(const Cam& c, const SE3& T, const Vec3& pw, double uv[2], Vec3& pc) {
    pc = transform(T, pw);
    if (pc.z <= 1e-6) return false;
    const double inv_z = 1.0 / pc.z;
    const double x = pc.x * inv_z, y = pc.y * inv_z;
    uv[0] = c.fx * x + c.cx;
    uv[1] = c.fy * y + c.cy;
    return true;
}

// ProjectionJacobian (local_ba.cpp:15-24), row-major 2x3
inline void proj_jac(const Cam& c, const Vec3& pc, double J[6]) {
    const double x = pc.x, y = pc.y, z = pc.z, z2 = z * z;
    J[0] = c.fx / z; J[1] = 0.0;        J[2] = -c.fx * x / z2;
    J[3] = 0.0;      J[4] = c.fy / z;   J[5] = -c.fy * y / z2;
}

// PoseJacobian (local_ba.cpp:26-33): Jp * [I | -hat(pc)], row-major 2x6
inline void pose_jac(const Cam& c, const Vec3& pc, double J[12]) {
    double Jp[6];
    proj_jac(c, pc, Jp);
    const double S[18] = {1, 0, 0, 0, pc.z, -pc.y,   // J_se3 (3x6)
                          0, 1, 0, -pc.z, 0, pc.x,
                          0, 0, 1, pc.y, -pc.x, 0};
    for (int r = 0; r < 2; ++r)
        for (int col = 0; col < 6; ++col)
            J[6 * r + col] = Jp[3 * r] * S[col] + Jp[3 * r + 1] * S[6 + col] + Jp[3 * r + 2] * S[12 + col];
}

inline double huber(double e, double d) { return e <= d ? 1.0 : d / e; }  // local_ba.cpp:35-40

}  // namespace

extern "C" int orc_ba_optimize_map(orc_map_view* m, uint64_t ref_kf_id, int has_ref,
                                   const orc_ba_options* opt, orc_ba_stats* st) {
    orc_ba_stats local{};
    if (!st) st = &local;
    *st = orc_ba_stats{};
    st->status = 1;
    st->gate_margin = std::numeric_limits<double>::infinity();
    if (!m || m->n_kf == 0) return 0;

    // Map::keyframes_ is a std::map ordered by id; Map::landmarks_ is keyed by id.
    std::map<uint64_t, int> kf_by_id;
    for (int i = 0; i < m->n_kf; ++i) kf_by_id[m->kf_id[i]] = i;
    std::unordered_map<uint64_t, int> lm_by_id;
    for (int i = 0; i < m->n_lm; ++i) lm_by_id[m->lm_id[i]] = i;

    // SelectKeyFrames (local_ba.cpp:42-62)
    const int window = std::max(1, (int)opt->window_size);
    const uint64_t max_id = has_ref ? ref_kf_id : kf_by_id.rbegin()->first;
    std::vector<int> kfs;
    for (auto it = kf_by_id.rbegin(); it != kf_by_id.rend() && (int)kfs.size() < window; ++it) {
        if (it->first > max_id) continue;
        kfs.push_back(it->second);
    }
    std::reverse(kfs.begin(), kfs.end());
    st->n_window_kf = (int)kfs.size();
    if (kfs.size() < 2) return 0;
    std::unordered_set<uint64_t> local_ids;
    for (int k : kfs) local_ids.insert(m->kf_id[k]);

    // landmark set (local_ba.cpp:83-108)
    std::unordered_set<uint64_t> lm_ids;
    for (int k : kfs)
        for (int64_t f = m->kf_feat_ptr[k]; f < m->kf_feat_ptr[k + 1]; ++f)
            if (m->feat_flags[f] & 1) lm_ids.insert(m->feat_lm_id[f]);
    std::vector<int> lms;
    for (uint64_t id : lm_ids) {
        auto it = lm_by_id.find(id);
        if (it == lm_by_id.end()) continue;
        const int l = it->second;
        if (m->lm_bad[l]) continue;
        if (m->lm_obs_ptr[l + 1] - m->lm_obs_ptr[l] < (int64_t)opt->min_point_observations) continue;
        lms.push_back(l);
    }
    std::sort(lms.begin(), lms.end());  // update order is irrelevant (independent per landmark)
    st->n_window_kf = (int)kfs.size();
    st->n_landmarks = (int)lms.size();
    if (lms.empty()) return 0;
    st->status = 0;

    auto pose_of = [&](int k) {
        const double* p = m->kf_pose + 7 * k;
        return SE3{{p[0], p[1], p[2], p[3]}, {p[4], p[5], p[6]}};
    };
    auto set_pose = [&](int k, const SE3& T) {
        double* p = m->kf_pose + 7 * k;
        p[0] = T.q.x; p[1] = T.q.y; p[2] = T.q.z; p[3] = T.q.w;
        p[4] = T.t.x; p[5] = T.t.y; p[6] = T.t.z;
    };
    auto cam_of = [&](int k) {
        const double* c = m->kf_intr + 4 * k;
        return Cam{c[0], c[1], c[2], c[3]};
    };
    auto margin = [&](double e) {
        st->gate_margin = std::min(st->gate_margin, std::fabs(e - opt->max_reproj_error));
    };

    double last_cost = std::numeric_limits<double>::max();
    for (int iter = 0; iter < opt->max_iterations; ++iter) {
        double total_cost = 0.0;
        int total_obs = 0;
        st->iterations = iter + 1;

        // === Pose optimization (fix landmarks) === local_ba.cpp:116-174
        for (int k : kfs) {
            if (!m->kf_has_cam[k]) continue;
            const Cam cam = cam_of(k);
            double H[36] = {0}, b[6] = {0};
            int obs = 0;
            for (int64_t f = m->kf_feat_ptr[k]; f < m->kf_feat_ptr[k + 1]; ++f) {
                const uint8_t fl = m->feat_flags[f];
                if (!(fl & 1) || (fl & 2)) continue;
                auto it = lm_by_id.find(m->feat_lm_id[f]);
                if (it == lm_by_id.end() || m->lm_bad[it->second]) continue;
                const double* P = m->lm_pos + 3 * it->second;
                double proj[2];
                Vec3 pc;
                if (!project(cam, pose_of(k), {P[0], P[1], P[2]}, proj, pc)) continue;
                const double e[2] = {m->feat_uv[2 * f] - proj[0], m->feat_uv[2 * f + 1] - proj[1]};
                const double en = std::sqrt(e[0] * e[0] + e[1] * e[1]);
                margin(en);
                if (en > opt->max_reproj_error) continue;
                const double w = huber(en, opt->huber_delta);
                double J[12];
                pose_jac(cam, pc, J);
                for (int i = 0; i < 6; ++i)
                    for (int j = 0; j < 6; ++j)
                        H[6 * i + j] += (w * J[i]) * J[j] + (w * J[6 + i]) * J[6 + j];
                for (int i = 0; i < 6; ++i) b[i] += w * ((-J[i]) * e[0] + (-J[6 + i]) * e[1]);
                total_cost += w * (e[0] * e[0] + e[1] * e[1]);
                total_obs++;
                obs++;
            }
            if (obs < opt->min_pose_observations) continue;
            for (int i = 0; i < 6; ++i) H[7 * i] += 1e-6;
            double dx[6];
            ldlt_solve<6>(H, b, dx);
            if (!all_finite(dx, 6)) continue;
            set_pose(k, left_update(dx, pose_of(k)));
        }

        // === Landmark optimization (fix poses) === local_ba.cpp:176-238
        for (int l : lms) {
            if (m->lm_bad[l]) continue;
            double H[9] = {0}, b[3] = {0};
            int obs = 0;
            double* P = m->lm_pos + 3 * l;
            for (int64_t o = m->lm_obs_ptr[l]; o < m->lm_obs_ptr[l + 1]; ++o) {
                const uint64_t kid = m->obs_kf_id[o];
                if (!local_ids.count(kid)) continue;
                auto kit = kf_by_id.find(kid);
                if (kit == kf_by_id.end()) continue;
                const int k = kit->second;
                if (!m->kf_has_cam[k]) continue;
                const uint64_t fi = m->obs_feat_idx[o];
                const int64_t nf = m->kf_feat_ptr[k + 1] - m->kf_feat_ptr[k];
                if (fi >= (uint64_t)nf) continue;
                const int64_t f = m->kf_feat_ptr[k] + (int64_t)fi;
                const uint8_t fl = m->feat_flags[f];
                if (!(fl & 1) || (fl & 2) || m->feat_lm_id[f] != m->lm_id[l]) continue;
                const Cam cam = cam_of(k);
                const SE3 T = pose_of(k);
                double proj[2];
                Vec3 pc;
                if (!project(cam, T, {P[0], P[1], P[2]}, proj, pc)) continue;
                const double e[2] = {m->feat_uv[2 * f] - proj[0], m->feat_uv[2 * f + 1] - proj[1]};
                const double en = std::sqrt(e[0] * e[0] + e[1] * e[1]);
                margin(en);
                if (en > opt->max_reproj_error) continue;
                const double w = huber(en, opt->huber_delta);
                double Jp[6], R[9], J[6];
                proj_jac(cam, pc, Jp);
                rotation_matrix(T.q, R);
                for (int r = 0; r < 2; ++r)
                    for (int c = 0; c < 3; ++c)
                        J[3 * r + c] = Jp[3 * r] * R[c] + Jp[3 * r + 1] * R[3 + c] + Jp[3 * r + 2] * R[6 + c];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)
                        H[3 * i + j] += (w * J[i]) * J[j] + (w * J[3 + i]) * J[3 + j];
                for (int i = 0; i < 3; ++i) b[i] += w * ((-J[i]) * e[0] + (-J[3 + i]) * e[1]);
                obs++;
            }
            if (obs < opt->min_point_observations) continue;
            for (int i = 0; i < 3; ++i) H[4 * i] += 1e-6;
            double dp[3];
            ldlt_solve<3>(H, b, dp);
            if (!all_finite(dp, 3)) continue;
            P[0] += dp[0]; P[1] += dp[1]; P[2] += dp[2];
        }

        if (iter < 16) { st->cost[iter] = total_cost; st->obs[iter] = total_obs; }
        if (total_obs == 0) break;
        if (std::fabs(last_cost - total_cost) < 1e-6 * last_cost) break;
        last_cost = total_cost;
    }
    return 0;
}
