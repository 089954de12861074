// ba_oracle.cpp — CPU restatement of LocalBA::Optimize.  TEST INFRASTRUCTURE ONLY.
//
// Line-for-line restatement of /root/reference/core/backend/local_ba.cpp:66-249 (alternating
// pose / landmark Gauss-Newton, including the reference's b = -J^T e step sign :156,:224, the
// 5 px gate :148,:214 and the stop rule :240-247), ProjectToPixel
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
#include <chrono>
#include <cmath>
#include <limits>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "ba_math.h"

using namespace orc_ba;

// wall time of the last call's two parts (bench.py's CPU baseline reports them apart): the window /
// landmark-set selection (local_ba.cpp:66-108, what a GPU plan build replaces) and the iterations
// (local_ba.cpp:110-248, what a GPU plan run replaces)
// (per thread: bench.py's multi-threaded CPU baseline runs frames on several threads at once)
static thread_local double g_setup_s = 0.0, g_iter_s = 0.0;

extern "C" void orc_ba_last_timing(double* out2) {
    out2[0] = g_setup_s;
    out2[1] = g_iter_s;
}

extern "C" int orc_ba_optimize_map(orc_map_view* m, uint64_t ref_kf_id, int has_ref,
                                   const orc_ba_options* opt, orc_ba_stats* st) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    g_setup_s = g_iter_s = 0.0;
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

    const auto t1 = clk::now();
    g_setup_s = std::chrono::duration<double>(t1 - t0).count();
    struct IterTimer {  // stops at every return below
        clk::time_point t;
        ~IterTimer() { g_iter_s = std::chrono::duration<double>(clk::now() - t).count(); }
    } iter_timer{t1};
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
