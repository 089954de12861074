// sba_oracle.cpp — CPU restatement of the Schur-complement joint BA of
// visionx-slam_amd/csrc/sba.hip.  TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// The reference has no joint solver: its LocalBA alternates per-keyframe and per-landmark steps
// (core/backend/local_ba.cpp:116-238).  BASELINE.json's north_star asks for the Schur-complement
// reduction into the dense 6N x 6N pose Hessian and a dense pose solve; SURVEY.md §8f rank 4 lists
// it as "not in the reference, validated against its own CPU restatement".  This file is that
// restatement, written with plain loops and a textbook dense Cholesky, independent of the GPU
// tiling.  What it keeps from the reference:
//   - keyframe window and landmark set: SelectKeyFrames + filter (local_ba.cpp:42-108),
//   - observations: the pose stage's feature-driven set (local_ba.cpp:126-138),
//   - residual e = uv - ProjectToPixel (projection.h:11-31), gates z > 1e-6 and |e| <= max_reproj,
//     Huber weight (local_ba.cpp:35-40), PoseJacobian (left perturbation, (upsilon, omega)),
//     landmark Jacobian Jp * R (local_ba.cpp:15-33, :219-221), T <- exp(dx) T, p <- p + dp,
//     the 1e-6 diagonal regulariser (local_ba.cpp:167, :232).
// What is new (documented in DESIGN.md §10):
//   - one joint Gauss-Newton system with b = +J^T W e (the reference's -J^T e diverges),
//   - Marquardt damping H_ii += lambda * H_ii on poses and landmarks, accept / reject on the
//     truncated Huber cost: rho(e) = e^2 (e <= delta), 2 delta e - delta^2 otherwise, and the
//     constant rho(max_reproj_error) for a gated observation (so observations re-entering the
//     gate lower the cost instead of raising it),
//   - the oldest `fixed_keyframes` window keyframes (and keyframes without a camera) held fixed;
//     a landmark with fewer valid observations than min_point_observations in an assembly is
//     held fixed for that iteration (the reference skips it, local_ba.cpp:228-229).
#include <cmath>
#include <limits>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "ba_math.h"
#include "oracle.h"

using namespace orc_ba;

namespace {

// Smallest Marquardt damping after accepted steps: keeps the directions the cost does not see
// (the monocular scale; whole gauge of a component without a fixed keyframe) regularised.
constexpr double kLambdaMin = 1e-6;

struct Obs {
    int kf;       // window row
    int lm;       // map landmark index
    int slot;     // optimised landmark slot, -1 for a fixed landmark
    double u, v;
};

struct Problem {
    int status = 1;
    int nk = 0;
    std::vector<int> win;          // map keyframe index per row
    std::vector<char> fixed;       // per row
    std::vector<int> opt;          // map landmark index per slot
    std::vector<Obs> obs;          // slot-major for optimised landmarks, then fixed-landmark ones
    std::vector<int> lm_ptr;       // slot -> first obs (n_opt + 1)
};

// Window + landmark set (local_ba.cpp:42-108) and the observation set (local_ba.cpp:126-138).
void build(const orc_map_view* m, uint64_t ref, int has_ref, const orc_sba_options* o, Problem& P) {
    P = Problem{};
    if (!m || m->n_kf == 0) return;
    std::map<uint64_t, int> kf_by_id;
    for (int i = 0; i < m->n_kf; ++i) kf_by_id[m->kf_id[i]] = i;
    std::unordered_map<uint64_t, int> lm_by_id;
    for (int i = 0; i < m->n_lm; ++i) lm_by_id[m->lm_id[i]] = i;
    const int window = std::max(1, (int)o->window_size);
    const uint64_t max_id = has_ref ? ref : kf_by_id.rbegin()->first;
    for (auto it = kf_by_id.rbegin(); it != kf_by_id.rend() && (int)P.win.size() < window; ++it) {
        if (it->first > max_id) continue;
        P.win.push_back(it->second);
    }
    std::reverse(P.win.begin(), P.win.end());
    P.nk = (int)P.win.size();
    if (P.nk < 2) return;
    std::unordered_set<uint64_t> lm_ids;
    for (int k : P.win)
        for (int64_t f = m->kf_feat_ptr[k]; f < m->kf_feat_ptr[k + 1]; ++f)
            if (m->feat_flags[f] & 1) lm_ids.insert(m->feat_lm_id[f]);
    for (uint64_t id : lm_ids) {
        auto it = lm_by_id.find(id);
        if (it == lm_by_id.end()) continue;
        const int l = it->second;
        if (m->lm_bad[l]) continue;
        if (m->lm_obs_ptr[l + 1] - m->lm_obs_ptr[l] < (int64_t)o->min_point_observations) continue;
        P.opt.push_back(l);
    }
    std::sort(P.opt.begin(), P.opt.end());
    if (P.opt.empty()) return;
    P.status = 0;
    std::vector<int> slot_of(m->n_lm, -1);
    for (int s = 0; s < (int)P.opt.size(); ++s) slot_of[P.opt[s]] = s;
    P.fixed.assign(P.nk, 0);
    std::vector<std::vector<Obs>> per_slot(P.opt.size());
    std::vector<Obs> fixed_obs;
    for (int r = 0; r < P.nk; ++r) {
        const int k = P.win[r];
        P.fixed[r] = (r < o->fixed_keyframes || !m->kf_has_cam[k]) ? 1 : 0;
        if (!m->kf_has_cam[k]) continue;
        for (int64_t f = m->kf_feat_ptr[k]; f < m->kf_feat_ptr[k + 1]; ++f) {
            const uint8_t fl = m->feat_flags[f];
            if (!(fl & 1) || (fl & 2)) continue;
            auto it = lm_by_id.find(m->feat_lm_id[f]);
            if (it == lm_by_id.end() || m->lm_bad[it->second]) continue;
            const int l = it->second;
            Obs ob{r, l, slot_of[l], m->feat_uv[2 * f], m->feat_uv[2 * f + 1]};
            if (ob.slot >= 0)
                per_slot[ob.slot].push_back(ob);
            else
                fixed_obs.push_back(ob);
        }
    }
    P.lm_ptr.assign(P.opt.size() + 1, 0);
    for (size_t s = 0; s < P.opt.size(); ++s) {
        for (const Obs& ob : per_slot[s]) P.obs.push_back(ob);
        P.lm_ptr[s + 1] = (int)P.obs.size();
    }
    for (const Obs& ob : fixed_obs) P.obs.push_back(ob);
}

struct State {
    std::vector<SE3> T;            // per window row
    std::vector<Vec3> p;           // per optimised slot
};

// Inverse of the symmetric 3x3 {a b c; b d e; c e f} by its adjugate (same formula as the GPU).
void sym3_inverse(const double V[6], double out[6]) {
    const double a = V[0], b = V[1], c = V[2], d = V[3], e = V[4], f = V[5];
    const double A = d * f - e * e, B = c * e - b * f, C = b * e - c * d;
    const double D = a * f - c * c, E = b * c - a * e, F = a * d - b * b;
    const double det = a * A + b * B + c * C;
    const double id = 1.0 / det;
    out[0] = A * id; out[1] = B * id; out[2] = C * id; out[3] = D * id; out[4] = E * id; out[5] = F * id;
}

inline void sym3_mul(const double Vi[6], const double x[3], double y[3]) {
    y[0] = Vi[0] * x[0] + Vi[1] * x[1] + Vi[2] * x[2];
    y[1] = Vi[1] * x[0] + Vi[3] * x[1] + Vi[4] * x[2];
    y[2] = Vi[2] * x[0] + Vi[4] * x[1] + Vi[5] * x[2];
}

struct System {
    int n = 0;
    std::vector<double> S, rhs;    // n x n (full, symmetric), n
    std::vector<double> Vinv;      // 6 per slot (damped landmark block inverse)
    std::vector<double> gp;        // 3 per slot
    std::vector<double> W;         // 18 per optimised-landmark observation (6 x 3, row-major)
    double cost = 0.0;
    int count = 0;
};

// One assembly at state X with damping lambda: cost, reduced pose system S x = rhs and the
// per-landmark / per-observation blocks the back-substitution needs.
// Sharded form (shard_count > 1, csrc/sba.hip): only the observations of this rank's landmarks
// (splitmix64(landmark id) mod shard_count == shard_rank, optimised and fixed alike) are assembled,
// and with finish = false the pose damping and the fixed-keyframe gauge are left out — they are
// applied once after the all-reduce of the ranks' partial systems; HTd (n) then receives this
// shard's pose-block diagonals, which that damping needs summed over the ranks too.
inline uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

void assemble(const orc_map_view* m, const Problem& P, const orc_sba_options* o, const State& X, double lambda,
              System& sys, int shard_rank = 0, int shard_count = 1, bool finish = true, double* HTd = nullptr) {
    const int nk = P.nk, n = 6 * nk;
    const int n_opt = (int)P.opt.size();
    const int n_oo = P.lm_ptr[n_opt];
    sys.n = n;
    sys.S.assign((size_t)n * n, 0.0);
    sys.rhs.assign(n, 0.0);
    sys.Vinv.assign((size_t)n_opt * 6, 0.0);
    sys.gp.assign((size_t)n_opt * 3, 0.0);
    sys.W.assign((size_t)n_oo * 18, 0.0);
    sys.cost = 0.0;
    sys.count = 0;
    std::vector<double> HT((size_t)nk * 36, 0.0), gT((size_t)nk * 6, 0.0);
    std::vector<double> Y((size_t)n_oo * 18, 0.0);
    std::vector<double> V((size_t)n_opt * 6, 0.0);
    std::vector<int> cnt(n_opt, 0);
    const double delta = o->huber_delta, me = o->max_reproj_error;
    const double rho_gate = me <= delta ? me * me : 2.0 * delta * me - delta * delta;
    for (int i = 0; i < (int)P.obs.size(); ++i) {
        const Obs& ob = P.obs[i];
        if (shard_count > 1 && (int)(splitmix64(m->lm_id[ob.lm]) % (uint64_t)shard_count) != shard_rank) continue;
        const int k = P.win[ob.kf];
        const double* ci = m->kf_intr + 4 * k;
        const Cam cam{ci[0], ci[1], ci[2], ci[3]};
        const SE3& T = X.T[ob.kf];
        const double* pw0 = m->lm_pos + 3 * ob.lm;
        const Vec3 pw = ob.slot >= 0 ? X.p[ob.slot] : Vec3{pw0[0], pw0[1], pw0[2]};
        double proj[2];
        Vec3 pc;
        // gated observations (behind the camera / beyond max_reproj_error) cost the constant
        // rho(max_reproj_error): the truncated robust cost the accept / reject test compares
        if (!project(cam, T, pw, proj, pc)) {
            sys.cost += rho_gate;
            continue;
        }
        const double e[2] = {ob.u - proj[0], ob.v - proj[1]};
        const double en = std::sqrt(e[0] * e[0] + e[1] * e[1]);
        if (en > o->max_reproj_error) {
            sys.cost += rho_gate;
            continue;
        }
        const double w = huber(en, delta);
        sys.cost += en <= delta ? en * en : 2.0 * delta * en - delta * delta;
        sys.count++;
        double JT[12], Jp[6], R[9], JP[6];
        pose_jac(cam, pc, JT);
        proj_jac(cam, pc, Jp);
        rotation_matrix(T.q, R);
        for (int r = 0; r < 2; ++r)
            for (int c = 0; c < 3; ++c)
                JP[3 * r + c] = Jp[3 * r] * R[c] + Jp[3 * r + 1] * R[3 + c] + Jp[3 * r + 2] * R[6 + c];
        double* H = HT.data() + 36 * ob.kf;
        double* g = gT.data() + 6 * ob.kf;
        for (int a = 0; a < 6; ++a) {
            for (int b = 0; b < 6; ++b) H[6 * a + b] += w * (JT[a] * JT[b] + JT[6 + a] * JT[6 + b]);
            g[a] += w * (JT[a] * e[0] + JT[6 + a] * e[1]);
        }
        if (ob.slot < 0) continue;
        cnt[ob.slot]++;
        double* Vs = V.data() + 6 * ob.slot;
        double* gs = sys.gp.data() + 3 * ob.slot;
        const int idx[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
        for (int t = 0; t < 6; ++t)
            Vs[t] += w * (JP[idx[t][0]] * JP[idx[t][1]] + JP[3 + idx[t][0]] * JP[3 + idx[t][1]]);
        for (int a = 0; a < 3; ++a) gs[a] += w * (JP[a] * e[0] + JP[3 + a] * e[1]);
        double* Wo = sys.W.data() + 18 * i;
        for (int a = 0; a < 6; ++a)
            for (int b = 0; b < 3; ++b) Wo[3 * a + b] = w * (JT[a] * JP[b] + JT[6 + a] * JP[3 + b]);
    }
    // damped landmark blocks and their inverses
    for (int s = 0; s < n_opt; ++s) {
        double Vd[6];
        const double* Vs = V.data() + 6 * s;
        for (int t = 0; t < 6; ++t) Vd[t] = Vs[t];
        Vd[0] += lambda * Vs[0] + 1e-6;
        Vd[3] += lambda * Vs[3] + 1e-6;
        Vd[5] += lambda * Vs[5] + 1e-6;
        // a landmark with fewer valid observations than min_point_observations is held fixed in
        // this iteration (V^-1 = 0: no Schur term, dp = 0), as local_ba.cpp:228-229 skips it
        if (cnt[s] >= o->min_point_observations)
            sym3_inverse(Vd, sys.Vinv.data() + 6 * s);
        for (int i = P.lm_ptr[s]; i < P.lm_ptr[s + 1]; ++i) {
            const double* Wo = sys.W.data() + 18 * i;
            double* Yo = Y.data() + 18 * i;
            for (int a = 0; a < 6; ++a) sym3_mul(sys.Vinv.data() + 6 * s, Wo + 3 * a, Yo + 3 * a);
        }
    }
    // S = blockdiag(H_TT) - sum_l sum_{o1, o2 in l} Y_o1 W_o2^T ;  rhs = g_T - sum_o Y_o g_p
    for (int r = 0; r < nk; ++r)
        for (int a = 0; a < 6; ++a) {
            for (int b = 0; b < 6; ++b) sys.S[(size_t)(6 * r + a) * n + 6 * r + b] = HT[36 * r + 6 * a + b];
            sys.rhs[6 * r + a] = gT[6 * r + a];
        }
    for (int s = 0; s < n_opt; ++s)
        for (int i1 = P.lm_ptr[s]; i1 < P.lm_ptr[s + 1]; ++i1) {
            const int r1 = P.obs[i1].kf;
            const double* Y1 = Y.data() + 18 * i1;
            for (int a = 0; a < 6; ++a)
                sys.rhs[6 * r1 + a] -= Y1[3 * a] * sys.gp[3 * s] + Y1[3 * a + 1] * sys.gp[3 * s + 1] +
                                       Y1[3 * a + 2] * sys.gp[3 * s + 2];
            for (int i2 = P.lm_ptr[s]; i2 < P.lm_ptr[s + 1]; ++i2) {
                const int r2 = P.obs[i2].kf;
                const double* W2 = sys.W.data() + 18 * i2;
                for (int a = 0; a < 6; ++a)
                    for (int b = 0; b < 6; ++b)
                        sys.S[(size_t)(6 * r1 + a) * n + 6 * r2 + b] -=
                            Y1[3 * a] * W2[3 * b] + Y1[3 * a + 1] * W2[3 * b + 1] + Y1[3 * a + 2] * W2[3 * b + 2];
            }
        }
    if (HTd)
        for (int r = 0; r < nk; ++r)
            for (int a = 0; a < 6; ++a) HTd[6 * r + a] = HT[36 * r + 7 * a];
    if (!finish) return;
    // pose damping and the gauge: fixed keyframes get identity rows / columns and rhs 0
    for (int r = 0; r < nk; ++r) {
        if (P.fixed[r]) {
            for (int a = 0; a < 6; ++a) {
                for (int c = 0; c < n; ++c) {
                    sys.S[(size_t)(6 * r + a) * n + c] = 0.0;
                    sys.S[(size_t)c * n + 6 * r + a] = 0.0;
                }
                sys.S[(size_t)(6 * r + a) * n + 6 * r + a] = 1.0;
                sys.rhs[6 * r + a] = 0.0;
            }
            continue;
        }
        for (int a = 0; a < 6; ++a) sys.S[(size_t)(6 * r + a) * (n + 1)] += lambda * HT[36 * r + 7 * a] + 1e-6;
    }
}

// Dense Cholesky S = L L^T (lower) and the solve; false if a pivot is not positive.
bool cholesky_solve(std::vector<double> A, int n, const std::vector<double>& b, std::vector<double>& x) {
    for (int j = 0; j < n; ++j) {
        double d = A[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
        if (!(d > 0.0)) return false;
        const double ljj = std::sqrt(d);
        A[(size_t)j * n + j] = ljj;
        for (int i = j + 1; i < n; ++i) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; ++k) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
            A[(size_t)i * n + j] = s / ljj;
        }
    }
    x = b;
    for (int i = 0; i < n; ++i) {
        double s = x[i];
        for (int k = 0; k < i; ++k) s -= A[(size_t)i * n + k] * x[k];
        x[i] = s / A[(size_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = x[i];
        for (int k = i + 1; k < n; ++k) s -= A[(size_t)k * n + i] * x[k];
        x[i] = s / A[(size_t)i * n + i];
    }
    for (double v : x)
        if (!std::isfinite(v)) return false;
    return true;
}

State initial_state(const orc_map_view* m, const Problem& P) {
    State X;
    for (int r = 0; r < P.nk; ++r) {
        const double* p = m->kf_pose + 7 * P.win[r];
        X.T.push_back(SE3{{p[0], p[1], p[2], p[3]}, {p[4], p[5], p[6]}});
    }
    for (int l : P.opt) X.p.push_back({m->lm_pos[3 * l], m->lm_pos[3 * l + 1], m->lm_pos[3 * l + 2]});
    return X;
}

}  // namespace

extern "C" int orc_sba_system(const orc_map_view* m, uint64_t ref, int has_ref, const orc_sba_options* o,
                              double lambda, double* S, double* rhs, int n) {
    Problem P;
    build(m, ref, has_ref, o, P);
    if (P.status != 0) return 1;
    if (n != 6 * P.nk) return -1;
    System sys;
    assemble(m, P, o, initial_state(m, P), lambda, sys);
    for (size_t i = 0; i < sys.S.size(); ++i) S[i] = sys.S[i];
    for (int i = 0; i < n; ++i) rhs[i] = sys.rhs[i];
    return 0;
}

extern "C" int orc_sba_system_shard(const orc_map_view* m, uint64_t ref, int has_ref, const orc_sba_options* o,
                                    double lambda, int shard_rank, int shard_count, double* S, double* rhs,
                                    double* HTd, double* cost_count, int n) {
    Problem P;
    build(m, ref, has_ref, o, P);
    if (P.status != 0) return 1;
    if (n != 6 * P.nk || shard_count < 1 || shard_rank < 0 || shard_rank >= shard_count) return -1;
    System sys;
    assemble(m, P, o, initial_state(m, P), lambda, sys, shard_rank, shard_count, false, HTd);
    for (size_t i = 0; i < sys.S.size(); ++i) S[i] = sys.S[i];
    for (int i = 0; i < n; ++i) rhs[i] = sys.rhs[i];
    cost_count[0] = sys.cost;
    cost_count[1] = sys.count;
    return 0;
}

extern "C" int orc_sba_optimize_map(orc_map_view* m, uint64_t ref, int has_ref, const orc_sba_options* o,
                                    orc_sba_stats* st) {
    orc_sba_stats local{};
    if (!st) st = &local;
    *st = orc_sba_stats{};
    st->status = 1;
    Problem P;
    build(m, ref, has_ref, o, P);
    st->n_window_kf = P.nk;
    st->n_landmarks = (int)P.opt.size();
    if (P.status != 0) return 0;
    st->status = 0;
    const int n_opt = (int)P.opt.size();

    State best = initial_state(m, P), trial = best;
    bool eval_trial = false;
    double lambda = o->lambda_init, best_cost = 0.0;
    System sys;
    for (int it = 0; it < o->max_iterations; ++it) {
        assemble(m, P, o, eval_trial ? trial : best, lambda, sys);
        st->iterations = it + 1;
        if (it < 16) {
            st->cost[it] = sys.cost;
            st->obs[it] = sys.count;
        }
        int step;
        bool stop = false;
        if (it == 0) {
            best_cost = sys.cost;
            st->initial_cost = sys.cost;
            step = 2;
        } else if (eval_trial) {
            if (sys.cost < best_cost) {
                const double rel = (best_cost - sys.cost) / best_cost;
                best = trial;
                best_cost = sys.cost;
                lambda = std::max(lambda * 0.1, kLambdaMin);
                st->accepted++;
                step = 1;
                stop = rel < o->rel_tol;
            } else {
                lambda *= 10.0;
                step = 0;
                stop = lambda > 1e12;
            }
        } else {
            step = 3;
        }
        if (it < 16) st->step[it] = step;
        if (sys.count == 0) stop = true;
        if (stop || it + 1 == o->max_iterations) break;
        if (step == 0) {  // rejected: re-assemble at the best state with the larger damping
            eval_trial = false;
            continue;
        }
        std::vector<double> x;
        if (!cholesky_solve(sys.S, sys.n, sys.rhs, x)) {
            lambda *= 10.0;
            eval_trial = false;
            continue;
        }
        // back-substitution and the trial state
        trial = best;
        for (int r = 0; r < P.nk; ++r)
            if (!P.fixed[r]) trial.T[r] = left_update(&x[6 * r], best.T[r]);
        for (int s = 0; s < n_opt; ++s) {
            double q[3] = {sys.gp[3 * s], sys.gp[3 * s + 1], sys.gp[3 * s + 2]};
            for (int i = P.lm_ptr[s]; i < P.lm_ptr[s + 1]; ++i) {
                const double* Wo = sys.W.data() + 18 * i;
                const double* xo = &x[6 * P.obs[i].kf];
                for (int b = 0; b < 3; ++b)
                    for (int a = 0; a < 6; ++a) q[b] -= Wo[3 * a + b] * xo[a];
            }
            double dp[3];
            sym3_mul(sys.Vinv.data() + 6 * s, q, dp);
            if (std::isfinite(dp[0]) && std::isfinite(dp[1]) && std::isfinite(dp[2]))
                trial.p[s] = {best.p[s].x + dp[0], best.p[s].y + dp[1], best.p[s].z + dp[2]};
        }
        eval_trial = true;
    }
    st->lambda = lambda;
    st->final_cost = best_cost;
    for (int r = 0; r < P.nk; ++r) {
        double* p = m->kf_pose + 7 * P.win[r];
        const SE3& T = best.T[r];
        p[0] = T.q.x; p[1] = T.q.y; p[2] = T.q.z; p[3] = T.q.w;
        p[4] = T.t.x; p[5] = T.t.y; p[6] = T.t.z;
    }
    for (int s = 0; s < n_opt; ++s) {
        double* q = m->lm_pos + 3 * P.opt[s];
        q[0] = best.p[s].x; q[1] = best.p[s].y; q[2] = best.p[s].z;
    }
    return 0;
}
