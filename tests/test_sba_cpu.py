"""Schur-complement joint BA: CPU checks of the restatement (oracle/sba_oracle.cpp).

The joint solver is not in the reference, so its restatement is pinned
here by an independent numpy statement of the same damped Gauss-Newton step: residuals built from
the map arrays directly, the Jacobian by central finite differences (no analytic formula shared
with the oracle), the FULL (poses + landmarks) normal equations solved densely.  Eliminating the
landmarks is exact algebra, so the oracle's reduced system S = H_pp - H_pl H_ll^-1 H_lp and its
solution must equal the numpy ones to finite-difference accuracy.
"""
import numpy as np
import pytest

from vxslam import synth


def _quat_to_mat(q):
    return synth.quat_to_mat(np.asarray(q, float))


def _rotvec_mat(w):
    return synth.quat_to_mat(synth.quat_from_rotvec(np.asarray(w, float)))


def _problem(m, window, min_point=2):
    """Window = the last `window` keyframes (no reference keyframe), landmark set and the
    feature-driven observation set, as local_ba.cpp:42-138 (restated in numpy)."""
    order = np.argsort(m["kf_id"])
    win = order[-window:]
    lm_index = {int(v): i for i, v in enumerate(m["lm_id"])}
    obs = []  # (row, lm, u, v)
    ids = set()
    for r, k in enumerate(win):
        for f in range(m["kf_feat_ptr"][k], m["kf_feat_ptr"][k + 1]):
            if m["feat_flags"][f] & 1:
                ids.add(int(m["feat_lm_id"][f]))
            if not (m["feat_flags"][f] & 1) or (m["feat_flags"][f] & 2):
                continue
            l = lm_index.get(int(m["feat_lm_id"][f]))
            if l is None or m["lm_bad"][l]:
                continue
            obs.append((r, l, m["feat_uv"][f, 0], m["feat_uv"][f, 1]))
    opt = sorted(lm_index[i] for i in ids if i in lm_index and not m["lm_bad"][lm_index[i]]
                 and m["lm_obs_ptr"][lm_index[i] + 1] - m["lm_obs_ptr"][lm_index[i]] >= min_point)
    return win, opt, obs


def _project(m, k, R, t, p):
    fx, fy, cx, cy = m["kf_intr"][k]
    pc = R @ p + t
    return np.array([fx * pc[0] / pc[2] + cx, fy * pc[1] / pc[2] + cy]), pc[2]


def _numpy_system(m, window, fixed, lam, huber=5.0, max_err=5.0, h=1e-6):
    win, opt, obs = _problem(m, window)
    free = [r for r in range(len(win)) if r >= fixed]
    col_pose = {r: 6 * i for i, r in enumerate(free)}
    Rs = [_quat_to_mat(m["kf_pose"][k, :4]) for k in win]
    ts = [m["kf_pose"][k, 4:].copy() for k in win]
    # landmarks with fewer than 2 valid observations are not variables of this step
    valid = {}
    for (r, l, u, v) in obs:
        proj, z = _project(m, win[r], Rs[r], ts[r], m["lm_pos"][l])
        if z > 1e-6 and np.linalg.norm(np.array([u, v]) - proj) <= max_err:
            valid[l] = valid.get(l, 0) + 1
    var = [l for l in opt if valid.get(l, 0) >= 2]
    slot = {l: i for i, l in enumerate(var)}
    npv = 6 * len(free)
    nv = npv + 3 * len(var)
    H = np.zeros((nv, nv))
    g = np.zeros(nv)
    for (r, l, u, v) in obs:
        k = win[r]
        p = m["lm_pos"][l]
        proj, z = _project(m, k, Rs[r], ts[r], p)
        if z <= 1e-6:
            continue
        e = np.array([u, v]) - proj
        en = np.linalg.norm(e)
        if en > max_err:
            continue
        w = 1.0 if en <= huber else huber / en
        J = np.zeros((2, nv))
        if r in col_pose:
            for d in range(6):
                def pr(s):
                    dv = np.zeros(6)
                    dv[d] = s
                    Rd = _rotvec_mat(dv[3:])
                    return _project(m, k, Rd @ Rs[r], Rd @ ts[r] + dv[:3], p)[0]
                J[:, col_pose[r] + d] = (pr(h) - pr(-h)) / (2 * h)
        if l in slot:
            for d in range(3):
                dp = np.zeros(3)
                dp[d] = h
                J[:, npv + 3 * slot[l] + d] = (_project(m, k, Rs[r], ts[r], p + dp)[0] -
                                                _project(m, k, Rs[r], ts[r], p - dp)[0]) / (2 * h)
        H += w * J.T @ J
        g += w * J.T @ e
    H[np.diag_indices(nv)] += lam * np.diag(H) + 1e-6
    return H, g, npv, free


def test_schur_system_matches_full_normal_equations(oracle):
    m = synth.make_ba_map(11, 5, 80, n_old_kf=0, frac_bad=0.05, frac_outlier=0.05, frac_single=0.1)
    opts = oracle.sba_options(window=5, fixed=1, lam=1e-3)
    S, rhs = oracle.sba_system(m, opts)
    H, g, npv, free = _numpy_system(m, 5, 1, 1e-3)
    Hpp, Hpl, Hll = H[:npv, :npv], H[:npv, npv:], H[npv:, npv:]
    S_np = Hpp - Hpl @ np.linalg.solve(Hll, Hpl.T)
    r_np = g[:npv] - Hpl @ np.linalg.solve(Hll, g[npv:])
    idx = np.concatenate([np.arange(6 * r, 6 * r + 6) for r in free])
    S_o = S[np.ix_(idx, idx)]
    S_o = np.tril(S_o) + np.tril(S_o, -1).T
    assert np.abs(S_o - S_np).max() <= 1e-6 * np.abs(S_np).max()
    assert np.abs(rhs[idx] - r_np).max() <= 1e-6 * np.abs(r_np).max()
    # the reduced solve equals the pose part of the full solve
    dx_full = np.linalg.solve(H, g)[:npv]
    dx_red = np.linalg.solve(S_o, rhs[idx])
    assert np.abs(dx_red - dx_full).max() <= 1e-6 * np.abs(dx_full).max()
    # fixed keyframe rows: identity, zero rhs
    assert np.array_equal(S[:6, :6], np.eye(6)) and not rhs[:6].any()


def test_schur_lm_converges_noise_free(oracle):
    # one fixed keyframe: the similarity gauge absorbs its perturbation, so zero cost is reachable
    m = synth.make_ba_map(5, 6, 400, n_old_kf=0, noise_px=0.0, frac_outlier=0.0, frac_single=0.0,
                          lm_sigma=0.002, rot_deg=0.05, trans_m=0.003)
    st = oracle.sba_optimize(m, oracle.sba_options(window=6, iters=20, fixed=1))
    assert st.status == 0 and st.accepted >= 2
    assert st.final_cost < 1e-6 * st.initial_cost
    costs = [st.cost[i] for i in range(min(st.iterations, 16)) if st.step[i] in (1, 2)]
    assert all(b < a for a, b in zip(costs, costs[1:]))  # accepted steps strictly decrease


def test_schur_lm_reject_and_recover(oracle):
    """A huge initial damping still converges (accept path), a tiny one exercises the
    rejection path on a badly perturbed window without diverging."""
    m = synth.make_ba_map(9, 6, 500, n_old_kf=0, rot_deg=2.0, trans_m=0.05, lm_sigma=0.1)
    st = oracle.sba_optimize(m.copy(), oracle.sba_options(window=6, iters=16, lam=1e3))
    assert st.final_cost < st.initial_cost
    st2 = oracle.sba_optimize(m.copy(), oracle.sba_options(window=6, iters=16, lam=1e-12))
    assert st2.final_cost <= st2.initial_cost
    steps = list(st.step[:min(st.iterations, 16)]) + list(st2.step[:min(st2.iterations, 16)])
    assert steps.count(2) == 2


def test_schur_early_returns(oracle):
    m = synth.make_ba_map(3, 4, 100, n_old_kf=0)
    st = oracle.sba_optimize(m, oracle.sba_options(window=1))
    assert st.status == 1 and st.iterations == 0
    mm = m.copy()
    mm["lm_bad"][:] = 1
    st = oracle.sba_optimize(mm, oracle.sba_options(window=4))
    assert st.status == 1 and st.n_landmarks == 0
