"""PnP RANSAC: CPU checks of the restatement (oracle/ransac_oracle.cpp) that
the GPU path (csrc/ransac.hip) is held to, for cv::solvePnPRansac in Tracking::TrackWithPnP
(tracking.cpp:414-423).

OpenCV is not installed and the reference ships no fixtures for this call, so parity against
OpenCV is unpinned (its cv::RNG stream and EPnP kernel are not reproduced).  The restatement is
pinned here by what the contract promises independently of the hypothesis stream: polynomial roots
against numpy, noise-free P3P recovers the true pose, RANSAC recovers ground truth with outliers,
the reported inlier mask / count are those of the kept model (re-derived in numpy), and the kept
hypothesis and iteration count are those of RANSACPointSetRegistrator::run's sequential loop
(replayed in Python over the per-hypothesis counts)."""
import math

import numpy as np
import pytest

from vxslam import synth


def _project(R, t, obj, intr):
    fx, fy, cx, cy = intr
    pc = obj.astype(np.float64) @ R.T + t
    with np.errstate(divide="ignore", invalid="ignore"):
        uv = np.stack([fx * (pc[:, 0] / pc[:, 2]) + cx, fy * (pc[:, 1] / pc[:, 2]) + cy], -1)
    return pc, uv


def _inliers(R, t, d, thr):
    pc, uv = _project(R, t, d["obj"], d["intr"])
    e = ((uv - d["img"].astype(np.float64)) ** 2).sum(1)
    return (pc[:, 2] > 0) & (e <= thr * thr)


def _update_iters(p, ep, max_iters):
    """RANSACUpdateNumIters (OpenCV calib3d ptsetreg.cpp), modelPoints = 4."""
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, 2.2250738585072014e-308)
    denom = 1.0 - (1.0 - ep) ** 4
    if denom < 2.2250738585072014e-308:
        return 0
    num, denom = math.log(num), math.log(denom)
    return max_iters if denom >= 0 or -num >= max_iters * -denom else int(np.rint(num / denom))


def test_poly_roots_match_numpy(oracle):
    rng = np.random.default_rng(1)
    for _ in range(300):
        d = int(rng.integers(1, 5))
        r = np.sort(rng.uniform(-5, 5, d))
        if d > 1 and np.diff(r).min() < 1e-3:
            continue
        c = np.poly(r)[::-1] * rng.uniform(0.5, 3)  # ascending coefficients
        got = oracle.poly_roots(c)
        assert len(got) == d, (r, got)
        assert np.allclose(got, r, atol=1e-9, rtol=1e-9)
    # no real roots / double root / leading zeros
    assert len(oracle.poly_roots([1.0, 0.0, 1.0])) == 0
    assert len(oracle.poly_roots([1.0, 0.0, 2.0, 0.0, 1.0])) == 0  # (x^2 + 1)^2
    assert np.allclose(oracle.poly_roots([-6.0, 11.0, -6.0, 1.0, 0.0]), [1, 2, 3])


def test_p3p_noise_free_recovers_pose(oracle):
    rng = np.random.default_rng(2)
    d = synth.make_pnp_problem(5, 400, outlier_frac=0.0, noise_px=0.0)
    fx, fy, cx, cy = d["intr"]
    hits = 0
    for k in range(200):
        idx = rng.choice(400, 3, replace=False)
        P = d["obj"][idx].astype(np.float64)
        uv = d["img"][idx].astype(np.float64)
        f = np.stack([(uv[:, 0] - cx) / fx, (uv[:, 1] - cy) / fy, np.ones(3)], -1)
        f /= np.linalg.norm(f, axis=1)[:, None]
        sols = oracle.p3p(P, f)
        err = min((np.abs(R - d["R"]).max() + np.abs(t - d["t"]).max() for R, t in sols), default=np.inf)
        # float32 storage of obj / img is the only error source
        hits += err < 1e-4
        for R, _ in sols:  # every candidate is a rotation
            assert np.abs(R @ R.T - np.eye(3)).max() < 1e-9 and abs(np.linalg.det(R) - 1) < 1e-9
    assert hits >= 198


def test_update_iters_formula(oracle):
    for p, ep, m in [(0.99, 0.5, 100), (0.99, 0.3, 100), (0.999, 0.7, 1000), (0.99, 0.0, 100), (0.99, 1.0, 50),
                     (0.5, 0.9, 4096), (0.99, 0.05, 7)]:
        assert oracle.pnp_update_iters(p, ep, m) == _update_iters(p, ep, m), (p, ep, m)
    assert oracle.pnp_update_iters(0.99, 0.5, 100) == 71  # log(0.01) / log(1 - 0.5^4) = 71.4


@pytest.mark.parametrize("frac", [0.0, 0.3, 0.5])
def test_ransac_recovers_ground_truth(oracle, frac):
    d = synth.make_pnp_problem(10 + int(frac * 10), 1000, outlier_frac=frac)
    r, mask = oracle.pnp_ransac(d["obj"], d["img"], d["intr"], oracle.pnp_options(1000))
    assert r["ok"] == 1
    assert np.abs(r["pose"] - d["pose"]).max() < 5e-3
    assert (mask.astype(bool) & d["outlier"]).sum() <= 1
    assert r["n_inliers"] == mask.sum() >= 0.8 * (~d["outlier"]).sum() * 0.9
    assert r["cost"] <= r["cost0"]
    # rvec / tvec are the same pose as the quaternion
    th = np.linalg.norm(r["rvec"])
    assert abs(th - 2 * math.atan2(np.linalg.norm(r["pose"][:3]), r["pose"][3])) < 1e-12
    assert np.array_equal(r["tvec"], r["pose"][4:])


def test_mask_and_loop_replay(oracle):
    """Inlier mask = the kept hypothesis's inliers; kept index and iteration count = the sequential
    loop (strictly more inliers than max(best, 3), budget shrunk by RANSACUpdateNumIters)."""
    for seed, n, frac, H in [(30, 300, 0.4, 100), (31, 50, 0.2, 100), (32, 600, 0.6, 300), (33, 12, 0.0, 24)]:
        d = synth.make_pnp_problem(seed, n, outlier_frac=frac)
        o = oracle.pnp_options(n, max_iterations=H, seed=seed * 7)
        r, mask = oracle.pnp_ransac(d["obj"], d["img"], d["intr"], o)
        counts = []
        for h in range(H):
            m = oracle.pnp_hypothesis(d["obj"], d["img"], d["intr"], int(o["seed"]), h)
            counts.append(None if m is None else int(_inliers(m[0], m[1], d, 2.0).sum()))
        niters, best, good, h = H, -1, 0, 0
        while h < niters:
            c = counts[h]
            if c is not None and c > max(good, 3):
                best, good = h, c
                niters = _update_iters(0.99, (n - c) / n, niters)
            h += 1
        assert r["best_hypothesis"] == best and r["hypotheses_run"] == h and r["n_inliers"] == good
        assert r["ok"] == (best >= 0)
        if best >= 0:
            R, t = oracle.pnp_hypothesis(d["obj"], d["img"], d["intr"], int(o["seed"]), best)
            assert np.array_equal(mask.astype(bool), _inliers(R, t, d, 2.0))


def test_edges(oracle):
    d = synth.make_pnp_problem(40, 100)
    for n in (0, 1, 3):
        r, mask = oracle.pnp_ransac(d["obj"][:n], d["img"][:n], d["intr"], oracle.pnp_options(n))
        assert r["ok"] == 0 and r["best_hypothesis"] == -1 and mask.sum() == 0
    r, _ = oracle.pnp_ransac(d["obj"], d["img"], d["intr"], oracle.pnp_options(100, max_iterations=0))
    assert r["ok"] == 0 and r["hypotheses_run"] == 0
    # all correspondences wrong: no model keeps more than a handful
    bad = synth.make_pnp_problem(41, 200, outlier_frac=1.0)
    r, mask = oracle.pnp_ransac(bad["obj"], bad["img"], bad["intr"], oracle.pnp_options(200))
    assert r["n_inliers"] == mask.sum() <= 10
    # collinear world points: P3P has no solution, nothing is kept
    line = d["obj"].copy()
    line[:, 1:] = 0.0
    line[:, 0] = np.linspace(-1, 1, 100)
    line[:, 2] = 3.0
    r, _ = oracle.pnp_ransac(line, d["img"], d["intr"], oracle.pnp_options(100))
    assert r["ok"] == 0


def test_batch_equals_single(oracle):
    ps = [synth.make_pnp_problem(50 + k, n, outlier_frac=0.3) for k, n in enumerate([40, 300, 4, 120])]
    offs = np.cumsum([0] + [len(p["obj"]) for p in ps])
    opts = np.stack([oracle.pnp_options(len(p["obj"]), seed=k) for k, p in enumerate(ps)])
    out, mask = oracle.pnp_ransac_batch(offs, np.concatenate([p["obj"] for p in ps]),
                                        np.concatenate([p["img"] for p in ps]), np.stack([p["intr"] for p in ps]),
                                        opts)
    for k, p in enumerate(ps):
        r, m = oracle.pnp_ransac(p["obj"], p["img"], p["intr"], opts[k])
        assert out[k].tobytes() == r.tobytes()
        assert np.array_equal(mask[offs[k]:offs[k + 1]], m)
