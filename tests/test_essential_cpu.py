"""Essential-matrix RANSAC + recoverPose: CPU checks of the restatement
(oracle/essential_oracle.cpp) the GPU path (csrc/essential.hip) is held to, for
cv::findEssentialMat + cv::recoverPose in Tracking::EstimatePoseByEssential (tracking.cpp:503-547).

OpenCV is not installed and the reference ships no fixtures, so parity against OpenCV is unpinned.
The restatement is pinned by what holds independently of the hypothesis stream: the five-point
solutions satisfy the essential-matrix constraints and contain the true E on noise-free data,
RANSAC + recoverPose recover ground truth under outliers, and the kept model / iteration count /
masks re-derived in numpy (sampler, Sampson error, the sequential loop, cheirality) agree."""
import math

import numpy as np
import pytest

from vxslam import synth

M64 = (1 << 64) - 1


def _hat(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def _norm(d):
    fx, fy, cx, cy = d["intr"]
    p1 = d["pts_last"].astype(np.float64)
    p2 = d["pts_curr"].astype(np.float64)
    return (np.stack([(p1[:, 0] - cx) / fx, (p1[:, 1] - cy) / fy], -1),
            np.stack([(p2[:, 0] - cx) / fx, (p2[:, 1] - cy) / fy], -1))


def _mix(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def _sample5(seed, h, n):
    idx = []
    for a in range(64):
        i = ((_mix((seed + h * 64 + a) & M64) >> 32) * n) >> 32
        if i not in idx:
            idx.append(i)
        if len(idx) == 5:
            return idx
    return None


def _sampson(E, x1, x2):
    Ex1 = x1 @ E[:, :2].T + E[:, 2]
    Etx2 = x2 @ E[:2, :] + E[2, :]
    x2tEx1 = x2[:, 0] * Ex1[:, 0] + x2[:, 1] * Ex1[:, 1] + Ex1[:, 2]
    return x2tEx1 ** 2 / (Ex1[:, 0] ** 2 + Ex1[:, 1] ** 2 + Etx2[:, 0] ** 2 + Etx2[:, 1] ** 2)


def _update5(p, ep, max_iters):
    num = max(1.0 - p, 2.2250738585072014e-308)
    denom = 1.0 - (1.0 - ep) ** 5
    if denom < 2.2250738585072014e-308:
        return 0
    num, denom = math.log(num), math.log(denom)
    return max_iters if denom >= 0 or -num >= max_iters * -denom else int(np.rint(num / denom))


def test_five_point_constraints_and_truth(oracle):
    d = synth.make_two_view(1, 300, outlier_frac=0.0, noise_px=0.0)
    x1, x2 = _norm(d)
    Et = _hat(d["t_dir"]) @ d["R"]
    Et /= np.linalg.norm(Et)
    rng = np.random.default_rng(0)
    hits = 0
    for k in range(60):
        idx = rng.choice(300, 5, replace=False)
        Es = oracle.five_point(x1[idx], x2[idx])
        assert 1 <= len(Es) <= 10
        for E in Es:
            assert abs(np.linalg.norm(E) - 1) < 1e-12
            assert abs(np.linalg.det(E)) < 1e-8
            assert np.abs(2 * E @ E.T @ E - np.trace(E @ E.T) * E).max() < 1e-8
            h1 = np.c_[x1[idx], np.ones(5)]
            h2 = np.c_[x2[idx], np.ones(5)]
            assert np.abs(np.einsum("ij,jk,ik->i", h2, E, h1)).max() < 1e-9
        hits += min(min(np.abs(E - Et).max(), np.abs(E + Et).max()) for E in Es) < 1e-4
    assert hits == 60


@pytest.mark.parametrize("frac", [0.0, 0.3, 0.5])
def test_ransac_recovers_ground_truth(oracle, frac):
    d = synth.make_two_view(10 + int(10 * frac), 1000, outlier_frac=frac)
    r, mask = oracle.essential_ransac(d["pts_last"], d["pts_curr"], d["intr"], oracle.essential_options())
    assert r["ok"] == 1
    R = r["R"].reshape(3, 3)
    assert np.abs(R @ R.T - np.eye(3)).max() < 1e-12 and abs(np.linalg.det(R) - 1) < 1e-12
    assert abs(np.linalg.norm(r["t"]) - 1) < 1e-12
    assert np.abs(R - d["R"]).max() < 0.02 and np.abs(r["t"] - d["t_dir"]).max() < 0.08
    # E = [t]x R up to scale and sign
    E = r["E"].reshape(3, 3)
    Ert = _hat(r["t"]) @ R
    Ert /= np.linalg.norm(Ert)
    assert min(np.abs(E - Ert).max(), np.abs(E + Ert).max()) < 1e-6
    assert (mask.astype(bool) & d["outlier"]).sum() <= 3
    assert r["n_inliers"] == mask.sum() <= r["n_ransac_inliers"]
    assert r["n_inliers"] >= 0.85 * r["n_ransac_inliers"]  # low-parallax points may triangulate behind


def test_loop_replay_and_masks(oracle):
    """Kept (hypothesis, model), hypotheses run and the RANSAC count re-derived in numpy; the output
    mask = RANSAC inliers of the kept E that triangulate in front of both views."""
    for seed, n, frac, H in [(30, 400, 0.4, 200), (31, 60, 0.2, 100), (32, 300, 0.6, 300)]:
        d = synth.make_two_view(seed, n, outlier_frac=frac)
        o = oracle.essential_options(max_iterations=H, seed=seed * 3)
        r, mask = oracle.essential_ransac(d["pts_last"], d["pts_curr"], d["intr"], o)
        x1, x2 = _norm(d)
        thr = 1.0 / ((d["intr"][0] + d["intr"][1]) * 0.5)
        niters, best, good, h = H, None, 0, 0
        models = {}
        while h < niters:
            idx = _sample5(int(o["seed"]), h, n)
            Es = oracle.five_point(x1[idx], x2[idx])
            for m, E in enumerate(Es):
                c = int((_sampson(E, x1, x2) <= thr * thr).sum())
                if c > max(good, 4):
                    best, good = (h, m), c
                    models[(h, m)] = E
                    niters = _update5(0.999, (n - c) / n, niters)
            h += 1
        assert (r["best_hypothesis"], r["best_model"]) == best
        assert r["hypotheses_run"] == h and r["n_ransac_inliers"] == good
        E = models[best]
        assert np.array_equal(r["E"].reshape(3, 3), E)
        ransac = _sampson(E, x1, x2) <= thr * thr
        assert np.array_equal(mask.astype(bool), mask.astype(bool) & ransac)
        # cheirality of the kept pose, by linear triangulation in numpy
        R, t = r["R"].reshape(3, 3), r["t"]
        P1 = np.c_[R, t]
        front = np.zeros(n, bool)
        for i in np.nonzero(ransac)[0]:
            A = np.stack([[-1, 0, x1[i, 0], 0], [0, -1, x1[i, 1], 0], x2[i, 0] * P1[2] - P1[0],
                          x2[i, 1] * P1[2] - P1[1]])
            X = np.linalg.svd(A)[2][3]
            if X[2] * X[3] > 0:
                p = X[:3] / X[3]
                z2 = (R @ p + t)[2]
                front[i] = p[2] < 50 and 0 < z2 < 50
        assert (mask.astype(bool) != front).sum() <= 2


def test_edges(oracle):
    d = synth.make_two_view(40, 100)
    for n in (0, 4):
        r, mask = oracle.essential_ransac(d["pts_last"][:n], d["pts_curr"][:n], d["intr"], oracle.essential_options())
        assert r["ok"] == 0 and r["hypotheses_run"] == 0 and mask.sum() == 0
        assert np.array_equal(r["R"].reshape(3, 3), np.eye(3))
    r, _ = oracle.essential_ransac(d["pts_last"], d["pts_curr"], d["intr"], oracle.essential_options(max_iterations=0))
    assert r["ok"] == 0
    # identical points in both views (no baseline) and all-outlier matches do not crash
    r, _ = oracle.essential_ransac(d["pts_last"], d["pts_last"], d["intr"], oracle.essential_options(max_iterations=50))
    bad = synth.make_two_view(41, 200, outlier_frac=1.0)
    r, mask = oracle.essential_ransac(bad["pts_last"], bad["pts_curr"], bad["intr"],
                                      oracle.essential_options(max_iterations=100))
    assert r["n_inliers"] == mask.sum()


def test_batch_equals_single(oracle):
    ps = [synth.make_two_view(50 + k, n, outlier_frac=0.3) for k, n in enumerate([40, 300, 5, 120])]
    offs = np.cumsum([0] + [len(p["pts_last"]) for p in ps])
    opts = np.stack([oracle.essential_options(max_iterations=200, seed=k) for k in range(len(ps))])
    out, mask = oracle.essential_ransac_batch(offs, np.concatenate([p["pts_last"] for p in ps]),
                                              np.concatenate([p["pts_curr"] for p in ps]),
                                              np.stack([p["intr"] for p in ps]), opts)
    for k, p in enumerate(ps):
        r, m = oracle.essential_ransac(p["pts_last"], p["pts_curr"], p["intr"], opts[k])
        assert out[k].tobytes() == r.tobytes()
        assert np.array_equal(mask[offs[k]:offs[k + 1]], m)
