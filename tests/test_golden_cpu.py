"""The CPU restatement reproduces the committed golden vectors (tests/golden/make_golden.py).

These fixtures were produced by the oracle from seeded synthetic inputs; the tests guard the
oracle (and the generator) against drift.  They are the same fixtures the GPU tests check.
"""
import hashlib
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def orb_golden():
    return np.load(os.path.join(HERE, "golden", "orb_golden.npz"))


@pytest.mark.parametrize("case", G.ORB_CASES, ids=[c[0] for c in G.ORB_CASES])
def test_orb_golden(oracle, orb_golden, case):
    name, seed, h, w, ch, n = case
    img = G.orb_input(seed, h, w, ch)
    assert bytes(orb_golden[f"orb_{name}_sha"]).decode() == _sha(img), "generator drifted"
    kps, desc = oracle.orb_extract(img, n, order=oracle.ORDER_STL)
    assert np.array_equal(kps, orb_golden[f"orb_{name}_kp"])
    assert np.array_equal(desc, orb_golden[f"orb_{name}_desc"])
    kr, dr = oracle.orb_extract(img, n, order=oracle.ORDER_RASTER)
    assert np.array_equal(kr, orb_golden[f"orb_{name}_kp_raster"])
    assert np.array_equal(dr, orb_golden[f"orb_{name}_desc_raster"])


def test_match_golden(oracle):
    g = np.load(os.path.join(HERE, "golden", "match_golden.npz"))
    q, t = G.match_input(77, 512)
    assert np.array_equal(q, g["q"]) and np.array_equal(t, g["t"])
    idx, dist = oracle.knn2(q, t)
    assert np.array_equal(idx, g["idx"]) and np.array_equal(dist, g["dist"])
    assert np.array_equal(oracle.match(q, t), g["matches"])


@pytest.mark.parametrize("case", G.BA_CASES, ids=[c[0] for c in G.BA_CASES])
def test_ba_golden(oracle, case):
    from vxslam import synth

    g = np.load(os.path.join(HERE, "golden", "ba_golden.npz"))
    name, seed, nk, nl, nold, hub, merr, iters = case
    mp = synth.make_ba_map(seed, nk, nl, n_old_kf=nold)
    assert bytes(g[f"ba_{name}_sha"]).decode() == _sha(np.concatenate([mp["kf_pose"].ravel(), mp["lm_pos"].ravel()]))
    st = oracle.ba_optimize(mp, oracle.ba_options(window=nk, iters=iters, huber=hub, max_err=merr))
    assert np.array_equal(mp["kf_pose"], g[f"ba_{name}_pose"])
    assert np.array_equal(mp["lm_pos"], g[f"ba_{name}_lm"])
    assert [st.iterations, st.n_window_kf, st.n_landmarks, st.status] == g[f"ba_{name}_stats"].tolist()


@pytest.mark.parametrize("case", G.STAGE_CASES, ids=[c[0] for c in G.STAGE_CASES])
def test_orb_stage_golden(oracle, case):
    """Per-stage fixtures: the restatement reproduces every level's FAST list,
    candidate list, both retainBest orders and the pyramid / blur hashes, and the final keypoints
    are the candidates named by `fin`, in that order, level by level."""
    name, seed, h, w, ch, n = case
    g = np.load(os.path.join(HERE, "golden", "orb_stages_golden.npz"))
    img = G.orb_input(seed, h, w, ch)
    assert bytes(g[f"{name}_sha"]).decode() == _sha(img), "generator drifted"
    got = G.orb_stage_arrays(img, n)
    for k, v in got.items():
        assert np.array_equal(v, g[f"{name}_{k}"]), k
    kp = got["kp"]
    _, _, scales = oracle.level_sizes(w, h)
    for l in range(8):
        lv = kp[kp["octave"] == l]
        c = got[f"L{l}_cand"][got[f"L{l}_fin"]]
        assert np.array_equal(lv["x"], (c[:, 0] * scales[l]).astype(np.float32))
        assert np.array_equal(lv["y"], (c[:, 1] * scales[l]).astype(np.float32))
        assert np.array_equal(lv["response"], c[:, 3])
        # retainBest keeps {response >= k-th largest}: fin is a subset of keep1, keep1 of cand
        assert set(got[f"L{l}_fin"]) <= set(got[f"L{l}_keep1"])
        assert len(set(got[f"L{l}_keep1"])) == len(got[f"L{l}_keep1"])
