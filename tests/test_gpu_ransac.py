"""GPU parity of PnP RANSAC (vx_pnp_ransac / vx_pnp_ransac_batch, csrc/ransac.hip) against the CPU
restatement (oracle/ransac_oracle.cpp, pinned by tests/test_ransac_cpu.py).

Bars: ok, kept hypothesis, hypotheses run, inlier count and inlier mask identical (the hypothesis
stage is the same IEEE + - * / sqrt sequence on both sides); the LM-refined pose within 1e-9
(block-reduction order differs from the CPU's sequential sums)."""
import numpy as np
import pytest

from vxslam import synth

import vxslam

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-9


def _same(rg, mg, rc, mc):
    for k in ("ok", "best_hypothesis", "hypotheses_run", "n_inliers"):
        assert rg[k] == rc[k], (k, rg[k], rc[k])
    assert np.array_equal(mg, mc)
    if rc["ok"]:
        assert np.abs(rg["pose"] - rc["pose"]).max() <= POSE_TOL, (rg["pose"], rc["pose"])
        assert np.abs(rg["rvec"] - rc["rvec"]).max() <= POSE_TOL
        assert abs(rg["cost0"] - rc["cost0"]) <= 1e-9 * max(rc["cost0"], 1.0)
        assert abs(rg["cost"] - rc["cost"]) <= 1e-9 * max(rc["cost"], 1.0)


@pytest.mark.parametrize("n,frac,H", [(4, 0.0, 8), (5, 0.0, 10), (30, 0.2, 60), (300, 0.3, 100),
                                      (2000, 0.3, 100), (2000, 0.6, 100), (1000, 0.5, 1000), (500, 0.0, 1)])
def test_pnp_ransac_parity(ctx, oracle, n, frac, H):
    d = synth.make_pnp_problem(100 + n + int(frac * 10), n, outlier_frac=frac)
    o = vxslam.pnp_options(n, max_iterations=H, seed=n * 31 + H)
    rg, mg = ctx.pnp_ransac(d["obj"], d["img"], d["intr"], o)
    rc, mc = oracle.pnp_ransac(d["obj"], d["img"], d["intr"], o)
    _same(rg, mg, rc, mc)
    if frac <= 0.3 and n >= 300:
        assert rg["ok"] == 1 and np.abs(rg["pose"] - d["pose"]).max() < 5e-3


def test_pnp_ransac_batch_parity(ctx, oracle):
    ps = [synth.make_pnp_problem(200 + k, n, outlier_frac=f)
          for k, (n, f) in enumerate([(400, 0.3), (0, 0.0), (3, 0.0), (50, 0.1), (1200, 0.5), (4, 0.0), (250, 1.0),
                                      (800, 0.2)])]
    offs = np.cumsum([0] + [len(p["obj"]) for p in ps])
    opts = np.stack([vxslam.pnp_options(len(p["obj"]), seed=7 * k + 1) for k, p in enumerate(ps)])
    opts["max_iterations"][5] = 0  # a problem with no budget
    opts["refine_iterations"][3] = 0
    obj = np.concatenate([p["obj"] for p in ps])
    img = np.concatenate([p["img"] for p in ps])
    intr = np.stack([p["intr"] for p in ps])
    intr[3] *= [1.1, 1.1, 1.0, 1.0]
    og, mg = ctx.pnp_ransac_batch(offs, obj, img, intr, opts)
    oc, mc = oracle.pnp_ransac_batch(offs, obj, img, intr, opts)
    for k in range(len(ps)):
        _same(og[k], mg[offs[k]:offs[k + 1]], oc[k], mc[offs[k]:offs[k + 1]])


def test_pnp_ransac_refine_off_and_edges(ctx, oracle):
    d = synth.make_pnp_problem(300, 500, outlier_frac=0.3)
    o = vxslam.pnp_options(500, refine_iterations=0)
    rg, mg = ctx.pnp_ransac(d["obj"], d["img"], d["intr"], o)
    rc, mc = oracle.pnp_ransac(d["obj"], d["img"], d["intr"], o)
    _same(rg, mg, rc, mc)
    assert rg["refine_iterations"] == 0 and rg["cost"] == rg["cost0"]
    # collinear points: no model
    line = d["obj"].copy()
    line[:, 1:] = 0.0
    line[:, 2] = 3.0
    rg, mg = ctx.pnp_ransac(line, d["img"], d["intr"], vxslam.pnp_options(500))
    assert rg["ok"] == 0 and mg.sum() == 0
    for n in (0, 3):
        rg, mg = ctx.pnp_ransac(d["obj"][:n], d["img"][:n], d["intr"], vxslam.pnp_options(n))
        assert rg["ok"] == 0 and rg["hypotheses_run"] == 0
    with pytest.raises(vxslam.VxError):
        ctx.pnp_ransac(d["obj"], d["img"], d["intr"], vxslam.pnp_options(500, max_iterations=5000))


def test_pnp_ransac_repeatable(ctx):
    d = synth.make_pnp_problem(301, 1500, outlier_frac=0.4)
    o = vxslam.pnp_options(1500)
    a = ctx.pnp_ransac(d["obj"], d["img"], d["intr"], o)
    b = ctx.pnp_ransac(d["obj"], d["img"], d["intr"], o)
    assert a[0].tobytes() == b[0].tobytes() and np.array_equal(a[1], b[1])
