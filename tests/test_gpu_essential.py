"""GPU parity of the essential-matrix RANSAC + recoverPose (vx_essential_ransac / _batch,
csrc/essential.hip) against the CPU restatement (oracle/essential_oracle.cpp, pinned by
tests/test_essential_cpu.py).

Bar: bit-identical — every decision and every number (E, R, t, counts, both masks) comes from the same
IEEE + - * / sqrt sequence on both sides."""
import numpy as np
import pytest

import vxslam
from vxslam import synth

pytestmark = pytest.mark.gpu


def _same(rg, mg, rc, mc):
    assert rg.tobytes() == rc.tobytes(), (rg, rc)
    assert np.array_equal(mg, mc)


@pytest.mark.parametrize("n,frac,H", [(5, 0.0, 10), (6, 0.0, 20), (50, 0.2, 100), (500, 0.3, 1000),
                                      (2000, 0.3, 1000), (1000, 0.5, 1000), (300, 0.6, 2000), (400, 0.0, 1)])
def test_essential_parity(ctx, oracle, n, frac, H):
    d = synth.make_two_view(500 + n + int(frac * 10), n, outlier_frac=frac)
    o = vxslam.essential_options(max_iterations=H, seed=n * 7 + H)
    rg, mg = ctx.essential_ransac(d["pts_last"], d["pts_curr"], d["intr"], o)
    rc, mc = oracle.essential_ransac(d["pts_last"], d["pts_curr"], d["intr"], o)
    _same(rg, mg, rc, mc)
    if frac <= 0.3 and n >= 500:
        assert rg["ok"] == 1 and np.abs(rg["R"].reshape(3, 3) - d["R"]).max() < 0.02


def test_essential_batch_parity(ctx, oracle):
    ps = [synth.make_two_view(600 + k, n, outlier_frac=f)
          for k, (n, f) in enumerate([(400, 0.3), (0, 0.0), (4, 0.0), (60, 0.1), (1200, 0.5), (5, 0.0), (250, 1.0),
                                      (800, 0.2)])]
    offs = np.cumsum([0] + [len(p["pts_last"]) for p in ps])
    opts = np.stack([vxslam.essential_options(max_iterations=300, seed=11 * k + 2) for k in range(len(ps))])
    opts["max_iterations"][5] = 0
    opts["threshold"][3] = 2.0
    intr = np.stack([p["intr"] for p in ps])
    intr[7] *= [1.05, 1.05, 1.0, 1.0]
    args = (offs, np.concatenate([p["pts_last"] for p in ps]), np.concatenate([p["pts_curr"] for p in ps]), intr,
            opts)
    og, mg = ctx.essential_ransac_batch(*args)
    oc, mc = oracle.essential_ransac_batch(*args)
    for k in range(len(ps)):
        _same(og[k], mg[offs[k]:offs[k + 1]], oc[k], mc[offs[k]:offs[k + 1]])


def test_essential_edges(ctx, oracle):
    d = synth.make_two_view(700, 300, outlier_frac=0.2)
    # no baseline: identical points in both views
    o = vxslam.essential_options(max_iterations=100)
    rg, mg = ctx.essential_ransac(d["pts_last"], d["pts_last"], d["intr"], o)
    rc, mc = oracle.essential_ransac(d["pts_last"], d["pts_last"], d["intr"], o)
    _same(rg, mg, rc, mc)
    with pytest.raises(vxslam.VxError):
        ctx.essential_ransac(d["pts_last"], d["pts_curr"], d["intr"], vxslam.essential_options(max_iterations=5000))
    rg, _ = ctx.essential_ransac(d["pts_last"][:0], d["pts_curr"][:0], d["intr"], o)
    assert rg["ok"] == 0 and rg["hypotheses_run"] == 0
