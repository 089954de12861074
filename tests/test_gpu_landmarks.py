"""GPU parity of keyframe-insertion landmark creation (vx_depth_landmarks, vx_triangulate)
against the CPU restatement (oracle/landmark_oracle.cpp, pinned by tests/test_landmarks_cpu.py).

Bars: the created set and its numbering identical (no gate flips); depth landmarks bit-exact (same
IEEE operations in the same order); triangulated points within 1e-9 relative (the SVD's rotation
sequence rounds differently)."""
import numpy as np
import pytest

from vxslam import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", ["u16", "f32", "f64"])
def test_depth_landmarks_bit_exact(ctx, oracle, dt):
    d = synth.make_keyframe_pair(21, 2000, depth_type=dt)
    uv = d["uv2"].copy()
    uv[:16] = [[-0.7, 12.0]] * 16
    uv[16:24] = [[639.6, 479.4]] * 8
    ig, pg = ctx.depth_landmarks(uv, d["has2"], d["depth"], d["intr"], d["pose2"])
    ic, pc = oracle.depth_landmarks(uv, d["has2"], d["depth"], d["intr"], d["pose2"])
    assert np.array_equal(ig, ic)
    assert np.array_equal(pg, pc)


def test_depth_landmarks_edges(ctx, oracle):
    d = synth.make_keyframe_pair(22, 300)
    ig, pg = ctx.depth_landmarks(d["uv2"], d["has2"], None, d["intr"], d["pose2"])  # no depth image
    assert (ig == -1).all() and len(pg) == 0
    ig, pg = ctx.depth_landmarks(d["uv2"], np.ones(300, np.uint8), d["depth"], d["intr"], d["pose2"])
    assert (ig == -1).all() and len(pg) == 0
    ig, pg = ctx.depth_landmarks(d["uv2"][:0], d["has2"][:0], d["depth"], d["intr"], d["pose2"])
    assert len(ig) == 0
    # a depth image with padded rows (row stride > cols * 2)
    padded = np.zeros((480, 700), np.uint16)
    padded[:, :640] = d["depth"]
    view = padded[:, :640]
    ig, pg = ctx.depth_landmarks(d["uv2"], d["has2"], view, d["intr"], d["pose2"])
    ic, pc = oracle.depth_landmarks(d["uv2"], d["has2"], d["depth"], d["intr"], d["pose2"])
    assert np.array_equal(ig, ic) and np.array_equal(pg, pc)


@pytest.mark.parametrize("seed,n,kw", [(31, 2000, {}), (32, 4000, dict(width=1280, height=960, intr=(1041.8, 1042.0, 650.2, 499.4))),
                                       (33, 1500, dict(frac_dup_train=0.25, frac_has=0.3)),
                                       (34, 1000, dict(baseline_m=0.3, yaw_deg=8.0))])
def test_triangulate_parity(ctx, oracle, seed, n, kw):
    d = synth.make_keyframe_pair(seed, n, **kw)
    for ang, err in [(1.0, 5.0), (0.5, 2.0)]:
        ig, pg = ctx.triangulate(d, ang, err)
        ic, pc = oracle.triangulate(d, ang, err)
        assert np.array_equal(ig, ic), (np.nonzero(ig != ic)[0][:10])
        assert len(pc) > 0
        assert np.abs(pg - pc).max() <= 1e-9 * np.abs(pc).max()


def test_triangulate_rejects_bad_matches(ctx):
    import vxslam

    d = synth.make_keyframe_pair(35, 200)
    dd = dict(d)
    m = d["matches"].copy()
    m["query_idx"][1] = m["query_idx"][0]
    dd["matches"] = m
    with pytest.raises(vxslam.VxError):
        ctx.triangulate(dd)
    m = d["matches"].copy()
    m["train_idx"][0] = 10_000
    dd["matches"] = m
    with pytest.raises(vxslam.VxError):
        ctx.triangulate(dd)
    dd["matches"] = d["matches"][:0]
    ig, pg = ctx.triangulate(dd)
    assert len(ig) == 0 and len(pg) == 0
