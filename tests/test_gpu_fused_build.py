"""The fused LocalBA layout built on the device (ba_fused_build.hip) against the host packing
(ba.hip build_fused, the specification; plans built with VX_PLAN_HOST_BUILD keep it): the index
tables k_ba_iter reads must be equal byte for byte, and so the runs bitwise.  Windows: C2 / C3, the
1024-thread packing (C4), windows beyond 64 keyframes (the 64-entry keyframe cap binds; 2 and 7
words per keyframe set), a narrow packing cap (many workgroups), a keyframe no optimised landmark
touches (owned by workgroup 0, empty entries), and shard plans."""
import numpy as np
import pytest

import vxslam
from vxslam import synth

pytestmark = pytest.mark.gpu


def _tables(ctx, m, opts, **kw):
    out = []
    for hb in (True, False):
        p = ctx.ba_plan(m, opts, host_build=hb, **kw)
        lay = p.layout()
        out.append((lay, p.fused_tables() if lay["fused"] else b"", p))
    return out


def _check_equal(ctx, m, opts, run=True, **kw):
    (lh, th, ph), (ld, td, pd) = _tables(ctx, m, opts, **kw)
    assert lh == ld
    assert lh["fused"] == 1
    assert len(th) == len(td) and th == td
    if run:
        mh, md = m.copy(), m.copy()
        ph.run_async()
        sh = ph.fetch(mh)
        pd.run_async()
        sd = pd.fetch(md)
        assert np.array_equal(mh["kf_pose"], md["kf_pose"]) and np.array_equal(mh["lm_pos"], md["lm_pos"])
        assert sh.iterations == sd.iterations
    ph.close(), pd.close()
    return ld


@pytest.mark.parametrize("cfg", ["C2", "C3", "C4"])
def test_device_layout_equals_host_packing(ctx, cfg, slot_sums):
    nk, nl, _ = synth.ba_config(cfg)
    m = synth.make_ba_map(0x5EED0003, nk, nl)
    lay = _check_equal(ctx, m, vxslam.default_ba_options(window=nk))
    if cfg == "C4":
        assert lay["threads"] == 1024


@pytest.mark.parametrize("nk,nl,streams", [(100, 30000, 4), (200, 50000, 8), (440, 60000, 8)])
def test_device_layout_wide_windows(ctx, nk, nl, streams, slot_sums):
    m = synth.make_ba_map(0x5EED0100 + nk, nk, nl, n_streams=streams, n_old_kf=2 * streams)
    _check_equal(ctx, m, vxslam.default_ba_options(window=nk), run=nk <= 200)


def test_device_layout_narrow_cap(ctx, monkeypatch, slot_sums):
    monkeypatch.setenv("VX_BA_FUSED_CAP", "96")
    m = synth.make_ba_map(0x5EED0004, 50, 20000)
    lay = _check_equal(ctx, m, vxslam.default_ba_options(window=50))
    assert lay["workgroups"] > 500


def test_device_layout_untouched_keyframe(ctx, slot_sums):
    """A window keyframe without features (no pose- or landmark-stage observation): no workgroup
    touches it, so workgroup 0 owns it with an empty entry."""
    m = synth.make_ba_map(0x5EED0005, 12, 3000)
    new_id = int(m["kf_id"].max()) + 1
    m["kf_id"] = np.append(m["kf_id"], np.uint64(new_id))
    m["kf_pose"] = np.ascontiguousarray(np.concatenate([m["kf_pose"], m["kf_pose"][-1:]]))
    m["kf_intr"] = np.ascontiguousarray(np.concatenate([m["kf_intr"], m["kf_intr"][-1:]]))
    m["kf_has_cam"] = np.append(m["kf_has_cam"], m["kf_has_cam"][-1])
    m["kf_feat_ptr"] = np.append(m["kf_feat_ptr"], m["kf_feat_ptr"][-1])
    m["ref_kf_id"] = new_id
    opts = vxslam.default_ba_options(window=13)
    (lh, th, ph), (ld, td, pd) = _tables(ctx, m, opts)
    assert lh == ld and th == td and lh["fused"] == 1
    ph.close(), pd.close()


@pytest.mark.parametrize("n", [2, 4])
def test_device_layout_shard_plans(ctx, n):
    nk, nl = 50 * n, 20000 * n
    m = synth.make_ba_map(0x5EED0003, nk, nl, n_streams=n, n_old_kf=2 * n)
    opts = vxslam.default_ba_options(window=nk)
    for r in range(n):
        _check_equal(ctx, m, opts, run=False, shard_rank=r, shard_count=n)
