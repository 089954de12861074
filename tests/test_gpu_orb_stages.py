"""Per-stage ORB parity: every intermediate list of the device
extraction against the CPU restatement, not only the final keypoints and descriptor bits.

Read through the vx_orb_set_debug / vx_orb_debug_read test hooks after a single-frame extraction:
  * the gray / INTER_LINEAR_EXACT pyramid level and its 7x7 GaussianBlur, byte for byte
    (the blur was otherwise checked only through descriptor bits);
  * the FAST-9/16 + strict 3x3 NMS list (x, y, score) over the whole FAST domain [3, W-3) x
    [3, H-3), i.e. before runByImageBorder (VX_ORB_DEBUG_FAST_NO_BORDER: k_fast with the border at
    3) — the unretained candidates are checked directly;
  * after the border: the raster candidate list with FAST score and Harris response (bitwise);
  * retainBest(2q)'s output order (indices into that list) and retainBest(q)'s output records —
    the reference's libstdc++ permutation.
Over 100 seeded frames at the C2 / C3 / C4 sizes (BASELINE.json configs), plus the committed
per-stage fixtures (tests/golden/orb_stages_golden.npz).
"""
import hashlib
import os
import sys

import numpy as np
import pytest

from vxslam import synth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402


def _xy(rec):
    return (rec["xy"] & 0xFFFF).astype(np.int64), (rec["xy"] >> 16).astype(np.int64)


def _stages(ctx, img, n, levels=8):
    """Device stage lists in the oracle's layout (orb_stages) + the pyramid / blur levels."""
    import vxslam

    p = vxslam.default_orb_params(n_features=n)
    ctx.set_debug(vxslam.DEBUG_FAST_NO_BORDER | vxslam.DEBUG_STAGES)
    ctx.orb_extract(img, p)
    fast = []
    for l in range(levels):
        r = ctx.debug_read(l, 2)
        x, y = _xy(r)
        fast.append(np.stack([x, y, r["score"]], 1).astype(np.int32) if len(r) else np.zeros((0, 3), np.int32))
    ctx.set_debug(vxslam.DEBUG_STAGES)
    kd = ctx.orb_extract(img, p)
    out = []
    for l in range(levels):
        c = ctx.debug_read(l, 2)
        x, y = _xy(c)
        cand = np.stack([x.astype(np.float32), y.astype(np.float32), c["score"].astype(np.float32), c["harris"]], 1)
        fin_rec = ctx.debug_read(l, 4)
        out.append(dict(fast=fast[l], cand=cand.reshape(-1, 4), keep1=ctx.debug_read(l, 3), fin_rec=fin_rec,
                        pyr=ctx.debug_read(l, 0), blur=ctx.debug_read(l, 1)))
    ctx.set_debug(0)
    return out, kd


def _check(st, ref, pyr_ref=None, blur_ref=None):
    for l, (g, c) in enumerate(zip(st, ref)):
        assert np.array_equal(g["fast"], c["fast"]), ("FAST list", l, len(g["fast"]), len(c["fast"]))
        assert g["cand"].view(np.uint32).tobytes() == c["cand"].view(np.uint32).tobytes(), ("candidates", l)
        assert np.array_equal(g["keep1"], c["keep1"]), ("retainBest(2q) order", l)
        fr = g["fin_rec"]
        fx, fy = _xy(fr)
        cf = c["cand"][c["fin"]]
        assert len(fr) == len(cf), ("retainBest(q) size", l)
        assert np.array_equal(fx, cf[:, 0].astype(np.int64)) and np.array_equal(fy, cf[:, 1].astype(np.int64)), l
        assert np.array_equal(fr["harris"].view(np.uint32), cf[:, 3].view(np.uint32)), ("retainBest(q) order", l)
        if pyr_ref is not None:
            assert np.array_equal(g["pyr"], pyr_ref[l].ravel()), ("pyramid", l)
            assert np.array_equal(g["blur"], blur_ref[l].ravel()), ("blur", l)


def test_orb_stages_golden(ctx):
    g = np.load(os.path.join(HERE, "golden", "orb_stages_golden.npz"))
    for name, seed, h, w, ch, n in G.STAGE_CASES:
        img = G.orb_input(seed, h, w, ch)
        st, (kg, dg) = _stages(ctx, img, n)
        ref = [dict(fast=g[f"{name}_L{l}_fast"], cand=g[f"{name}_L{l}_cand"], keep1=g[f"{name}_L{l}_keep1"],
                    fin=g[f"{name}_L{l}_fin"]) for l in range(8)]
        _check(st, ref)
        for l in range(8):
            assert hashlib.sha256(st[l]["pyr"].tobytes()).hexdigest() == bytes(g[f"{name}_L{l}_pyr_sha"]).decode(), l
            assert hashlib.sha256(st[l]["blur"].tobytes()).hexdigest() == bytes(g[f"{name}_L{l}_blur_sha"]).decode(), l
        assert np.array_equal(kg, g[f"{name}_kp"]) and np.array_equal(dg, g[f"{name}_desc"])


# 100 seeded frames: C2 (640x480, 1000 features), C3 (640x480, 2000), C4 (1280x960, 4000)
SWEEP = [(480, 640, 1000, s) for s in range(40)] + [(480, 640, 2000, s) for s in range(40, 80)] + \
        [(960, 1280, 4000, s) for s in range(80, 100)]


@pytest.mark.parametrize("chunk", range(5))
def test_orb_stages_sweep(ctx, oracle, chunk):
    for h, w, n, s in SWEEP[chunk * 20:(chunk + 1) * 20]:
        img = synth.make_frames(0x57A6E000 + s, 1, h, w)[0]
        st, kd = _stages(ctx, img, n)
        pyr = oracle.pyramid(img)
        blur = [oracle.blur_level(pl) for pl in pyr] if s % 10 == 0 else None
        _check(st, oracle.orb_stages(img, n), pyr if blur else None, blur)
        kc, dc = oracle.orb_extract(img, n)
        assert np.array_equal(kd[0], kc) and np.array_equal(kd[1], dc), s


def test_debug_hook_guards(ctx):
    import vxslam

    c = vxslam.Context(0)
    try:
        with pytest.raises(vxslam.VxError):
            c.debug_read(0, 0)  # nothing extracted yet
        c.orb_extract(synth.make_frames(3, 1, 120, 160)[0], vxslam.default_orb_params(n_features=200))
        assert len(c.debug_read(0, 0)) == 120 * 160
        with pytest.raises(vxslam.VxError):
            c.debug_read(0, 3)  # selection stages need the debug flag
        with pytest.raises(vxslam.VxError):
            c.set_debug(8)
        # the stage buffers are shared with the other slots and the batches: after a batch (or an
        # extraction into another slot) they no longer hold slot 0's frame, so the hook refuses
        fr = synth.make_frames(4, 2, 120, 160)
        c.orb_extract_batch(np.stack(fr), vxslam.default_orb_params(n_features=200))
        with pytest.raises(vxslam.VxError):
            c.debug_read(0, 0)
        c.orb_extract(fr[0], vxslam.default_orb_params(n_features=200))
        assert len(c.debug_read(0, 0)) == 120 * 160
    finally:
        c.close()
