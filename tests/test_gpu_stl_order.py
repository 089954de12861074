"""The reference's keypoint order on the device (k_select_stl, csrc/orb.hip).

ORBExtractor::Extract numbers Frame::Features() in the order cv::ORB leaves its keypoints
(core/feature/orb_extractor.cpp:13-24): per level, KeyPointsFilter::retainBest by FAST score and
then by Harris response, each std::nth_element + std::partition — under libstdc++ a specific
permutation.  Every downstream consumer that works by feature or
match index (solvePnPRansac's sampling, triangulation's skip rule, landmark_id_ numbering) sees
that order, so the GPU reproduces it bit for bit (VX_ORDER_STL, the default); VX_ORDER_RASTER is
the opt-in canonical order of the same set.

Bars: the selection primitive (vx_test_retain_best) returns exactly the kept indices, in order, of
the real std::nth_element / std::partition (oracle.retain_best_keys) — random, tie-heavy, sorted
and McIlroy-adversarial keys (the latter reach libstdc++'s heap-select fallback), both element
widths, LDS and global storage; every ORB output (keypoints, descriptors) bitwise equal to the
oracle in ORDER_STL, single frames and batches of 1..64.
"""
import os
import sys

import numpy as np
import pytest

from vxslam import synth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402

LDS_BYTES = 160 * 1024 - 256 - 65920  # kStlLds - kRgBytes: the arrays after the engine scratch


def _fits_lds(n, wide):
    return (8 if wide else 4) * (n + 2 * (n // 2 + 1)) <= LDS_BYTES


def _eq(a, b):
    (kg, dg), (kc, dc) = a, b
    assert len(kg) == len(kc), (len(kg), len(kc))
    for f in ("octave", "x", "y", "response", "angle"):
        bad = np.nonzero(kg[f] != kc[f])[0]
        assert bad.size == 0, (f, bad[:5])
    assert np.array_equal(dg, dc)


# ---------------------------------------------------------------------------- the primitive
@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("use_lds", [True, False])
def test_retain_best_random(ctx, oracle, wide, use_lds):
    rng = np.random.default_rng(17 + 2 * wide + use_lds)
    cases = [(1, 1), (2, 1), (3, 2), (4, 1), (5, 3), (17, 8), (64, 63), (65, 2), (100, 50), (1024, 300),
             (1025, 512), (1763, 868), (3000, 1500), (5000, 100), (6000, 5999)]
    if not use_lds:
        cases += [(20000, 9000), (40000, 1)]
    for n, npts in cases:
        if use_lds and not _fits_lds(n, wide):
            continue
        for hi in (2, 8, 90, 256) if not wide else (3, 1000, 1 << 32):
            keys = rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32)
            if hi == 90:
                keys += 20  # FAST scores start above the threshold
            got = ctx.test_retain_best(keys, npts, wide, use_lds)
            ref = oracle.retain_best_keys(keys, npts)
            assert np.array_equal(got, ref), (n, npts, hi)


@pytest.mark.parametrize("wide", [False, True])
def test_retain_best_ordered_and_equal_keys(ctx, oracle, wide):
    for n in (10, 999, 2500):
        for keys in (np.arange(n) % 256, (np.arange(n) % 256)[::-1], np.full(n, 77), np.arange(n) // 7 % 256):
            keys = np.ascontiguousarray(keys, np.uint32)
            for npts in (1, n // 3, n // 2, n - 1):
                if npts < 1:
                    continue
                for use_lds in (True, False):
                    got = ctx.test_retain_best(keys, npts, wide, use_lds)
                    assert np.array_equal(got, oracle.retain_best_keys(keys, npts)), (n, npts, use_lds)


def test_retain_best_adversarial_heap_select(ctx, oracle):
    """McIlroy's antiqsort against std::nth_element: inputs that exhaust introselect's depth limit,
    so libstdc++ finishes with __heap_select (tests/cpp/stl_select_model.cpp confirms it is reached)."""
    for n in (16, 64, 257, 1000, 1763, 4096, 6781):
        for npts in (1, 2, n // 3, n // 2, n - 1):
            keys = oracle.antiqsort(n, npts - 1)
            ref = oracle.retain_best_keys(keys, npts)
            for use_lds in (True, False):
                if use_lds and not _fits_lds(n, True):
                    continue
                assert np.array_equal(ctx.test_retain_best(keys, npts, True, use_lds), ref), (n, npts, use_lds)
            if keys.max() <= 255:
                assert np.array_equal(ctx.test_retain_best(keys, npts, False, True), ref), (n, npts)


# ---------------------------------------------------------------------------- ORB in the reference's order
@pytest.mark.parametrize("case", G.ORB_CASES, ids=[c[0] for c in G.ORB_CASES])
def test_orb_order_golden_and_raster_opt_in(oracle, case):
    """Golden fixtures (oracle, ORDER_STL) on a fresh context; then VX_ORDER_RASTER on the same
    context (the golden raster variant), then back to STL (captured graphs must be dropped)."""
    import torch

    import vxslam

    name, seed, h, w, ch, n = case
    g = np.load(os.path.join(HERE, "golden", "orb_golden.npz"))
    img = G.orb_input(seed, h, w, ch)
    p = vxslam.default_orb_params(n_features=n)
    c = vxslam.Context(0)
    try:
        assert c.order == vxslam.ORDER_STL
        _eq(c.orb_extract(img, p), (g[f"orb_{name}_kp"], g[f"orb_{name}_desc"]))
        d = torch.from_numpy(img).to("cuda:0")
        for order, key in ((vxslam.ORDER_RASTER, "_raster"), (vxslam.ORDER_STL, "")):
            c.set_order(order)
            for _ in range(3):  # eager, capture, replay
                c.orb_extract_async(d.data_ptr(), w, h, ch, d.stride(0), 1, p)
                _eq(c.orb_fetch(1), (g[f"orb_{name}_kp{key}"], g[f"orb_{name}_desc{key}"]))
            _eq(c.orb_extract(img, p), (g[f"orb_{name}_kp{key}"], g[f"orb_{name}_desc{key}"]))
        with pytest.raises(vxslam.VxError):
            c.set_order(7)
    finally:
        c.close()


@pytest.mark.parametrize("seed,h,w,n", [(51, 480, 640, 1000), (52, 480, 640, 2000), (53, 960, 1280, 4000),
                                        (54, 64, 80, 100), (55, 333, 517, 800)])
def test_orb_stl_random_frames(ctx, oracle, seed, h, w, n):
    import vxslam

    img = synth.make_frames(seed, 1, h, w)[0]
    _eq(ctx.orb_extract(img, vxslam.default_orb_params(n_features=n)), oracle.orb_extract(img, n))


@pytest.mark.parametrize("h,w,n", [(480, 640, 2000), (960, 1280, 4000)])
def test_orb_stl_noise_global_fallback(ctx, oracle, h, w, n):
    """Uniform noise: ~24k (VGA) / ~109k (1280 x 960) FAST candidates on level 0, beyond the LDS
    arrays — the selection runs from the level's global scratch."""
    import vxslam

    rng = np.random.default_rng(h)
    for img in (rng.integers(0, 256, (h, w), dtype=np.uint8), rng.integers(0, 256, (h, w, 3), dtype=np.uint8)):
        _eq(ctx.orb_extract(img, vxslam.default_orb_params(n_features=n)), oracle.orb_extract(img, n))


def test_orb_stl_ties_and_strides(ctx, oracle):
    import vxslam

    p = vxslam.default_orb_params(n_features=500)
    yy, xx = np.mgrid[0:240, 0:320]
    chk = (((yy // 7) + (xx // 9)) % 2 * 120 + 60).astype(np.uint8)  # heavy FAST / Harris ties
    for img in (chk, np.ascontiguousarray(chk[:, ::-1]), np.ascontiguousarray(chk.T)):
        _eq(ctx.orb_extract(img, p), oracle.orb_extract(img, 500))
    big = synth.make_frames(21, 1, 480, 700)[0]
    view = np.ascontiguousarray(big[:, 20:660])
    _eq(ctx.orb_extract(view, p), oracle.orb_extract(view, 500))


@pytest.mark.parametrize("b,h,w,n", [(1, 240, 320, 500), (2, 240, 320, 500), (7, 240, 320, 500),
                                     (16, 240, 320, 500), (64, 240, 320, 500), (8, 480, 640, 2000)])
def test_orb_stl_batched(ctx, oracle, b, h, w, n):
    import vxslam

    frames = synth.make_frames(0x57100 + b, b, h, w)
    out = ctx.orb_extract_batch(np.stack(frames), vxslam.default_orb_params(n_features=n), bank=b % 2)
    for f in range(b):
        _eq(out[f], oracle.orb_extract(frames[f], n))
