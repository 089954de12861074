"""Batched extraction and matching (vx_orb_extract_batch_async, vx_match_batch_async) against the
single-frame GPU path and the CPU restatement.

Bar: every frame of a batch bit-exact with the oracle (keypoints, descriptors); every pair of a
batched match identical to the oracle's BFMatcher kNN-2 + ratio (orb_matcher.cpp:22-36).
"""
import numpy as np
import pytest

from vxslam import synth

pytestmark = pytest.mark.gpu


def _eq(a, b):
    (kg, dg), (kc, dc) = a, b
    assert len(kg) == len(kc), (len(kg), len(kc))
    for f in ("octave", "x", "y", "response", "angle"):
        assert np.array_equal(kg[f], kc[f]), f
    assert np.array_equal(dg, dc)


def _device_stack(frames):
    import torch

    return torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to("cuda:0")


@pytest.mark.parametrize("b,h,w,n,gray", [(1, 240, 320, 500, False), (3, 240, 320, 500, True),
                                          (8, 480, 640, 2000, False), (5, 333, 517, 800, False),
                                          (6, 333, 517, 800, True), (3, 961, 1283, 4000, False)])
def test_orb_batch_matches_oracle(ctx, oracle, b, h, w, n, gray):
    import vxslam

    frames = synth.make_frames(0xBA7C0 + b, b, h, w)
    if gray:
        frames = [f.mean(axis=2).astype(np.uint8) for f in frames]
    p = vxslam.default_orb_params(n_features=n)
    out = ctx.orb_extract_batch(np.stack(frames), p, bank=b % 2)
    assert len(out) == b
    for f in range(b):
        ref = oracle.orb_extract(frames[f], n) if f < 3 else ctx.orb_extract(frames[f], p)
        _eq(out[f], ref)


@pytest.mark.parametrize("b", [2, 4])
def test_orb_batch_fused_pyramid_with_grid_share(oracle, b):
    """Grid share 1/B: the fused pyramid's grid for B frames fits one round, so the batch runs the
    fused pyramid (blockIdx.z = frame) instead of the level chain; same results."""
    import vxslam

    c = vxslam.Context(0)
    try:
        c.set_grid_share(1.0 / b)
        frames = synth.make_frames(0xBA7C8 + b, b, 480, 640)
        p = vxslam.default_orb_params(n_features=2000)
        out = c.orb_extract_batch(np.stack(frames), p)
        for f in range(b):
            _eq(out[f], oracle.orb_extract(frames[f], 2000))
    finally:
        c.close()


def test_orb_batch_padded_strides_and_blank_frame(ctx, oracle):
    """Frames in a pitched allocation (row stride > width, frame stride > frame) and a blank frame
    (no corners: zero keypoints) inside the batch."""
    import torch

    import vxslam

    h, w, n = 200, 260, 300
    frames = synth.make_frames(0xBA7D0, 3, h, w)
    frames[1] = np.full((h, w, 3), 117, np.uint8)
    buf = np.zeros((3, h + 5, w * 3 + 40), np.uint8)
    for f in range(3):
        buf[f, :h, :w * 3] = frames[f].reshape(h, w * 3)
    d = torch.from_numpy(buf).to("cuda:0")
    p = vxslam.default_orb_params(n_features=n)
    ctx.orb_extract_batch_async(d.data_ptr(), 3, d.stride(0), w, h, 3, d.stride(1), 0, p)
    for f in range(3):
        got = ctx.orb_batch_fetch(0, f)
        _eq(got, oracle.orb_extract(frames[f], n))
    assert len(ctx.orb_batch_fetch(0, 1)[0]) == 0


def test_orb_batch_interleaved_with_single_frames(ctx, oracle):
    """Single-frame extraction (graph-replayed) before and after a batch that grows the scratch
    buffers: the single-frame graphs must not replay stale pointers."""
    import vxslam

    h, w, n = 240, 320, 500
    frames = synth.make_frames(0xBA7E0, 6, h, w)
    p = vxslam.default_orb_params(n_features=n)
    ref = [oracle.orb_extract(f, n) for f in frames[:2]]
    d = _device_stack(frames)
    for _ in range(3):  # eager, capture, replay
        ctx.orb_extract_async(d[0].data_ptr(), w, h, 3, d.stride(1), 0, p)
    _eq(ctx.orb_fetch(0), ref[0])
    for rep in range(3):
        ctx.orb_extract_batch_async(d.data_ptr(), 6, d.stride(0), w, h, 3, d.stride(1), 1, p)
        _eq(ctx.orb_batch_fetch(1, 0), ref[0])
        _eq(ctx.orb_batch_fetch(1, 1), ref[1])
    for _ in range(3):
        ctx.orb_extract_async(d[1].data_ptr(), w, h, 3, d.stride(1), 0, p)
        _eq(ctx.orb_fetch(0), ref[1])


def test_match_batch_matches_oracle(ctx, oracle):
    """Two banks of a 4-camera rig (frames t-1 and t): each camera's pair matched in one batched
    call, plus a pair against an empty set; identical to the oracle pair by pair."""
    import vxslam

    h, w, n = 240, 320, 500
    cams = 4
    seq = [synth.make_frames(0xBA7F0 + c, 2, h, w) for c in range(cams)]
    prev = np.stack([s[0] for s in seq])
    cur = np.stack([s[1] for s in seq])
    cur[3] = 117  # blank frame: no descriptors
    p = vxslam.default_orb_params(n_features=n)
    d0, d1 = _device_stack(list(prev)), _device_stack(list(cur))
    ctx.orb_extract_batch_async(d0.data_ptr(), cams, d0.stride(0), w, h, 3, d0.stride(1), 0, p)
    ctx.orb_extract_batch_async(d1.data_ptr(), cams, d1.stride(0), w, h, 3, d1.stride(1), 1, p)
    pairs = [(ctx.batch_device(0, c), ctx.batch_device(1, c)) for c in range(cams)]
    ctx.match_batch_async(pairs)
    for c in range(cams):
        q = ctx.orb_batch_fetch(0, c)[1]
        t = ctx.orb_batch_fetch(1, c)[1]
        got = ctx.match_batch_fetch(c)
        ref = oracle.match(q, t)
        assert np.array_equal(got, ref), c
    assert len(ctx.match_batch_fetch(3)) == 0
    # the same pairs one at a time through vx_match_device_async
    for c in range(cams):
        ctx.match_device_async(*pairs[c])
        assert np.array_equal(ctx.match_fetch(), ctx.match_batch_fetch(c))


def test_batch_maximum_sizes(ctx, oracle):
    """VX_MAX_BATCH frames in one call and VX_MAX_MATCH_PAIRS pairs in one match call (small frames),
    including pairs with an empty query or train side."""
    import vxslam

    h, w, n = 96, 128, 150
    frames = synth.make_frames(0xBA800, 64, h, w)
    for f in (5, 17):
        frames[f] = np.full_like(frames[f], 90)
    p = vxslam.default_orb_params(n_features=n)
    out = ctx.orb_extract_batch(np.stack(frames), p, bank=0)
    for f in (0, 5, 17, 63):
        _eq(out[f], oracle.orb_extract(frames[f], n))
    for f in range(64):
        _eq(out[f], ctx.orb_extract(frames[f], p))
    pairs = [(ctx.batch_device(0, 2 * i), ctx.batch_device(0, 2 * i + 1)) for i in range(16)]
    pairs[2] = (ctx.batch_device(0, 5), ctx.batch_device(0, 6))    # empty query side
    pairs[8] = (ctx.batch_device(0, 16), ctx.batch_device(0, 17))  # empty train side
    ctx.match_batch_async(pairs)
    idx = [(2 * i, 2 * i + 1) for i in range(16)]
    idx[2], idx[8] = (5, 6), (16, 17)
    for i, (a, b) in enumerate(idx):
        ref = oracle.match(out[a][1], out[b][1]) if len(out[a][1]) and len(out[b][1]) else []
        got = ctx.match_batch_fetch(i)
        assert len(got) == len(ref), i
        if len(ref):
            assert np.array_equal(got, ref), i


def test_batch_invalid_arguments(ctx):
    import vxslam

    p = vxslam.default_orb_params(n_features=100)
    d = _device_stack([np.zeros((64, 80, 3), np.uint8)])
    with pytest.raises(vxslam.VxError):
        ctx.orb_extract_batch_async(d.data_ptr(), 0, d.stride(0), 80, 64, 3, d.stride(1), 0, p)
    with pytest.raises(vxslam.VxError):
        ctx.orb_extract_batch_async(d.data_ptr(), 65, d.stride(0), 80, 64, 3, d.stride(1), 0, p)
    with pytest.raises(vxslam.VxError):
        ctx.orb_extract_batch_async(d.data_ptr(), 1, d.stride(0), 80, 64, 3, d.stride(1), 2, p)
    with pytest.raises(vxslam.VxError):  # frame stride shorter than a frame
        ctx.orb_extract_batch_async(d.data_ptr(), 2, 100, 80, 64, 3, d.stride(1), 0, p)
    ctx.orb_extract_batch_async(d.data_ptr(), 1, d.stride(0), 80, 64, 3, d.stride(1), 0, p)
    with pytest.raises(vxslam.VxError):
        ctx.orb_batch_fetch(0, 1)
    with pytest.raises(vxslam.VxError):
        ctx.match_batch_async([])
    with pytest.raises(vxslam.VxError):
        ctx.match_batch_fetch(99)
