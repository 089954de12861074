"""Landmark-sharded LocalBA on one GPU (vx_ba_shard_emulate_run).

The sharded path of bench.py at N GPUs — N shard plans of one global window (landmarks split by
splitmix64(id) mod N, each with all its observations), per iteration every shard's pose stage, the
sum of the per-(keyframe, slice) partial blocks over the shards (ncclAllReduce on a real rig),
every shard's landmark stage — run on one device with the all-reduce replaced by a rank-order sum.
Every shard must end with bitwise-identical poses and stop decisions, the union of the shards'
landmarks must be the unsharded result (≤ 1e-4, no gate flips), and both must match the CPU
restatement.  The windows are the ones bench.py builds at N = 2, 4, 8 (N x 50 KF / N x 20k)."""
import numpy as np
import pytest

import vxslam
from vxslam import synth

from test_gpu_parity import _assert_ba_close, _canon

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["fused", "two-kernel"])
def ba_path(request, monkeypatch):
    """Both sharded LocalBA paths: the fused one (k_ba_iter + per-row sums + one all-reduce per
    iteration) and the two-kernel one (k_pose_kf + all-reduce + k_landmark_solve, VX_BA_FUSED=0)."""
    if request.param == "two-kernel":
        monkeypatch.setenv("VX_BA_FUSED", "0")
    else:
        monkeypatch.delenv("VX_BA_FUSED", raising=False)
    return request.param


def _shard_run(ctx, m, opts, n, path=None):
    plans = [ctx.ba_plan(m, opts, shard_rank=r, shard_count=n) for r in range(n)]
    infos = [p.info() for p in plans]
    if path is not None:  # the shard plans carry the fused layout exactly when that path is enabled
        assert [p.layout()["fused"] for p in plans] == [int(path == "fused")] * n
    ctx.ba_shard_emulate(plans)
    outs, stats = [], []
    for p in plans:
        mm = m.copy()
        stats.append(p.fetch(mm))
        outs.append(mm)
        p.close()
    return infos, outs, stats


@pytest.mark.parametrize("n", [2, 4, 8])
def test_sharded_localba_bench_windows(ctx, oracle, n, ba_path):
    nk, nl = 50 * n, 20000 * n
    m = synth.make_ba_map(0x5EED0003, nk, nl, n_streams=n, n_old_kf=2 * n)  # bench.py's rig window
    opts = vxslam.default_ba_options(window=nk)
    infos, outs, stats = _shard_run(ctx, m, opts, n, ba_path)
    assert len({i["n_split"] for i in infos}) == 1 and len({i["n_kf"] for i in infos}) == 1
    assert sum(i["n_opt"] for i in infos) == stats[0].n_landmarks  # the shards partition the landmark set
    # every rank: the same poses (bitwise) and the same stop decisions
    for o, s in zip(outs[1:], stats[1:]):
        assert np.array_equal(o["kf_pose"], outs[0]["kf_pose"])
        assert (s.iterations, list(s.obs[:16]), list(s.cost[:16])) == \
               (stats[0].iterations, list(stats[0].obs[:16]), list(stats[0].cost[:16]))
    # union of the shards' landmarks
    shard = np.array([vxslam.lib().vx_ba_shard_of(int(i), n) for i in m["lm_id"]])
    got = m.copy()
    got["kf_pose"] = outs[0]["kf_pose"]
    lp = got["lm_pos"].reshape(-1, 3).copy()
    for r in range(n):
        sel = shard == r
        lp[sel] = outs[r]["lm_pos"].reshape(-1, 3)[sel]
    got["lm_pos"] = lp.reshape(m["lm_pos"].shape)
    # vs the unsharded GPU run and the CPU restatement
    one = m.copy()
    st1 = ctx.ba_optimize(one, opts)
    _assert_ba_close(got, one, stats[0], st1)
    mc = m.copy()
    stc = oracle.ba_optimize(mc, oracle.ba_options(window=nk))
    # (never skipped; sharded plans sum their rows in slot order, bitwise run to run, so the margin
    # only has to cover GPU-vs-CPU rounding: 1e-7 px, the 8-way window's is 2.4e-7)
    assert stc.gate_margin >= 1e-7, f"gate margin {stc.gate_margin}: reseed this case"
    _assert_ba_close(got, mc, stats[0], stc)


def test_sharded_kernel_choice_is_shared(ctx, oracle, ba_path):
    """A window near the kernel-choice threshold (workgroups x keyframes = 80,000 at 200
    keyframes): the unsharded window runs the large-window kernels, its 2- and 3-way shards the
    LDS-pose kernel, chosen from the maximum workgroup count over the shards so every rank runs the
    same kernels; poses are bitwise equal across ranks and match the unsharded run."""
    nk, nl = 200, 125000
    m = synth.make_ba_map(0x5EED0200, nk, nl, n_streams=8, n_old_kf=16)
    opts = vxslam.default_ba_options(window=nk)
    one = m.copy()
    ctx.ba_optimize(one, opts)
    pc = one["kf_pose"].copy()
    pc[:, :4] = _canon(pc[:, :4])
    for n in (2, 3):
        infos, outs, stats = _shard_run(ctx, m, opts, n, ba_path)
        for o in outs[1:]:
            assert np.array_equal(o["kf_pose"], outs[0]["kf_pose"])
        pg = outs[0]["kf_pose"].copy()
        pg[:, :4] = _canon(pg[:, :4])
        assert (np.abs(pg - pc) / np.maximum(np.abs(pc), 1e-3)).max() <= 1e-4


def test_shard_emulation_rejects_mismatched_plans(ctx):
    m = synth.make_ba_map(7, 12, 2000, n_old_kf=2)
    opts = vxslam.default_ba_options(window=12)
    a = ctx.ba_plan(m, opts, shard_rank=0, shard_count=2)
    b = ctx.ba_plan(m, opts, shard_rank=0, shard_count=2)  # rank 0 twice
    with pytest.raises(vxslam.VxError):
        ctx.ba_shard_emulate([a, b])
    c = ctx.ba_plan(m, vxslam.default_ba_options(window=6), shard_rank=1, shard_count=2)  # another window
    with pytest.raises(vxslam.VxError):
        ctx.ba_shard_emulate([a, c])
    a.close(), b.close(), c.close()


def test_landmark_with_more_observations_than_a_workgroup(ctx, oracle):
    """A snapshot that lists a landmark's (keyframe, feature) pairs over and over (600+ entries,
    more than the 512 observations of a k_landmark_solve workgroup; a Landmark's unordered_map
    cannot hold that, a hand-built snapshot can): the plan reports it (max_lm_obs) and runs the
    one-thread-per-landmark kernels; the result equals the restatement, which walks the same list.
    (The whole list is repeated, not one pair: 600 copies of one ray leave the 3x3 system nearly
    singular along it, where both sides only agree to rounding amplified by the conditioning.)"""
    m = synth.make_ba_map(0x5EED0300, 10, 2000, n_old_kf=2)
    optr = m["lm_obs_ptr"]
    # a landmark observation in the newest keyframe whose feature is a valid observation of it
    k = int(np.argmax(m["kf_id"]))
    f0 = m["kf_feat_ptr"][k]
    ok = False
    for l in range(len(m["lm_id"])):
        if optr[l + 1] - optr[l] < 3:  # a well-conditioned landmark (three rays or more)
            continue
        for o in range(optr[l], optr[l + 1]):
            f = f0 + int(m["obs_feat_idx"][o])
            if (m["obs_kf_id"][o] == m["kf_id"][k] and f < m["kf_feat_ptr"][k + 1] and m["feat_flags"][f] == 1
                    and m["feat_lm_id"][f] == m["lm_id"][l]):
                ok = True
                break
        if ok:
            break
    assert ok
    a, b = int(optr[l]), int(optr[l + 1])
    reps = -(-600 // (b - a))
    extra = (reps - 1) * (b - a)
    for key in ("obs_kf_id", "obs_feat_idx"):
        m[key] = np.concatenate([m[key][:a], np.tile(m[key][a:b], reps), m[key][b:]])
    m["lm_obs_ptr"] = optr + np.concatenate([np.zeros(l + 1, np.int64), np.full(len(optr) - l - 1, extra)])
    opts = vxslam.default_ba_options(window=10)
    plan = ctx.ba_plan(m, opts)
    assert plan.info()["max_lm_obs"] >= 512
    plan.run_async()
    mg = m.copy()
    stg = plan.fetch(mg)
    plan.close()
    mc = m.copy()
    stc = oracle.ba_optimize(mc, oracle.ba_options(window=10))
    _assert_ba_close(mg, mc, stg, stc)


@pytest.mark.parametrize("n", [2, 4])
def test_sharded_sequence_graph_replay(ctx, n, ba_path):
    """The sharded iteration sequence (row sums -> the reduction that stands in for ncclAllReduce ->
    k_ba_iter, or pose stage -> reduction -> landmark stage) through the graph cache, as a real
    sharded plan's runs after its first (vx_ba_plan_run_async): run 1 decides the kernels eagerly,
    run 2 is the first sighting (eager), run 3 is captured, runs 4-5 replay — every run bitwise equal."""
    nk, nl = 50 * n, 20000 * n
    m = synth.make_ba_map(0x5EED0003, nk, nl, n_streams=n, n_old_kf=2 * n)
    opts = vxslam.default_ba_options(window=nk)
    plans = [ctx.ba_plan(m, opts, shard_rank=r, shard_count=n) for r in range(n)]
    cap0, lau0 = ctx.graph_counts()
    runs = []
    for _ in range(5):
        ctx.ba_shard_emulate(plans)
        res = []
        for p in plans:
            mm = m.copy()
            st = p.fetch(mm)
            res.append((mm["kf_pose"].copy(), mm["lm_pos"].copy(), st.iterations, list(st.obs[:16]), list(st.cost[:16])))
        runs.append(res)
    cap1, lau1 = ctx.graph_counts()
    assert cap1 == cap0 + 1 and lau1 >= lau0 + 3, (cap0, lau0, cap1, lau1)
    for res in runs[1:]:
        for a, b in zip(res, runs[0]):
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2:] == b[2:]
    for p in plans:
        p.close()


@pytest.mark.parametrize("n", [2, 4])
def test_sharded_peer_reduction_matches_rank_order_sum(ctx, monkeypatch, n):
    """The one-shot peer reduction ($VX_BA_PEER=1: each shard publishes its row sums into its own
    block with a generation flag, every shard waits for all flags and sums the blocks in rank order)
    in place of the emulated all-reduce: bitwise the rank-order sum's results — poses, positions and
    stop decisions — over repeated runs of the same plans (generations advancing, both parities)."""
    nk, nl = 50 * n, 20000 * n
    m = synth.make_ba_map(0x5EED0003, nk, nl, n_streams=n, n_old_kf=2 * n)
    opts = vxslam.default_ba_options(window=nk)
    monkeypatch.delenv("VX_BA_FUSED", raising=False)
    monkeypatch.delenv("VX_BA_PEER", raising=False)
    _, ref_outs, ref_stats = _shard_run(ctx, m, opts, n, "fused")
    monkeypatch.setenv("VX_BA_PEER", "1")
    plans = [ctx.ba_plan(m, opts, shard_rank=r, shard_count=n) for r in range(n)]
    try:
        for rep in range(3):  # (generations 5 rep + 1 .. 5 rep + 5: both parities, flags from earlier runs)
            ctx.ba_shard_emulate(plans)
            for p, ro, rs in zip(plans, ref_outs, ref_stats):
                mm = m.copy()
                st = p.fetch(mm)
                assert (st.iterations, list(st.obs[:16]), list(st.cost[:16])) == \
                       (rs.iterations, list(rs.obs[:16]), list(rs.cost[:16]))
                assert np.array_equal(mm["kf_pose"], ro["kf_pose"])
                assert np.array_equal(mm["lm_pos"], ro["lm_pos"])
    finally:
        for p in plans:
            p.close()
