"""The N > 1 path on CPU with torch.distributed gloo, world_size 2 (no GPU).

* bench.py's distributed harness: barrier-bracketed timing, max over ranks.
* landmark-sharded BA: each rank's host plan (vx_ba_plan_inspect) owns a disjoint
  landmark shard; the per-keyframe normal equations of the pose stage computed from each shard
  and summed by an all-reduce equal the unsharded ones.  On the GPU the same reduction is one
  ncclAllReduce(sum, f64) of the 32-double keyframe blocks per iteration (ba.hip).
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world=2):
    import torch.multiprocessing as mp

    port = _free_port()
    mp.spawn(fn, args=(world, port), nprocs=world, join=True)


def _init(rank, world, port):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    for p in (os.path.join(ROOT, "visionx-slam_amd", "python"), ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _timing_worker(rank, world, port):
    import time

    dist = _init(rank, world, port)
    import bench

    d = bench.Dist(world)
    assert d.world == world and d.rank == rank
    calls = []

    def step(i):
        calls.append(i)
        time.sleep(0.002 * (rank + 1))  # rank 1 is slower: the reported time must be rank 1's

    el = bench.timed_loop(step, 5, 2, lambda: None, d)
    assert calls == list(range(7))
    assert el >= 5 * 0.004 * 0.9
    uid = d.broadcast_bytes(b"x" * 128 if rank == 0 else None)
    assert uid == b"x" * 128
    dist.destroy_process_group()


def test_bench_harness_max_over_ranks():
    _spawn(_timing_worker)


def pose_normal_equations(m, opts_window, lm_subset=None):
    """Per-window-keyframe 29-term blocks of the first pose stage (local_ba.cpp:131-161), numpy."""
    from vxslam import synth

    ids = m["kf_id"]
    order = np.argsort(ids)
    win = order[-opts_window:]
    lm_index = {int(i): n for n, i in enumerate(m["lm_id"])}
    out = np.zeros((len(win), 29))
    for r, k in enumerate(win):
        q, t = m["kf_pose"][k, :4], m["kf_pose"][k, 4:]
        R = synth.quat_to_mat(q)
        fx, fy, cx, cy = m["kf_intr"][k]
        for f in range(m["kf_feat_ptr"][k], m["kf_feat_ptr"][k + 1]):
            fl = m["feat_flags"][f]
            if not (fl & 1) or (fl & 2):
                continue
            l = lm_index.get(int(m["feat_lm_id"][f]))
            if l is None or m["lm_bad"][l] or (lm_subset is not None and l not in lm_subset):
                continue
            pc = R @ m["lm_pos"][l] + t
            if pc[2] <= 1e-6:
                continue
            e = m["feat_uv"][f] - np.array([fx * pc[0] / pc[2] + cx, fy * pc[1] / pc[2] + cy])
            if np.linalg.norm(e) > 5.0:
                continue
            x, y, z = pc
            Jp = np.array([[fx / z, 0, -fx * x / z ** 2], [0, fy / z, -fy * y / z ** 2]])
            J = Jp @ np.hstack([np.eye(3), -np.array([[0, -z, y], [z, 0, -x], [-y, x, 0]])])
            H = J.T @ J
            out[r, :21] += H[np.triu_indices(6)]
            out[r, 21:27] += -J.T @ e
            out[r, 27] += e @ e
            out[r, 28] += 1
    return out


def _shard_worker(rank, world, port):
    dist = _init(rank, world, port)
    import torch

    import vxslam
    from vxslam import synth

    m = synth.make_ba_map(17, 6, 600, n_old_kf=2)
    opts = vxslam.default_ba_options(window=6)
    mine = vxslam.ba_plan_inspect(m, opts, shard_rank=rank, shard_count=world)
    full = vxslam.ba_plan_inspect(m, opts)
    part = pose_normal_equations(m, 6, set(mine["lm_map_idx"].tolist()))
    assert int(part[:, 28].sum()) <= full["n_pose_obs"]
    t = torch.from_numpy(part.copy())
    dist.all_reduce(t)
    ref = pose_normal_equations(m, 6)
    got = t.numpy()
    assert np.allclose(got, ref, rtol=1e-9, atol=1e-9 * np.abs(ref).max())
    counts = torch.tensor([mine["n_opt"], mine["n_pose_obs"], mine["n_lm_obs"]], dtype=torch.int64)
    dist.all_reduce(counts)
    assert counts.tolist() == [full["n_opt"], full["n_pose_obs"], full["n_lm_obs"]]
    dist.destroy_process_group()


def test_sharded_pose_normal_equations_allreduce():
    _spawn(_shard_worker)


def _parity_worker(rank, world, port):
    """bench.py's N > 1 parity path (shard_result -> Dist.gather -> parity_vs_unsharded -> the JSON
    field) with the restatement standing in for the GPU runs: the unsharded result split by the shard
    hash is what a correct sharded run returns."""
    import json

    dist = _init(rank, world, port)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    import pyoracle
    import vxslam
    from vxslam import synth

    m = synth.make_ba_map(23, 6, 800, n_old_kf=2)
    opts = vxslam.default_ba_options(window=6)
    mm = m.copy()
    st = pyoracle.ba_optimize(mm, pyoracle.ba_options(window=6))
    mine = bench.shard_result(mm, vxslam.ba_plan_inspect(m, opts, shard_rank=rank, shard_count=world), st)
    d = bench.Dist(world)
    shards = d.gather(mine)
    if rank == 0:
        assert len(shards) == world
        ref = bench.shard_result(mm, vxslam.ba_plan_inspect(m, opts), st)
        par = bench.parity_vs_unsharded(shards, ref)
        assert par["ok"] and par["shards_partition"] and par["ranks_agree"] and par["gate_flips"] == 0, par
        assert par["landmarks"] == sum(len(s["lm_idx"]) for s in shards) > 0
        json.dumps(par)  # (goes into the JSON line)
        bad = [dict(s) for s in shards]
        bad[1]["lm_pos"] = bad[1]["lm_pos"] * (1 + 1e-3)
        assert not bench.parity_vs_unsharded(bad, ref)["ok"]
        bad = [dict(s) for s in shards]
        bad[0]["lm_idx"], bad[0]["lm_pos"] = bad[0]["lm_idx"][1:], bad[0]["lm_pos"][1:]
        assert not bench.parity_vs_unsharded(bad, ref)["shards_partition"]
        bad = [dict(s) for s in shards]
        bad[1]["pose"] = bad[1]["pose"].copy()
        bad[1]["pose"][0, 4] += 1e-12  # ranks must agree bitwise
        assert not bench.parity_vs_unsharded(bad, ref)["ranks_agree"]
        bad = [dict(s) for s in shards]
        bad[0]["obs"] = [o + 1 for o in bad[0]["obs"]]
        assert bench.parity_vs_unsharded(bad, ref)["gate_flips"] > 0
    else:
        assert shards is None
    dist.destroy_process_group()


def test_bench_sharded_parity_field():
    _spawn(_parity_worker)


def _gate_worker(rank, world, port):
    """bench.py's N > 1 parity gate: a passing verdict lets every rank through; a failing one (rank 0's
    verdict, broadcast) makes rank 0 print an INVALID JSON line and every rank exit with status 3."""
    import contextlib
    import io
    import json
    import types

    _init(rank, world, port)
    import bench

    d = bench.Dist(world)
    args = types.SimpleNamespace(steps=5, warmup=2)
    assert bench.sharded_parity_gate({"ok": True} if rank == 0 else None, d, args) is True
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        try:
            bench.sharded_parity_gate({"ok": False, "gate_flips": 1} if rank == 0 else None, d, args)
            raise AssertionError("a failing sharded parity must stop the run")
        except SystemExit as e:
            assert e.code == 3
    if rank == 0:
        line = json.loads(out.getvalue().strip())
        assert line["metric"].startswith("INVALID") and line["value"] is None
        assert line["parity_vs_unsharded"]["gate_flips"] == 1 and line["n_gpus"] == world
    else:
        assert out.getvalue() == ""


def test_bench_parity_gate_failing_branch():
    _spawn(_gate_worker)


def _sba_shard_worker(rank, world, port):
    """The Schur-complement BA's sharded reduction (csrc/sba.hip: every rank assembles the reduced
    pose system from its own landmark shard, one ncclAllReduce sums the ranks' systems, damping and
    the fixed-keyframe gauge are applied once after it) with gloo standing in for RCCL: the partial
    systems of the restatement, all-reduced and finished, equal its unsharded system."""
    dist = _init(rank, world, port)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch

    import pyoracle as O
    from vxslam import synth

    nk = 8
    m = synth.make_ba_map(29, nk, 1500, n_streams=2, n_old_kf=4)
    opts = O.sba_options(window=nk, iters=4)
    lam = 3e-3
    S, rhs, htd, cost, cnt = O.sba_system_shard(m, rank, world, opts, lam)
    # every observation belongs to exactly one shard, so no rank holds everything
    full = O.sba_system_shard(m, 0, 1, opts, lam)
    assert 0 < cnt < full[4]
    buf = torch.from_numpy(np.concatenate([S.ravel(), rhs, htd, [cost, cnt]]))
    dist.all_reduce(buf)  # (the GPU: one ncclAllReduce(sum, f64) of the same blocks per LM iteration)
    n = 6 * nk
    b = buf.numpy()
    Ss, rs, hs = b[: n * n].reshape(n, n).copy(), b[n * n: n * n + n].copy(), b[n * n + n: n * n + 2 * n]
    assert int(round(b[-1])) == full[4] and abs(b[-2] - full[3]) <= 1e-9 * full[3]
    # finish once, after the reduction: fixed rows (the oldest fixed_keyframes window rows; every synth
    # keyframe has a camera) get the identity and rhs 0, the free rows the Marquardt damping
    for r in range(nk):
        sl = slice(6 * r, 6 * r + 6)
        if r < opts.fixed_keyframes:
            Ss[sl, :] = 0.0
            Ss[:, sl] = 0.0
            Ss[sl, sl] = np.eye(6)
            rs[sl] = 0.0
        else:
            Ss[sl, sl] += np.diag(lam * hs[sl] + 1e-6)
    Sref, rref = O.sba_system(m, opts, lam)
    tol = 1e-9 * np.abs(Sref).max()
    assert np.abs(np.tril(Ss) - np.tril(Sref)).max() <= tol
    assert np.abs(rs - rref).max() <= 1e-9 * np.abs(rref).max()
    # the shards' landmark sets partition the window's: the rank totals of valid observations add up
    counts = torch.tensor([cnt], dtype=torch.int64)
    dist.all_reduce(counts)
    assert int(counts.item()) == full[4]
    dist.destroy_process_group()


def test_sharded_schur_system_allreduce():
    _spawn(_sba_shard_worker)


def _peer_worker(rank, world, port):
    """The peer reduction's protocol (ba.hip k_peer_publish / k_peer_gather, $VX_BA_PEER=1) between
    processes: every rank's block in memory the others map (shared memory here, IPC over xGMI on the
    GPUs; the names gathered over gloo as the IPC handles are over RCCL), rows double-buffered by
    generation parity, a flag per block set after the rows; a rank waits for every flag >= gen, then
    sums the blocks in rank order.  Ranks run at skewed, random speeds: no rank may read a block a
    faster rank has already overwritten, and every sum must equal the all-reduce of the same rows."""
    dist = _init(rank, world, port)
    import time
    from multiprocessing import shared_memory

    import torch

    nrow = 64
    rng = np.random.default_rng(1000 + rank)
    shm = shared_memory.SharedMemory(create=True, size=(2 * nrow + 1) * 8)
    own = np.ndarray((2 * nrow + 1,), np.float64, buffer=shm.buf)
    own[:] = 0.0
    names = [None] * world
    dist.all_gather_object(names, shm.name)  # (the IPC handle exchange)
    peers = [shared_memory.SharedMemory(name=nm) for nm in names]
    blocks = [np.ndarray((2 * nrow + 1,), np.float64, buffer=p.buf) for p in peers]
    sent, summed = [], []
    try:
        for gen in range(1, 41):
            rows = np.round(rng.normal(size=nrow) * 1e3) + gen * 1e6 + rank  # (exact in float64)
            par = gen & 1
            own[par * nrow:(par + 1) * nrow] = rows  # publish, then the flag
            own[2 * nrow] = float(gen)
            t0 = time.time()
            while min(b[2 * nrow] for b in blocks) < gen:
                assert time.time() - t0 < 20.0, "a flag did not arrive"
                time.sleep(1e-4)
            time.sleep(float(rng.random()) * 3e-3)  # (skew: a slow reader while the others run ahead)
            got = blocks[0][par * nrow:(par + 1) * nrow].copy()
            for b in blocks[1:]:
                got += b[par * nrow:(par + 1) * nrow]
            sent.append(rows)
            summed.append(got)
        # (compared only at the end: a collective per generation would hold the ranks in step)
        ref = torch.from_numpy(np.stack(sent))
        dist.all_reduce(ref)
        bad = np.nonzero(~np.all(np.stack(summed) == ref.numpy(), axis=1))[0]
        assert bad.size == 0, f"rank {rank}: generations {bad + 1} read an overwritten or stale block"
        dist.barrier()
    finally:
        for p in peers:
            p.close()
        shm.close()
        dist.barrier()
        shm.unlink()
        dist.destroy_process_group()


def test_peer_reduction_protocol():
    _spawn(_peer_worker)
