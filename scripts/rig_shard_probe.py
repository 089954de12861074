"""Per-rank LocalBA work of the N-GPU bench rig, on one GPU: the rig's global window (N x 50 KF /
N x 20k landmarks) restricted to one shard's landmarks (the others marked bad, their features
unlinked) and run as an unsharded plan — the same kernels and sizes a rank runs, without the
per-iteration RCCL all-reduce.  Prints ms per LocalBA run (graph replay, 200 runs)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (loads the HIP runtime the library links against)
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402


def shard_map(m, n, rank):
    mm = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in m.items()}
    own = np.array([vxslam.ba_shard_of(int(i), n) == rank for i in m["lm_id"]])
    mm["lm_bad"] = np.where(own, m["lm_bad"], 1).astype(np.uint8)
    mine = set(m["lm_id"][own].tolist())
    linked = (m["feat_flags"] & 1).astype(bool)
    keep = np.array([(not f) or (int(i) in mine) for f, i in zip(linked, m["feat_lm_id"])])
    mm["feat_flags"] = np.where(keep, m["feat_flags"], m["feat_flags"] & 0xFE).astype(np.uint8)
    return mm


def run(ctx, m, window, reps=200):
    plan = ctx.ba_plan(m, vxslam.default_ba_options(window=window))
    for _ in range(10):
        plan.run_async()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.run_async()
    ctx.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / reps
    info = plan.info()
    plan.close()
    return ms, info


def main():
    ctx = vxslam.Context(0)
    for n in (1, 2, 4, 8):
        m = synth.make_ba_map(0x5EED0003, 50 * n, 20000 * n, n_streams=n, n_old_kf=2 * n)
        full_ms, full_info = run(ctx, m, 50 * n)
        ms, info = run(ctx, shard_map(m, n, 0) if n > 1 else m, 50 * n)
        print(f"N={n}: whole window {full_ms:.4f} ms ({full_info}); rank-0 shard {ms:.4f} ms ({info})", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
