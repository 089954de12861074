"""LocalBA alone (one context, graph replay) across window sizes: the default kernel choice
(plan_run: k_pose_kf + k_landmark_solve with every pose in LDS below the crossover, the
large-window kernels above it) against the large-window kernels forced by VX_PLAN_GLOBAL_POSES
(k_pose_kf + k_pose_solve_g + k_landmark): ms per run and whether both give the same final state.
Run with the crossover disabled, it measured the rule plan_run encodes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

CASES = [(50, 20000, 1), (100, 20000, 2), (200, 20000, 4), (300, 20000, 6), (400, 20000, 8),
         (100, 50000, 1), (50, 100000, 1), (200, 50000, 4), (200, 100000, 8), (400, 40000, 8),
         (400, 60000, 8), (400, 80000, 8), (300, 60000, 6), (400, 160000, 8)]
c = vxslam.Context(0)
for nk, nl, ns in CASES:
    m = synth.make_ba_map(0x5EED0003, nk, nl, n_streams=ns, n_old_kf=2 * ns)
    opts = vxslam.default_ba_options(window=nk)
    res = {}
    for gp in (False, True):
        plan = c.ba_plan(m, opts, global_poses=gp)
        for _ in range(3):
            plan.run_async()
        c.synchronize()
        K = 50
        t0 = time.perf_counter()
        for _ in range(K):
            plan.run_async()
        c.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / K
        mm = m.copy()
        st = plan.fetch(mm)
        res[gp] = (ms, st.iterations, mm["kf_pose"].copy(), mm["lm_pos"].copy())
        info = plan.info()
        plan.close()
    (a, ia, pa, la), (b, ib, pb, lb) = res[False], res[True]
    same = ia == ib and np.array_equal(pa, pb) and np.array_equal(la, lb)
    dl = float(np.max(np.abs(la - lb) / np.maximum(np.abs(lb), 1e-3)))
    print(f"[blocks {info['n_lm_blocks']:5d}, kf*blocks {nk * info['n_lm_blocks']:7d}] "
          f"{nk:4d} KF {nl:6d} LM: default {a:.4f} ms  global-poses {b:.4f} ms  iters {ia}/{ib}  "
          f"bitwise-equal {same}  max rel diff {dl:.2e}", flush=True)
c.close()
