"""Essential-matrix RANSAC + recoverPose (vx_essential_ransac) on one MI355X: per-call wall time
(host buffers in / out), the two kernels' device time (HIP events), a batch of 8, and the CPU
restatement on the same input.  One JSON line per case."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402
import pyoracle  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = vxslam.Context(0)
for n, frac, P, H in [(1000, 0.3, 1, 1000), (2000, 0.3, 1, 1000), (1000, 0.5, 1, 1000), (1000, 0.3, 8, 1000),
                      (1000, 0.3, 1, 128)]:
    ps = [synth.make_two_view(7 + k, n, outlier_frac=frac) for k in range(P)]
    offs = np.cumsum([0] + [n] * P)
    p1 = np.concatenate([p["pts_last"] for p in ps])
    p2 = np.concatenate([p["pts_curr"] for p in ps])
    intr = np.stack([p["intr"] for p in ps])
    opts = np.stack([vxslam.essential_options(max_iterations=H, seed=k) for k in range(P)])
    for _ in range(2):
        ctx.essential_ransac_batch(offs, p1, p2, intr, opts)
    t0 = time.perf_counter()
    for _ in range(K):
        out, mask = ctx.essential_ransac_batch(offs, p1, p2, intr, opts)
    wall = (time.perf_counter() - t0) / K * 1e3
    ctx.prof_enable(True, ["em_hypotheses", "em_select"])
    for _ in range(K):
        ctx.essential_ransac_batch(offs, p1, p2, intr, opts)
    st = ctx.prof_read(reset=True)
    ctx.prof_enable(False)
    dev = {k: round(ms / c * 1e3, 2) for k, (ms, c) in st.items() if c and k.startswith("em")}
    t0 = time.perf_counter()
    reps = max(1, 4 // P)
    for _ in range(reps):
        pyoracle.essential_ransac_batch(offs, p1, p2, intr, opts)
    cpu = (time.perf_counter() - t0) / reps * 1e3
    err = max(float(np.abs(out[k]["R"].reshape(3, 3) - ps[k]["R"]).max()) for k in range(P))
    print(json.dumps({"n": n, "outlier_frac": frac, "problems": P, "max_iterations": H,
                      "hypotheses_run": [int(x) for x in out["hypotheses_run"]],
                      "ransac_inliers": [int(x) for x in out["n_ransac_inliers"]],
                      "inliers": [int(x) for x in out["n_inliers"]], "ms_per_call": round(wall, 4),
                      "kernel_us": dev, "cpu_restatement_ms": round(cpu, 3), "R_err_vs_truth": err}), flush=True)
