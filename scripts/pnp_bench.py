"""PnP RANSAC (vx_pnp_ransac) on one MI355X: per-call wall time (host buffers in and out, as the
tracking thread calls it), the two kernels' device time (HIP events), a batch of 8 problems (C5 rig),
and the CPU restatement on the same input.  One JSON line per case."""
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

K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = vxslam.Context(0)
for n, frac, P, refine in [(1000, 0.3, 1, 20), (2000, 0.3, 1, 20), (2000, 0.3, 1, 0), (2000, 0.6, 1, 20),
                           (1000, 0.3, 8, 20)]:
    ps = [synth.make_pnp_problem(7 + k, n, outlier_frac=frac) for k in range(P)]
    offs = np.cumsum([0] + [n] * P)
    obj = np.concatenate([p["obj"] for p in ps])
    img = np.concatenate([p["img"] for p in ps])
    intr = np.stack([p["intr"] for p in ps])
    opts = np.stack([vxslam.pnp_options(n, seed=k, refine_iterations=refine) for k in range(P)])
    for _ in range(3):
        ctx.pnp_ransac_batch(offs, obj, img, intr, opts)
    t0 = time.perf_counter()
    for _ in range(K):
        out, mask = ctx.pnp_ransac_batch(offs, obj, img, intr, opts)
    wall = (time.perf_counter() - t0) / K * 1e3
    ctx.prof_enable(True, ["pnp_hypotheses", "pnp_refine"])
    for _ in range(K):
        ctx.pnp_ransac_batch(offs, obj, img, intr, opts)
    st = ctx.prof_read(reset=True)
    ctx.prof_enable(False)
    dev = {k: round(ms / c * 1e3, 2) for k, (ms, c) in st.items() if c and k.startswith("pnp")}
    t0 = time.perf_counter()
    reps = max(1, 20 // P)
    for _ in range(reps):
        oc, _ = pyoracle.pnp_ransac_batch(offs, obj, img, intr, opts)
    cpu = (time.perf_counter() - t0) / reps * 1e3
    err = max(float(np.abs(out[k]["pose"] - ps[k]["pose"]).max()) for k in range(P))
    print(json.dumps({"n": n, "outlier_frac": frac, "problems": P, "hypotheses": int(opts[0]["max_iterations"]),
                      "hypotheses_run": [int(x) for x in out["hypotheses_run"]],
                      "inliers": [int(x) for x in out["n_inliers"]],
                      "refine_iterations": [int(x) for x in out["refine_iterations"]], "ms_per_call": round(wall, 4),
                      "kernel_us": dev, "cpu_restatement_ms": round(cpu, 3), "pose_err_vs_truth": err}), flush=True)
