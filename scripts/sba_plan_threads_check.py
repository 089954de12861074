#!/usr/bin/env python3
"""The Schur plan built on 1 host thread and on the default thread count gives the same run,
bitwise (poses, landmark positions, iterations, cost), at C3 / C4 / C5; prints the plan-build time
of each (VX_SBA_PLAN_THREADS is read once per process, so each setting runs in a child process)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))

CHILD = r"""
import json, sys, time
import numpy as np
sys.path.insert(0, sys.argv[1])
import vxslam
from vxslam import synth
ctx = vxslam.Context(0)
out = {}
for cfg in ("C3", "C4", "C5"):
    nk, nl, ns = synth.ba_config(cfg)
    m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns)
    o = vxslam.default_sba_options(window=nk, iters=8)
    ts = []
    for r in range(4):
        t0 = time.perf_counter()
        p = ctx.sba_plan(m, o)
        ts.append(1e3 * (time.perf_counter() - t0))
        if r < 3:
            p.close()
    mm = m.copy()
    p.run_async()
    st = p.fetch(mm)
    p.close()
    out[cfg] = {"build_ms": round(min(ts[1:]), 3), "iterations": int(st.iterations),
                "pose": np.asarray(mm["kf_pose"]).tobytes().hex()[:0] or
                        __import__("hashlib").sha256(np.asarray(mm["kf_pose"]).tobytes()).hexdigest(),
                "pos": __import__("hashlib").sha256(np.asarray(mm["lm_pos"]).tobytes()).hexdigest()}
print(json.dumps(out))
"""

res = {}
for threads in ("1", ""):
    env = dict(os.environ)
    if threads:
        env["VX_SBA_PLAN_THREADS"] = threads
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "visionx-slam_amd", "python")],
                       env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        print(r.stderr[-2000:])
        sys.exit(1)
    res[threads or "default"] = json.loads(r.stdout.strip().splitlines()[-1])
for cfg in ("C3", "C4", "C5"):
    a, b = res["1"][cfg], res["default"][cfg]
    same = a["pose"] == b["pose"] and a["pos"] == b["pos"] and a["iterations"] == b["iterations"]
    print(f"{cfg}: plan build {a['build_ms']} ms (1 thread) -> {b['build_ms']} ms (default); "
          f"runs bitwise equal: {same}")
    if not same:
        sys.exit(2)
