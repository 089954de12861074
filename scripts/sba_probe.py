"""Times the Schur-complement BA (vx_sba_*) per stage on one MI355X: C2 / C3 windows.
Usage: python scripts/sba_probe.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import numpy as np  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = vxslam.Context(0)
for cfg in ["C2", "C3", "C4"]:
    nk, nl, ns = synth.ba_config(cfg)
    m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns)
    plan = ctx.sba_plan(m, vxslam.default_sba_options(window=nk, iters=8))
    info = plan.info()
    for _ in range(3):
        plan.run_async()
    ctx.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        plan.run_async()
    ctx.synchronize()
    dt = (time.perf_counter() - t) / reps
    st = plan.fetch()
    ctx.prof_enable(True)
    plan.run_async()
    plan.fetch()
    prof = ctx.prof_read()
    ctx.prof_enable(False)
    stages = {k: (round(v[0] * 1e3 / max(v[1], 1), 2), v[1]) for k, v in prof.items() if k.startswith("sba") and v[1]}
    print(f"{cfg}: {info} iterations {st.iterations} accepted {st.accepted} cost {st.initial_cost:.1f} -> "
          f"{st.final_cost:.1f}  run {dt * 1e3:.3f} ms  per-launch us {stages}", flush=True)
    plan.close()
ctx.close()
