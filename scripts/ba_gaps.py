"""LocalBA alone on one stream: per-run time with and without hipGraph replay, against the sum
of its kernels' durations (HIP events per launch) -> the inter-kernel gap cost per run."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

nk, nl = 50, 20000
for graphs in (False, True):
    c = vxslam.Context(0)
    c.graph_enable(graphs)
    plan = c.ba_plan(synth.make_ba_map(0x5EED0003, nk, nl), vxslam.default_ba_options(window=nk))
    for _ in range(5):
        plan.run_async()
    c.synchronize()
    K = 200
    t0 = time.perf_counter()
    for _ in range(K):
        plan.run_async()
    c.synchronize()
    per = (time.perf_counter() - t0) / K
    c.prof_enable(True)
    for _ in range(20):
        plan.run_async()
    c.synchronize()
    prof = c.prof_read()
    c.prof_enable(False)
    ksum = sum(v[0] for k, v in prof.items() if k.startswith("ba")) / 20
    print(f"graphs={graphs}: {1e3 * per:.4f} ms/run, sum of kernel durations {ksum:.4f} ms/run "
          f"-> gaps {1e3 * per - ksum:.4f} ms/run ({plan.fetch().iterations} iterations)", flush=True)
    plan.close()
    c.close()
