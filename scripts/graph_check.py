"""Host cost of one LocalBA plan replay (vx_ba_plan_run_async) and whether it is a graph replay:
the context's graph counters before / after 200 replays of the C3 plan."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

c = vxslam.Context(0)
m = synth.make_ba_map(0x5EED0003, 50, 20000)
plan = c.ba_plan(m, vxslam.default_ba_options(window=50))
for _ in range(5):
    plan.run_async()
c.synchronize()
print("after warm-up: captured / launched", c.graph_counts(), "layout", plan.layout(), flush=True)
K = 200
t = 0.0
for _ in range(K):
    t0 = time.perf_counter()
    plan.run_async()
    t += time.perf_counter() - t0
    c.synchronize()
print(f"run_async host {1e6 * t / K:.2f} us per call; captured / launched {c.graph_counts()}", flush=True)
plan.close()
c.close()
