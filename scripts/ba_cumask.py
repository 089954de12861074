"""LocalBA (C3) alone under different CU masks: does keeping it on one XCD's CUs (one L2) help?"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

ncu = vxslam.lib().vx_device_cus(0)
m = synth.make_ba_map(0x5EED0003, 50, 20000)
masks = {"all": None, "first32": range(32), "first64": range(64), "first128": range(128),
         "every8th": range(0, ncu, 8), "every4th": range(0, ncu, 4), "last32": range(ncu - 32, ncu),
         "32 stride1 from 1": range(1, 33)}
for name, mk in masks.items():
    c = vxslam.Context(0, cu_mask=mk)
    plan = c.ba_plan(m, vxslam.default_ba_options(window=50))
    for _ in range(5):
        plan.run_async()
    c.synchronize()
    K = 200
    t0 = time.perf_counter()
    for _ in range(K):
        plan.run_async()
    c.synchronize()
    print(f"{name:18s} {1e3 * (time.perf_counter() - t0) / K:.4f} ms/run", flush=True)
    plan.close()
    c.close()
