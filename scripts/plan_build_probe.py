"""Device plan builds of one window, back to back (for rocprofv3 kernel / copy traces of the build):
`python scripts/plan_build_probe.py [C3|C4] [n]`."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
nk, nl, _ = synth.ba_config(cfg)
m = synth.make_ba_map(0x5EED0003, nk, nl)
o = vxslam.default_ba_options(window=nk)
ctx = vxslam.Context(0)
for _ in range(3):
    ctx.ba_plan(m, o).close()
t = time.perf_counter()
for _ in range(n):
    ctx.ba_plan(m, o).close()
print(f"{cfg}: {1e3 * (time.perf_counter() - t) / n:.3f} ms per device plan build", flush=True)
ctx.close()
