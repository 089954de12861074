"""bench.py's per_keyframe_ms legs alone (snapshot plan, resident plan + apply, one-call resident) on
the C3 window, printing after each leg — a probe for tool runs (rocprofv3 --pmc) of those paths."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

ctx = vxslam.Context(0)
nk, nl, ns = synth.ba_config("C3")
m0 = synth.make_ba_map(0x5EED0003, nk, nl)
opts = vxslam.default_ba_options(window=nk)
m = m0.copy()
for i in range(9):
    p = ctx.ba_plan(m, opts)
    p.run_async()
    p.fetch(m)
    p.close()
print("snapshot ok", flush=True)
dm = vxslam.DMap(ctx)
vxslam.dmap_load(dm, m0)
ctx.synchronize()
for i in range(9):
    p = dm.plan(opts)
    p.run_async()
    p.apply(dm)
    ctx.synchronize()
    p.close()
    print("resident", i, flush=True)
for i in range(9):
    dm.optimize(opts)
    print("one_call", i, flush=True)
dm.close()
print("done", flush=True)
