"""Time of vx_ba_plan_create (window selection + landmark set + CSRs + upload): device build vs
the host reference build, C2 / C3 / C4."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

ctx = vxslam.Context(0)
for cfg in ("C2", "C3", "C4"):
    nk, nl, ns = synth.ba_config(cfg)
    m = synth.make_ba_map(0x5EED0003, nk, nl)
    o = vxslam.default_ba_options(window=nk)
    res = {}
    for hb in (False, True):
        for _ in range(2):
            ctx.ba_plan(m, o, host_build=hb).close()
        t = time.perf_counter()
        for _ in range(10):
            ctx.ba_plan(m, o, host_build=hb).close()
        res["host" if hb else "device"] = 1e3 * (time.perf_counter() - t) / 10
    print(f"{cfg}: plan build device {res['device']:.3f} ms, host {res['host']:.3f} ms", flush=True)
ctx.close()
