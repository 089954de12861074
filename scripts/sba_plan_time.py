"""Schur-complement BA plan build: host build from the snapshot (vx_sba_plan_create) against the
device build from the resident map (vx_sba_plan_create_dmap; create + close per build, so each
build allocates and releases the plan's buffers), the same plan rebuilt in place
(vx_sba_plan_rebuild_dmap: buffers reused, the drop-in's per-Optimize cost), and one run of the
plan; median ms of 5 after one warm-up, at C3 and the connected C5 rig.

    python scripts/sba_plan_time.py [out.json]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import numpy as np  # noqa: E402

import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402


def med(f, n=5):
    f()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        t.append(1e3 * (time.perf_counter() - t0))
    return round(float(np.median(t)), 3)


out = {}
ctx = vxslam.Context(0)
for name, (nk, nl, ns, cf) in {"C3": (50, 20000, 1, 0.0), "C5-connected": (200, 100000, 8, 0.03)}.items():
    m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns, cross_frac=cf)
    opts = vxslam.default_sba_options(window=nk, iters=8)
    dm = vxslam.DMap(ctx)
    vxslam.dmap_load(dm, m)
    ctx.synchronize()

    def host():
        ctx.sba_plan(m, opts).close()

    def dev():
        dm.sba_plan(opts).close()

    p = dm.sba_plan(opts)
    info = p.info()

    def rebuild():
        dm.sba_plan_rebuild(p)

    def run():
        p.run_async()
        p.fetch()

    r = {"plan_host_ms": med(host), "plan_device_ms": med(dev), "plan_device_rebuild_ms": med(rebuild),
         "run_ms": med(run), "info": info}
    p.run_async()
    st = p.fetch()
    r["iterations"], r["accepted"] = int(st.iterations), int(st.accepted)
    p.close()
    dm.close()
    out[name] = r
    print(name, r, flush=True)
ctx.close()
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
