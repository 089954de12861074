"""Schur plan rebuilt in place from the resident map N times (connected C5 by default), for a
kernel trace of the device build (vx_sba_plan_rebuild_dmap).

    rocprofv3 --kernel-trace --stats -d D -o kt -- python3 scripts/sba_rebuild_loop.py [N] [C3]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
nk, nl, ns, cf = (50, 20000, 1, 0.0) if "C3" in sys.argv[2:] else (200, 100000, 8, 0.03)
ctx = vxslam.Context(0)
m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns, cross_frac=cf)
dm = vxslam.DMap(ctx)
vxslam.dmap_load(dm, m)
p = dm.sba_plan(vxslam.default_sba_options(window=nk, iters=8))
ctx.synchronize()
t = []
for _ in range(n):
    t0 = time.perf_counter()
    dm.sba_plan_rebuild(p)
    t.append(1e3 * (time.perf_counter() - t0))
t.sort()
print(f"rebuild x{n}: median {t[len(t) // 2]:.3f} ms, min {t[0]:.3f} ms", flush=True)
p.close()
dm.close()
ctx.close()
