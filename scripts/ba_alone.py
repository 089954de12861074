"""LocalBA alone (one context, graph replay): ms per run of one window under the current
environment (VX_BA_FUSED, VX_BA_FUSED_THREADS, VX_BA_FUSED_CAP are read at plan build).

    python scripts/ba_alone.py [n_kf n_lm n_streams]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

nk, nl, ns = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (50, 20000, 1)
c = vxslam.Context(0)
m = synth.make_ba_map(0x5EED0003, nk, nl, n_streams=ns, n_old_kf=2 * ns)
plan = c.ba_plan(m, vxslam.default_ba_options(window=nk), host_build=os.environ.get("BA_HOST_BUILD") == "1")
for _ in range(5):
    plan.run_async()
c.synchronize()
best = 1e9
for rep in range(3):
    K = 100
    t0 = time.perf_counter()
    for _ in range(K):
        plan.run_async()
    c.synchronize()
    best = min(best, 1e3 * (time.perf_counter() - t0) / K)
print(f"{nk} KF {nl} LM env {[k + '=' + v for k, v in os.environ.items() if k.startswith('VX_BA')]}: "
      f"{best:.4f} ms/run  plan {plan.info()} layout {plan.layout()}", flush=True)
plan.close()
c.close()
