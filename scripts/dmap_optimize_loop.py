"""The drop-in LocalBA::Optimize on the resident map (vx_ba_optimize_dmap, one call: lean build, five
iterations, scatter, one synchronisation) repeated on the C3 window, for a rocprofv3 kernel trace of
that path.  Prints the median host ms per call.

    rocprofv3 --kernel-trace --stats -d D -o run -- python3 scripts/dmap_optimize_loop.py [calls]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = vxslam.Context(0)
m = synth.make_ba_map(0x5EED0003, 50, 20000)
dm = vxslam.DMap(ctx)
vxslam.dmap_load(dm, m)
opts = vxslam.default_ba_options(window=50)
ms = []
for i in range(n + 5):
    t0 = time.perf_counter()
    st = dm.optimize(opts, ref_kf_id=m.get("ref_kf_id"))
    if i >= 5:
        ms.append(1e3 * (time.perf_counter() - t0))
print(f"vx_ba_optimize_dmap C3: median {np.median(ms):.4f} ms over {n} calls "
      f"(status {st.status}, iterations {st.iterations}, landmarks {st.n_landmarks})", flush=True)
dm.close()
ctx.close()
