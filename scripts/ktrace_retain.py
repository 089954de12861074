#!/usr/bin/env python3
"""Phase timestamps of the retainBest primitive (k_test_retain, trace build): load (1), team
passes (2), wave-0 passes (3), nth_element done (4), partition (5), output (6), us from the start.

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so python3 scripts/ktrace_retain.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import vxslam  # noqa: E402
from ktrace_ba import read  # noqa: E402

ctx = vxslam.Context(0)
rng = np.random.default_rng(1)
for n, npts, hi in [(64, 40, 90), (256, 200, 90), (1024, 500, 90), (1868, 868, 90), (1868, 868, 1 << 30),
                    (6800, 1800, 90)]:
    keys = (rng.integers(0, hi, n) + (20 if hi == 90 else 0)).astype(np.uint32)
    rows = []
    for _ in range(8):
        ctx.test_retain_best(keys, npts, hi > 255, True)
        tr, cy = read("vx_ktrace_read_orb")
        rows.append([(tr[0, s] - tr[0, 0]) / 100 for s in range(1, 7)] + [(cy[0, 6] - cy[0, 0]) / max(tr[0, 6] - tr[0, 0], 1) / 10])
    r = np.median(np.array(rows[2:]), 0)
    print(f"n={n:5d} npts={npts:5d} {'u64' if hi > 255 else 'u32'}: load {r[0]:6.2f} team {r[1]:6.2f} wave {r[2]:6.2f} "
          f"nth {r[3]:6.2f} part {r[4]:6.2f} end {r[5]:6.2f} us  [{r[6]:.2f} GHz]", flush=True)
ctx.close()
