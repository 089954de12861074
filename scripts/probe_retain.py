#!/usr/bin/env python3
"""Kernel time of the device retainBest primitive (vx_test_retain_best -> k_test_retain) per input
size and key spread; run under rocprofv3 --kernel-trace --stats (one launch per call, in order)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402

ctx = vxslam.Context(0)
rng = np.random.default_rng(1)
for n, npts, hi in [(64, 40, 90), (256, 200, 90), (307, 244, 90), (1024, 500, 90), (1868, 868, 90),
                    (1868, 868, 1 << 30)]:
    keys = (rng.integers(0, hi, n) + (20 if hi == 90 else 0)).astype(np.uint32)
    wide = hi > 255
    for _ in range(20):
        ctx.test_retain_best(keys, npts, wide, True)
    print(n, npts, hi, flush=True)
ctx.close()
