#!/usr/bin/env python3
"""One vx_test_retain_best call per size (for rocprofv3 --pmc): n = 64, 256, 1868 (u32 keys)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402

ctx = vxslam.Context(0)
rng = np.random.default_rng(1)
for n, npts in [(64, 40), (256, 200), (1868, 868)]:
    keys = (rng.integers(0, 90, n) + 20).astype(np.uint32)
    for _ in range(3):
        ctx.test_retain_best(keys, npts, False, True)
ctx.close()
