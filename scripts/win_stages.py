#!/usr/bin/env python3
"""k_ba_win's landmark and pose stages apart (trace variant -DVX_WIN_TRACE_LM: slot 1 + 3i = the
landmark stage of iteration i done, in place of rows ready): per iteration, over the workgroups,
solve barrier -> landmark stage done -> next pose stage done (+ its hand-off), medians / p90 / max.

    VX_LIB=visionx-slam_amd/lib/libvxslam_trace_lm.so python3 scripts/win_stages.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

KT_BLOCKS, KT_SLOTS = 256, 16
nk, nl, ns = synth.ba_config("C3")
m = synth.make_ba_map(0x5EED0003, nk, nl)
ctx = vxslam.Context(0)
plan = ctx.ba_plan(m, vxslam.default_ba_options(window=nk, iters=5))
nb = plan.layout()["workgroups"]
L, P, S = [], [], []
for rep in range(20):
    for _ in range(5):
        plan.run_async()
    ctx.synchronize()
    out = np.zeros(2 * KT_BLOCKS * KT_SLOTS, np.int64)
    assert vxslam.lib().vx_ktrace_read_ba(C.c_void_p(out.ctypes.data)) == 0
    tr = out.reshape(2, KT_BLOCKS, KT_SLOTS)[0][:nb].astype(np.float64) / 100.0
    if (tr[:, 0] <= 0).any():
        continue
    L.append(np.stack([tr[:, 1 + 3 * i] - tr[:, 2 + 3 * i] for i in range(4)], 1))
    P.append(np.stack([tr[:, 3 + 3 * i] - tr[:, 1 + 3 * i] for i in range(4)], 1))
    # solve: from the previous pose stage done (slot 15 for it 0, else 3 + 3(i - 1)) to the solve barrier
    prev = [tr[:, 15]] + [tr[:, 3 + 3 * (i - 1)] for i in range(1, 5)]
    S.append(np.stack([tr[:, 2 + 3 * i] - prev[i] for i in range(5)], 1))
for name, X in (("landmark stage", L), ("pose stage (+ barrier)", P), ("pose stage done -> solve barrier (hand-off + solve)", S)):
    A = np.median(np.stack(X), 0)
    print(f"{name:52s} median {np.median(A):6.2f}  p90 {np.percentile(A, 90):6.2f}  max {A.max():6.2f} us   per it (max): "
          + " ".join(f"{v:5.2f}" for v in A.max(0)))
plan.close()
ctx.close()
