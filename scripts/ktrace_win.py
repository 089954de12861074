#!/usr/bin/env python3
"""Timeline of the persistent LocalBA window k_ba_win (trace build, csrc/vx_ktrace.hpp) on the C3
window: per recorded point, median / max over the traced workgroups, launch-absolute (µs after the
earliest workgroup's start).  Slots: 0 start (loads done), 15 wave 0's prologue pose stage done;
per iteration i: 1 + 3i wave 0's rows ready, 2 + 3i the solve barrier, 3 + 3i wave 0's next pose stage done.

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so python3 scripts/ktrace_win.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

KT_BLOCKS, KT_SLOTS = 256, 16


def main():
    nk, nl, ns = synth.ba_config("C3")
    m = synth.make_ba_map(0x5EED0003, nk, nl)
    ctx = vxslam.Context(0)
    plan = ctx.ba_plan(m, vxslam.default_ba_options(window=nk, iters=5))
    print("plan", plan.info(), "persistent", plan.persistent())
    for _ in range(30):
        plan.run_async()
    ctx.synchronize()
    out = np.zeros(2 * KT_BLOCKS * KT_SLOTS, np.int64)
    assert vxslam.lib().vx_ktrace_read_ba(C.c_void_p(out.ctypes.data)) == 0
    tr = out.reshape(2, KT_BLOCKS, KT_SLOTS)[0]
    ok = tr[:, 0] > 0
    t0 = tr[ok, 0].min()
    names = {0: "start", 15: "prologue pose stage (wave 0)"}
    for i in range(5):
        names[1 + 3 * i] = f"it {i}: rows ready (wave 0)"
        names[2 + 3 * i] = f"it {i}: solve barrier"
        if i < 4:
            names[3 + 3 * i] = f"it {i}: pose stage {i + 1} done (wave 0)"
    print(f"{int(ok.sum())} workgroups traced")
    for s in [0, 15] + list(range(1, 15)):
        v = tr[ok, s]
        if (v > 0).sum() == 0:
            continue
        d = (v[v > 0] - t0) / 100.0
        print(f"  slot {s:2d} {names.get(s, ''):40s} median {np.median(d):7.2f}  min {d.min():7.2f}  max {d.max():7.2f} us")


if __name__ == "__main__":
    main()
