#!/usr/bin/env python3
"""Per-pass timeline of k_select_stl's level 0 (trace build, VX_KP pass log) for a C3 frame, and of
the bare retainBest primitive per size: each introselect / partition pass with its range and kind
(mem / team / wave pivot passes, the partition), us since the previous entry.

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so python3 scripts/kpass_select.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

KIND = {0: "mem", 1: "team", 2: "wave", 3: "nth-done/part", 4: "part-done", 5: "tail64", 6: "tail128", 7: "tail256"}


def read():
    buf = np.zeros(1024, np.int64)
    assert vxslam.lib().vx_kpass_read_orb(buf.ctypes.data_as(C.c_void_p)) == 0
    n = int(buf[0])
    return [(int(buf[2 * i]), int(buf[2 * i + 1])) for i in range(1, n + 1)]


def show(title, log):
    print(title)
    for i, (t, tag) in enumerate(log):
        dt = (log[i + 1][0] - t) / 100 if i + 1 < len(log) else 0.0
        print(f"  {KIND.get(tag >> 24, '?'):14s} len {tag & 0xffffff:6d}  {dt:6.2f} us")


ctx = vxslam.Context(0)
f = synth.make_frames(0x5EED0003, 1, 480, 640)[0]
p = vxslam.default_orb_params(n_features=2000)
for _ in range(10):
    ctx.orb_extract(f, p)
show("k_select_stl level 0, C3 frame", read())
rng = np.random.default_rng(1)
for n, npts, hi in [(64, 40, 90), (1868, 868, 90), (868, 434, 1 << 30)]:
    keys = (rng.integers(0, hi, n) + (20 if hi == 90 else 0)).astype(np.uint32)
    for _ in range(5):
        ctx.test_retain_best(keys, npts, hi > 255, True)
    show(f"retainBest n={n} npts={npts} {'u64' if hi > 255 else 'u32'}", read())
ctx.close()
