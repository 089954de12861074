#!/usr/bin/env python3
"""Phase timestamps of k_select_stl per pyramid level (trace build, csrc/vx_ktrace.hpp):
gather (9), retainBest(2q) by FAST score (10), Harris key build (11), retainBest(q) (13), output (15).

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so python3 scripts/ktrace_select.py [C4]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402
from ktrace_ba import read  # noqa: E402


def main():
    h, w, n = (960, 1280, 4000) if sys.argv[1:] == ["C4"] else (480, 640, 2000)
    f = synth.make_frames(0x5EED0003, 1, h, w)[0]
    ctx = vxslam.Context(0)
    p = vxslam.default_orb_params(n_features=n)
    for _ in range(30):
        ctx.orb_extract(f, p)
    tr, cy = read("vx_ktrace_read_orb")
    names = [(9, "gather"), (10, "retain(2q)"), (11, "harris keys"), (13, "retain(q)"), (15, "output")]
    print(f"k_select_stl {w}x{h} n={n}: per level, us since the workgroup start (phase length)")
    for l in range(8):
        t0 = tr[l, 12]
        prev, row = t0, []
        for s, nm in names:
            t = tr[l, s]
            row.append(f"{nm} {(t - t0) / 100:6.2f} ({(t - prev) / 100:5.2f})")
            prev = t
        ghz = (cy[l, 15] - cy[l, 12]) / max((tr[l, 15] - tr[l, 12]) / 100.0, 1e-3) / 1e3
        print(f"  L{l}: " + "  ".join(row) + f"  [{ghz:.2f} GHz]")
    ctx.close()


if __name__ == "__main__":
    main()
