#!/usr/bin/env python3
"""Phase timestamps of the ORB kernels (trace build, csrc/vx_ktrace.hpp) on a C3 frame
(argument C4: a 1280x960 frame with 4000 features).

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so python3 scripts/ktrace_orb.py [C4]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402
from ktrace_ba import read, report  # noqa: E402


def main():
    h, w, n = (960, 1280, 4000) if sys.argv[1:] == ["C4"] else (480, 640, 2000)
    f = synth.make_frames(0x5EED0003, 1, h, w)[0]
    ctx = vxslam.Context(0)
    p = vxslam.default_orb_params(n_features=n)
    for _ in range(30):
        ctx.orb_extract(f, p)
    tr = read("vx_ktrace_read_orb")
    report(tr, [0, 1, 2, 3], "k_pyramid (1 tables + BGR staged, 2 gray level 0, 3 levels 1..L-1)")
    report(tr, [4, 5, 6, 7, 8], "k_fast (5 tiles staged, 6 FAST scores + blur row pass, 7 blur column pass + NMS + cells, 8 Harris + stores)")
    report(tr, [12, 9, 10, 11, 13, 14, 15],
           "k_select (9 histogram -> thr1, 10 first pass counts + records, 11 its scan, 13 gather done, "
           "14 radix select, 15 compaction)")
    ctx.close()


if __name__ == "__main__":
    main()
