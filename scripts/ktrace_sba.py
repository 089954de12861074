#!/usr/bin/env python3
"""Phase timestamps of k_sba_solve (trace build) on the C2 / C3 windows.

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so python3 scripts/ktrace_sba.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(os.path.dirname(ROOT), "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402
from ktrace_ba import read, report  # noqa: E402


def main():
    ctx = vxslam.Context(0)
    for cfg in ("C2", "C3"):
        nk, nl, ns = synth.ba_config(cfg)
        m = synth.make_ba_map(0x5EED0000 + nk, nk, nl)
        plan = ctx.sba_plan(m, vxslam.default_sba_options(window=nk, iters=2))
        print(cfg, plan.info())
        for _ in range(20):
            plan.run_async()
        ctx.synchronize()
        report(read("vx_ktrace_read_sba"), [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12],
               "k_sba_solve (1 copy | 2,3,4 step 0 factor/panel/trail | 5,6,7 step 1 | 8,9,10 step nt/2 | 11 factor done | 12 back-sub)")
        plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
