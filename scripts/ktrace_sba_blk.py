#!/usr/bin/env python3
"""Phase timestamps of the blocked Schur factor (trace build) on the connected C5 window: launch
t = nt / 8 of k_sba_fac_blk (workgroup 0: 11 slot tables, 14 B operands staged, 0-7 each wave's
look-ahead rows, 12 look-ahead tiles in LDS, 13 column 0's POTRF + inverse, 15 the block done; the
other workgroups: 7 their trailing tiles).

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so \\
        python3 scripts/ktrace_sba_blk.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(os.path.dirname(ROOT), "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402
from ktrace_ba import read  # noqa: E402


def main():
    os.environ.setdefault("VX_SBA_FACTOR", "block")  # (read per run by the plan)
    ctx = vxslam.Context(0)
    m = synth.make_ba_map(0x5EED0000 + 200, 200, 100000, n_streams=8, n_old_kf=16, cross_frac=0.03)
    plan = ctx.sba_plan(m, vxslam.default_sba_options(window=200, iters=2))
    print(plan.info())
    for _ in range(5):
        plan.run_async()
    ctx.synchronize()
    tr, cy = read("vx_ktrace_read_sba")
    b0 = tr[0]
    names = {11: "tables", 14: "B staged", 12: "look-ahead", 13: "col0 POTRF", 15: "block done"}
    print("k_sba_fac_blk workgroup 0 (us from entry):",
          " ".join(f"{names[s]} {(b0[s] - b0[10]) / 100:.2f}" for s in (11, 14, 12, 13, 15) if b0[s] > 0))
    print("  per wave, look-ahead rows done:", " ".join(f"{(b0[w] - b0[10]) / 100:.2f}" for w in range(8) if b0[w] > 0))
    rest = [b for b in range(1, tr.shape[0]) if tr[b, 10] > 0 and tr[b, 7] > 0]
    if rest:
        d = np.array([(tr[b, 7] - tr[b, 10]) / 100 for b in rest])
        st = np.array([(tr[b, 10] - b0[10]) / 100 for b in rest])
        print(f"other workgroups ({len(rest)}): trailing tiles done {np.median(d):.2f} us after entry (max {d.max():.2f});"
              f" entry {np.median(st):.2f} us after workgroup 0's (max {st.max():.2f})")
    plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
