#!/usr/bin/env python3
"""Phase timestamps of the multi-workgroup Schur factor (trace build) on the connected C5 window:
launch k = nt / 2 of k_sba_fac_step (workgroup 0: 1 flags read, 2 slot map, 3 look-ahead update
issued, 4 after its barrier, 5 POTRF + inverse, 6 panel; the other workgroups: 7 their trailing
tiles) and k_sba_backsub (8 start, 9 back-substitution done).

    make -C visionx-slam_amd trace && VX_SBA_FACTOR_COLS=1 VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so \\
        python3 scripts/ktrace_sba_multi.py
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
    ctx = vxslam.Context(0)
    m = synth.make_ba_map(0x5EED0000 + 200, 200, 100000, n_streams=8, n_old_kf=16, cross_frac=0.03)
    plan = ctx.sba_plan(m, vxslam.default_sba_options(window=200, iters=2))
    print(plan.info())
    for _ in range(5):
        plan.run_async()
    ctx.synchronize()
    tr, cy = read("vx_ktrace_read_sba")
    b0 = tr[0]
    print("k_sba_fac_step workgroup 0 (us from entry):",
          " ".join(f"{s}:{(b0[s] - b0[0]) / 100:.2f}" for s in range(1, 7) if b0[s] > 0))
    rest = [b for b in range(1, tr.shape[0]) if tr[b, 0] > 0 and tr[b, 7] > 0]
    if rest:
        d = np.array([(tr[b, 7] - tr[b, 0]) / 100 for b in rest])
        st = np.array([(tr[b, 0] - b0[0]) / 100 for b in rest])
        print(f"other workgroups ({len(rest)}): trailing tiles done {np.median(d):.2f} us after entry (max {d.max():.2f});"
              f" entry {np.median(st):.2f} us after workgroup 0's (max {st.max():.2f})")
    print(f"k_sba_backsub: back-substitution {(b0[9] - b0[8]) / 100:.2f} us")
    plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
