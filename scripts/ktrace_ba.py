#!/usr/bin/env python3
"""Phase timestamps of the BA kernels (trace build, csrc/vx_ktrace.hpp) on the C3 window.

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so python3 scripts/ktrace_ba.py

Runs one iteration (max_iterations = 1) many times; after the last run prints, per recorded slot,
the median / max over the first 64 workgroups of (slot - that workgroup's first slot) in µs, and
the spread of the first slot over workgroups (dispatch ramp).
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

KT_BLOCKS, KT_SLOTS = 256, 16


def read(fn="vx_ktrace_read_ba"):
    """(wall_clock64 table, s_memtime table), each [block][slot]"""
    out = np.zeros(2 * KT_BLOCKS * KT_SLOTS, np.int64)
    assert getattr(vxslam.lib(), fn)(C.c_void_p(out.ctypes.data)) == 0
    return out.reshape(2, KT_BLOCKS, KT_SLOTS)


def report(tr2, slots, name):
    tr, cy = tr2
    base = tr[:, slots[0]]
    ok = base > 0
    print(f"{name}: {int(ok.sum())} workgroups traced, start spread {(base[ok].max() - base[ok].min()) / 100:.2f} us")
    for s in slots[1:]:
        d = (tr[ok, s] - base[ok]) / 100.0  # 100 MHz ticks -> us
        c = (cy[ok, s] - cy[ok, slots[0]])
        clk = np.median(c / np.maximum(d, 1e-3)) / 1e3  # cycles per us -> GHz
        print(f"  slot {s:2d}: median {np.median(d):7.2f} us  max {d.max():7.2f} us  ({np.median(c):8.0f} cycles, {clk:.2f} GHz)")


def main():
    if os.environ.get("KT_LOAD"):  # (torch's HIP initialisation must come before the library's)
        import torch

        torch.zeros(1, device="cuda")
    nk, nl, ns = synth.ba_config("C3")
    m = synth.make_ba_map(0x5EED0003, nk, nl)
    # KT_MASK=f (with KT_LOAD): LocalBA on a disjoint CU mask of that fraction of the CUs (every 3rd CU
    # to the extraction contexts for f = 2/3, as bench.py --ba-cus does)
    frac = float(os.environ.get("KT_MASK", "0"))
    ba_mask = ex_mask = None
    if frac > 0:
        ncu = vxslam.lib().vx_device_cus(0)
        small = min(frac, 1.0 - frac)
        k = max(2, int(round(1.0 / small)))
        few = [i for i in range(ncu) if i % k == k - 1]
        rest = [i for i in range(ncu) if i % k != k - 1]
        ba_mask, ex_mask = (few, rest) if frac <= 0.5 else (rest, few)
    ctx = vxslam.Context(0, cu_mask=ba_mask)
    # fused path (default): the traced launch is k_ba_iter(it = 1) of a 5-iteration run
    plan = ctx.ba_plan(m, vxslam.default_ba_options(window=nk, iters=5))
    print("plan", plan.info())
    # KT_LOAD=extract: the traced runs beside ORB extraction on two other contexts (grid share 1/3,
    # frames alternate), as in bench.py's pipeline — which phases the interference stretches
    load = os.environ.get("KT_LOAD", "")
    if load == "extract":
        import torch

        ex = [vxslam.Context(0, cu_mask=ex_mask), vxslam.Context(0, cu_mask=ex_mask)]
        for c in ex:
            c.set_grid_share(1.0 / 3.0)
        frames = torch.from_numpy(synth.make_frames(7, 8, 480, 640)).cuda()
        params = vxslam.default_orb_params(n_features=2000)
        torch.cuda.synchronize()
    for i in range(30):
        if load == "extract":
            for j in range(4):  # (twice the extraction work of a LocalBA run: the runs stay loaded)
                ex[j % 2].orb_extract_async(frames[(4 * i + j) % 8].data_ptr(), 640, 480, 3, 640 * 3, (i + j // 2) % 3, params)
        plan.run_async()
    ctx.synchronize()
    if load == "extract":
        for c in ex:
            c.synchronize()
    tr2 = read()
    report(tr2, [0, 1, 2, 3, 4, 6, 7, 5],
           "k_ba_iter (1 loads, 2 combine + totals + barrier, 3 pose solve + barrier, 4 landmark stage + barrier, "
           "6 pose-stage entry, 7 its rounds, 5 pose stage of it + 1 done)")
    # the slowest workgroups (and workgroup 0, which also runs the stop rule's totals): phase deltas
    tr = tr2[0]
    ok = tr[:, 0] > 0
    d = (tr[:, [1, 2, 3, 4, 5]] - tr[:, [0, 1, 2, 3, 4]]) / 100.0
    end = (tr[:, 5] - tr[:, 0]) / 100.0
    order = [b for b in np.argsort(-end) if ok[b]][:6]
    if 0 not in order and ok[0]:
        order.append(0)
    # per wave: end of its pose stage (slots 8..15) after the landmark stage's barrier (slot 4), beside
    # the wave's rounds from the layout
    lay = plan.layout()
    fw = lay["threads"] // 64
    bi = 4 * (1 + fw // 2)
    blk = np.frombuffer(plan.fused_tables(), np.int32)[: lay["workgroups"] * bi].reshape(-1, bi)
    print("  per-wave pose stage done after slot 4 (us) [rounds]:")
    for b in list(range(4)):
        if ok[b]:
            w = (tr[b, 8:8 + min(fw, 8)] - tr[b, 4]) / 100.0
            print(f"    wg {b}: " + "  ".join(f"{x:5.2f}[{blk[b, 5 + 2 * i]}]" for i, x in enumerate(w)))
    print("  slowest workgroups: wg  loads combine solve landmark pose-stage  total (us)")
    for b in order:
        print(f"    {b:3d}  " + "  ".join(f"{x:6.2f}" for x in d[b]) + f"  {end[b]:6.2f}")
    # launch-absolute view over every traced workgroup (one launch: the last run's it = 1): which
    # workgroups end last, and whether because they started late or ran long
    t0 = tr[ok, 0].min()
    st = (tr[:, 0] - t0) / 100.0
    en = (tr[:, 5] - t0) / 100.0
    nb = int(ok.sum())
    print(f"  launch view ({nb} workgroups): start spread {st[ok].max():.2f} us, end median {np.median(en[ok]):.2f} "
          f"max {en[ok].max():.2f} us; latest-ending (wg start +loads +combine +solve +landmark +pose = end, "
          f"pose-stage rounds per wave):")
    for b in [b for b in np.argsort(-en) if ok[b]][:8]:
        rounds = [int(blk[b, 5 + 2 * i]) for i in range(min(fw, 8))] if b < len(blk) else []
        print(f"    {b:3d}  {st[b]:5.2f} " + " ".join(f"{x:5.2f}" for x in d[b]) + f" = {en[b]:5.2f}  {rounds}")
    plan.close()
    # the two-kernel path (sharded plans, windows the fused layout does not fit)
    os.environ["VX_BA_FUSED"] = "0"
    plan = ctx.ba_plan(m, vxslam.default_ba_options(window=nk, iters=1))
    print("plan", plan.info())
    for _ in range(30):
        plan.run_async()
    ctx.synchronize()
    tr = read()
    report(tr, [0, 1, 2, 3, 4, 5], "k_pose_kf (1 loads T/C, 2 obs loop, 3 wave reduce, 4 LDS+barrier, 5 store)")
    report(tr, [8, 9, 10, 11, 13, 12],
           "k_landmark_solve (9 loads, 10 combine, 11 pose solve, 13 observation terms, 12 per-landmark sum + 3x3 + store)")
    plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
