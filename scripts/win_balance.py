#!/usr/bin/env python3
"""Where the persistent window's per-iteration time goes, workgroup by workgroup (trace build): the
landmark + pose stage duration of each workgroup (solve barrier -> its pose stage done, slots 2+3i ->
3+3i of csrc/vx_ktrace.hpp) against its layout (pose-stage rounds of its busiest wave / SIMD, entries,
landmark-stage observations), and when each iteration's last row arrives.

    make -C visionx-slam_amd trace && VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so python3 scripts/win_balance.py"""
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
lay = plan.layout()
nb, ft = lay["workgroups"], lay["threads"]
fw = ft // 64
bi = 4 * (1 + fw // 2)
tab = np.frombuffer(plan.fused_tables(), np.int32)
blk = tab[: nb * bi].reshape(nb, bi)
rounds = blk[:, 5::2][:, :fw]
simd = rounds.reshape(nb, -1, 4).sum(1) if fw >= 4 else rounds
n_lm, n_ob, n_ent = blk[:, 0], blk[:, 1], blk[:, 2]
print("plan", plan.info(), "persistent", plan.persistent(), f"{nb} workgroups x {ft}")
durs = []
for rep in range(20):
    for _ in range(5):
        plan.run_async()
    ctx.synchronize()
    out = np.zeros(2 * KT_BLOCKS * KT_SLOTS, np.int64)
    assert vxslam.lib().vx_ktrace_read_ba(C.c_void_p(out.ctypes.data)) == 0
    tr = out.reshape(2, KT_BLOCKS, KT_SLOTS)[0][:nb]
    if (tr[:, 0] <= 0).any():
        continue
    d = np.stack([tr[:, 3 + 3 * i] - tr[:, 2 + 3 * i] for i in range(4)], 1) / 100.0  # us
    lastrow = np.array([(tr[:, 1 + 3 * (i + 1)] - tr[:, 2 + 3 * i]).max() for i in range(4)]) / 100.0
    durs.append((d, lastrow, tr))
D = np.median(np.stack([x[0] for x in durs]), 0)  # [nb, 4]
Dm = D.mean(1)
print(f"{len(durs)} traced runs; landmark + pose stage per workgroup: median {np.median(Dm):.2f} us, "
      f"p90 {np.percentile(Dm, 90):.2f}, max {Dm.max():.2f}")
mw = rounds.max(1)
for r in sorted(set(mw.tolist())):
    sel = mw == r
    print(f"  busiest wave {r} rounds: {sel.sum():4d} workgroups, stage median {np.median(Dm[sel]):.2f} max {Dm[sel].max():.2f} us")
ms = simd.max(1)
for r in sorted(set(ms.tolist())):
    sel = ms == r
    print(f"  busiest SIMD {r} rounds: {sel.sum():4d} workgroups, stage median {np.median(Dm[sel]):.2f} max {Dm[sel].max():.2f} us")
worst = np.argsort(-Dm)[:8]
for b in worst:
    print(f"  wg {b:3d}: stage {Dm[b]:.2f} us  lm {n_lm[b]} obs {n_ob[b]} entries {n_ent[b]} wave rounds {rounds[b].tolist()}")
print("corr(stage, busiest wave rounds) %.2f, (stage, total rounds) %.2f, (stage, obs) %.2f" % (
    np.corrcoef(Dm, mw)[0, 1], np.corrcoef(Dm, rounds.sum(1))[0, 1], np.corrcoef(Dm, n_ob)[0, 1]))
lr = np.median(np.stack([x[1] for x in durs]), 0)
print("solve barrier -> last workgroup's rows ready, per iteration (max over workgroups):", np.round(lr, 2).tolist())
plan.close()
ctx.close()
