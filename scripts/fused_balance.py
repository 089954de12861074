"""Pose-stage balance of the fused LocalBA layout: per workgroup the rounds (64 observations) of each
wave, the most loaded SIMD (waves w and w + 4 share one at 512 threads), and the LPT bound
ceil(total / 4).  `python scripts/fused_balance.py [n_kf n_lm n_streams]`."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

nk, nl, ns = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (50, 20000, 1)
ctx = vxslam.Context(0)
m = synth.make_ba_map(0x5EED0003, nk, nl, n_streams=ns, n_old_kf=2 * ns)
p = ctx.ba_plan(m, vxslam.default_ba_options(window=nk))
lay = p.layout()
nb, ft = lay["workgroups"], lay["threads"]
fw = ft // 64
bi = 4 * (1 + fw // 2)
tab = np.frombuffer(p.fused_tables(), np.int32)
blk = tab[: nb * bi].reshape(nb, bi)
rounds = blk[:, 5::2][:, :fw]  # per wave
n_ent = blk[:, 2]
simd = rounds.reshape(nb, -1, 4).sum(1) if fw >= 4 else rounds
tot = rounds.sum(1)
print(f"{nk} KF / {nl} LM: {nb} workgroups x {ft}; entries/wg median {np.median(n_ent):.0f} max {n_ent.max()}")
print(f"rounds/wg median {np.median(tot):.0f} max {tot.max()}; max wave rounds median {np.median(rounds.max(1)):.0f} "
      f"max {rounds.max()}; busiest SIMD median {np.median(simd.max(1)):.0f} max {simd.max()}; "
      f"LPT bound ceil(total/4) median {np.median(np.ceil(tot / 4)):.0f} max {np.ceil(tot / 4).max():.0f}")
worst = np.argsort(-simd.max(1))[:5]
for b in worst:
    print(f"  wg {b}: entries {n_ent[b]}, wave rounds {list(rounds[b])}, SIMD rounds {list(simd[b])}")
p.close()
ctx.close()
