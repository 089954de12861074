"""Fused vs two-kernel LocalBA against the restatement: per config, per iteration observation counts
and the largest relative pose / landmark error of each path (diagnostic for DESIGN.md §7)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "visionx-slam_amd", "python"), os.path.join(ROOT, "oracle")]
import torch  # noqa: F401,E402  (loads torch's HIP runtime first, tests/conftest.py)
import pyoracle as O  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402


def canon(p):
    p = p.copy()
    neg = p[:, 3] < 0
    p[neg, :4] *= -1
    return p


ctx = vxslam.Context(0)
for cfg in sys.argv[1:] or ["C2", "C3", "C4", "C5"]:
    iters = 5
    if ":" in cfg:  # nk:nl[:iters]
        v = [int(x) for x in cfg.split(":")]
        nk, nl, ns = v[0], v[1], 1
        iters = v[2] if len(v) > 2 else 5
    else:
        nk, nl, ns = synth.ba_config(cfg)
    m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=ns * 2)
    mc = m.copy()
    sc = O.ba_optimize(mc, O.ba_options(window=nk, iters=iters))
    print(cfg, "oracle", list(sc.obs[:sc.iterations]), "margin", sc.gate_margin)
    for fused in ("1", "0"):
        os.environ["VX_BA_FUSED"] = fused
        mg = m.copy()
        plan = ctx.ba_plan(mg, vxslam.default_ba_options(window=nk, iters=iters))
        plan.run_async()
        st = plan.fetch(mg)
        plan.close()
        ep = np.abs(canon(mg["kf_pose"]) - canon(mc["kf_pose"])) / np.maximum(np.abs(canon(mc["kf_pose"])), 1e-3)
        el = np.abs(mg["lm_pos"] - mc["lm_pos"]) / np.maximum(np.abs(mc["lm_pos"]), 1e-3)
        print(f"  fused={fused} obs {list(st.obs[:st.iterations])} pose err {ep.max():.3e} lm err {el.max():.3e} "
              f"cost rel {[abs(a - b) / b for a, b in zip(st.cost[:st.iterations], sc.cost[:sc.iterations])]}")
ctx.close()
