"""A/B of the C++ drop-in's LocalBA::Optimize (both modes, no timing switches) on the C3 window:
alternates an environment variable unset / set over several rounds in fresh processes, so that box
noise falls on both arms alike.

    python scripts/adapter_ab.py VAR [rounds] [reps] [value (default 1)]"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
from vxslam import synth  # noqa: E402

var = sys.argv[1]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
val = sys.argv[4] if len(sys.argv) > 4 else "1"
m = synth.make_ba_map(0x5EED0003, 50, 20000, n_streams=1, n_old_kf=2)
keys = ["kf_id", "kf_pose", "kf_intr", "kf_has_cam", "kf_feat_ptr", "feat_uv", "feat_lm_id", "feat_flags",
        "lm_id", "lm_pos", "lm_bad", "lm_obs_ptr", "obs_kf_id", "obs_feat_idx"]
drv = os.path.join(ROOT, "visionx-slam_amd", "build", "adapter_driver")
res = {}
with tempfile.TemporaryDirectory() as d:
    for k in keys:
        np.ascontiguousarray(m[k]).tofile(os.path.join(d, k + ".bin"))
    for r in range(rounds):
        for arm in ("unset", val):
            env = dict(os.environ)
            env.pop(var, None)
            if arm != "unset":
                env[var] = arm
            for mode in ("snapshot", "resident"):
                out = subprocess.run([drv, "ba_calls", d, "50", "5", "-1", str(reps), mode], capture_output=True,
                                     text=True, timeout=300, env=env)
                if out.returncode:
                    print(out.stderr[-800:])
                    sys.exit(1)
                ms = float(out.stdout.split()[-1])
                res.setdefault((mode, arm), []).append(ms)
                print(f"round {r} {var}={arm} {mode}: {ms:.4f} ms", flush=True)
for (mode, arm), v in sorted(res.items()):
    print(f"{mode:9s} {var}={arm:5s} median {np.median(v):.4f} ms  all {' '.join(f'{x:.3f}' for x in v)}")
