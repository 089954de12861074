"""The C++ drop-in's per-call phases on the C3 window (resident mode: Flush, vx_ba_optimize_dmap,
results, write-back; $VX_RESIDENT_TIMING laps of visionx::LocalBA::OptimizeResident; snapshot mode:
Flatten's phases ($VX_FLATTEN_TIMING), vx_ba_optimize_map's ($VX_OPT_TIMING), write-back) and the
median call times of both modes through tests/cpp/adapter_driver ba_calls.

    python scripts/adapter_timing.py [reps]"""
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
from vxslam import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
m = synth.make_ba_map(0x5EED0003, 50, 20000, n_streams=1, n_old_kf=2)
keys = ["kf_id", "kf_pose", "kf_intr", "kf_has_cam", "kf_feat_ptr", "feat_uv", "feat_lm_id", "feat_flags",
        "lm_id", "lm_pos", "lm_bad", "lm_obs_ptr", "obs_kf_id", "obs_feat_idx"]
drv = os.path.join(ROOT, "visionx-slam_amd", "build", "adapter_driver")
with tempfile.TemporaryDirectory() as d:
    for k in keys:
        np.ascontiguousarray(m[k]).tofile(os.path.join(d, k + ".bin"))
    for mode in ("resident", "snapshot"):
        env = dict(os.environ, VX_RESIDENT_TIMING="1", VX_FLATTEN_TIMING="1", VX_OPT_TIMING="1", VX_PLAN_TIMING="1")
        r = subprocess.run([drv, "ba_calls", d, "50", "5", "-1", str(reps), mode], capture_output=True, text=True,
                           timeout=300, env=env)
        print(mode, "rc", r.returncode, "stdout", r.stdout.strip())
        laps = {}
        for line in r.stderr.splitlines():
            if line.startswith(("[vx resident]", "[vx snapshot]", "[vx optmap]")):
                parts = line.split()
                laps.setdefault(parts[1] + " " + parts[2], []).append(float(parts[3]))
            elif line.startswith("[vx plan]"):
                mt = re.match(r"\[vx plan\] (.+?)\s+([\d.]+) ms", line)
                if mt:
                    laps.setdefault("plan " + mt.group(1), []).append(1e3 * float(mt.group(2)))
            elif line.startswith("[flatten]"):
                parts = line.split()
                laps.setdefault("flatten " + parts[1], []).append(1e3 * float(parts[2]))
        for k, v in laps.items():
            print(f"  {k}: median {np.median(v[1:] or v):.1f} us since the call's start")
        if r.returncode:
            print(r.stderr[-800:])
    # the same calls without any timing switch (the laps above add synchronisations of their own)
    for mode in ("resident", "snapshot"):
        r = subprocess.run([drv, "ba_calls", d, "50", "5", "-1", str(reps), mode], capture_output=True, text=True,
                           timeout=300)
        print("untimed", mode, "rc", r.returncode, "stdout", r.stdout.strip())
