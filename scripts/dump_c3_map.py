#!/usr/bin/env python3
"""Write the C3 window's map (scripts/adapter_timing.py's synthetic map) as the .bin files
tests/cpp/adapter_driver reads, into <dir> (for profiling the driver directly under rocprofv3).

    python3 scripts/dump_c3_map.py <dir>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
from vxslam import synth  # noqa: E402

d = sys.argv[1]
os.makedirs(d, exist_ok=True)
m = synth.make_ba_map(0x5EED0003, 50, 20000, n_streams=1, n_old_kf=2)
for k in ["kf_id", "kf_pose", "kf_intr", "kf_has_cam", "kf_feat_ptr", "feat_uv", "feat_lm_id", "feat_flags",
          "lm_id", "lm_pos", "lm_bad", "lm_obs_ptr", "obs_kf_id", "obs_feat_idx"]:
    np.ascontiguousarray(m[k]).tofile(os.path.join(d, k + ".bin"))
