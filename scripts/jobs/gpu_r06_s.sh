#!/bin/bash
# round 6 (s): host threads 16 vs 8 for the drop-in; kernel trace of the resident call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06s}
mkdir -p $O
timeout -k 10 400 python3 -u scripts/adapter_ab.py VX_HOST_THREADS 6 100 16 > $O/ab_threads16.txt 2>&1 || { tail -30 $O/ab_threads16.txt; exit 2; }
tail -4 $O/ab_threads16.txt
timeout -k 10 400 python3 -u scripts/adapter_ab.py VX_HOST_THREADS 6 100 4 > $O/ab_threads4.txt 2>&1 || { tail -30 $O/ab_threads4.txt; exit 3; }
tail -4 $O/ab_threads4.txt
python3 - <<'PY' || exit 4
import os, sys, numpy as np
sys.path.insert(0, "visionx-slam_amd/python")
from vxslam import synth
m = synth.make_ba_map(0x5EED0003, 50, 20000, n_streams=1, n_old_kf=2)
d = "gpurun_out/r06s/map"; os.makedirs(d, exist_ok=True)
for k in ["kf_id", "kf_pose", "kf_intr", "kf_has_cam", "kf_feat_ptr", "feat_uv", "feat_lm_id", "feat_flags",
          "lm_id", "lm_pos", "lm_bad", "lm_obs_ptr", "obs_kf_id", "obs_feat_idx"]:
    np.ascontiguousarray(m[k]).tofile(os.path.join(d, k + ".bin"))
PY
for mode in resident snapshot; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$mode -o run -- visionx-slam_amd/build/adapter_driver ba_calls $O/map 50 5 -1 30 $mode > $O/kt_$mode.log 2>&1 || { tail -20 $O/kt_$mode.log; exit 5; }
done
rm -rf $O/map
find $O -name "*kernel_stats.csv" | head
