#!/bin/bash
# round 6 (x): k_ba_win with the pose-stage rounds split evenly over the waves (VX_BA_WIN_EVEN)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dmap.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread -k "ba or dmap or shard or win or graph or seq" > $O/t.txt 2>&1 || { tail -40 $O/t.txt; exit 2; }
tail -1 $O/t.txt
for i in 1 2 3; do
  for v in 1 0; do
    VX_BA_WIN_EVEN=$v timeout -k 10 120 python3 scripts/ba_alone.py 2>&1 | cut -c1-80 | sed "s/^/EVEN=$v /"
  done
done | tee $O/alone.txt
VX_LIB=visionx-slam_amd/lib/libvxslam_trace_lm.so timeout -k 10 300 python3 -u scripts/win_stages.py > $O/win_stages_even.txt 2>&1 || { cat $O/win_stages_even.txt; exit 3; }
cat $O/win_stages_even.txt
timeout -k 10 900 bash scripts/ab_env.sh 3 VX_BA_WIN_EVEN 1 0 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 4; }
cat $O/ab.txt
