#!/bin/bash
# round 6 (y): VX_BA_WIN_EVEN=1 (pose-stage rounds split evenly, unconditional loads) vs 0, alone + stages
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06y}
mkdir -p $O
VX_BA_WIN_EVEN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "ba_" > $O/t.txt 2>&1 || { tail -40 $O/t.txt; exit 2; }
tail -1 $O/t.txt
for i in 1 2 3; do
  for v in 1 0; do
    VX_BA_WIN_EVEN=$v timeout -k 10 120 python3 scripts/ba_alone.py 2>&1 | cut -c1-80 | sed "s/^/EVEN=$v /"
  done
done | tee $O/alone.txt
for v in 1 0; do
  VX_BA_WIN_EVEN=$v VX_LIB=visionx-slam_amd/lib/libvxslam_trace_lm.so timeout -k 10 300 python3 -u scripts/win_stages.py > $O/win_stages_$v.txt 2>&1 || { cat $O/win_stages_$v.txt; exit 3; }
  echo "EVEN=$v"; cat $O/win_stages_$v.txt
done
