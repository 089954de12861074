#!/bin/bash
# round 6 (e): k_ba_win timeline (trace build) with the wave-by-wave hand-off and with the
# workgroup-barrier one; LocalBA alone for both and the per-iteration launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06e}
mkdir -p $O
for v in 1 0; do
  VX_BA_WIN_WSIG=$v VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python scripts/ktrace_win.py > $O/ktrace_wsig$v.txt 2>&1 || { tail -20 $O/ktrace_wsig$v.txt; exit 2; }
  cat $O/ktrace_wsig$v.txt
done
for r in 1 2; do
  for v in 1 0; do
    VX_BA_WIN_WSIG=$v timeout -k 10 120 python scripts/ba_alone.py >> $O/alone.txt 2>&1 || { tail -5 $O/alone.txt; exit 4; }
  done
  VX_BA_PERSIST=0 timeout -k 10 120 python scripts/ba_alone.py >> $O/alone.txt 2>&1 || { tail -5 $O/alone.txt; exit 4; }
done
cut -c1-110 $O/alone.txt
echo done
