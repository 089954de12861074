#!/bin/bash
# round 6 (f): k_ba_win with its loop-invariant records in LDS — parity, timeline, alone, pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06f}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "ba_ or frontend" > $O/t_parity.txt 2>&1 || { tail -40 $O/t_parity.txt; exit 2; }
tail -2 $O/t_parity.txt
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python scripts/ktrace_win.py > $O/ktrace.txt 2>&1 || { tail -20 $O/ktrace.txt; exit 3; }
cat $O/ktrace.txt
for r in 1 2; do
  for v in 1 0; do
    VX_BA_PERSIST=$v timeout -k 10 120 python scripts/ba_alone.py >> $O/alone.txt 2>&1 || { tail -5 $O/alone.txt; exit 4; }
  done
done
cut -c1-90 $O/alone.txt
timeout -k 10 600 bash scripts/ab_env.sh 2 VX_BA_PERSIST 1 0 > $O/ab_bench.txt 2>&1 || { cat $O/ab_bench.txt; exit 5; }
cat $O/ab_bench.txt
timeout -k 10 300 python scripts/potrf_yardstick.py 50 > $O/potrf.txt 2>&1 || { tail -20 $O/potrf.txt; exit 6; }
cat $O/potrf.txt

echo done
