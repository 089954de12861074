#!/bin/bash
# round 4: LDS-only barriers in the Schur back-substitution / look-ahead; phase trace of the factor
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_sba.py -m gpu > $O/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench.jsonl 2>&1 || exit 4
for cols in 1 2; do
  VX_SBA_FACTOR_COLS=$cols SBA_CFGS=C5-connected timeout -k 10 200 python3 scripts/sba_bench.py 10 > $O/sba_cols$cols.jsonl 2>&1 || exit 6
done
VX_SBA_FACTOR_COLS=1 VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 200 python3 scripts/ktrace_sba_multi.py > $O/ktrace_sba_multi.txt 2>&1 || exit 7
cat $O/ktrace_sba_multi.txt
