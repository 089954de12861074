#!/bin/bash
# round 4: Schur factor with step descriptors as launch arguments and the prefetching
# back-substitution — SBA tests, the bench, a kernel trace of the connected C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_sba.py tests/test_gpu_dmap.py -m gpu > $O/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench.jsonl 2>&1 || exit 4
VX_SBA_FACTOR=single SBA_CFGS=C5-connected timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench_single_c5c.jsonl 2>&1 || exit 4
export TMPDIR=/tmp
SBA_CFGS=C5-connected timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/sba_bench.py 2 > /dev/null 2>&1 || exit 5
python3 scripts/sba_fac_trace.py $O/kt/kt_kernel_trace.csv > $O/sba_fac_trace.txt 2>&1
rm -f $O/kt/kt_kernel_trace.csv
cat $O/sba_fac_trace.txt
for cols in 1 2; do
  VX_SBA_FACTOR_COLS=$cols SBA_CFGS=C5-connected timeout -k 10 200 python3 scripts/sba_bench.py 10 > $O/sba_cols$cols.jsonl 2>&1 || exit 6
done
