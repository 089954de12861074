#!/bin/bash
# round 4: the multi-workgroup Schur factor with the look-ahead column in LDS — SBA tests, then the
# connected C5 with and without it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_sba.py -m gpu > $O/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for la in 1 0; do
    VX_SBA_LOOKAHEAD_LDS=$la SBA_CFGS=C5-connected timeout -k 10 200 python3 scripts/sba_bench.py 10 > $O/sba_la$la.$rep.jsonl 2>&1 || exit 4
  done
done
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench_all.jsonl 2>&1 || exit 5
