#!/bin/bash
# round 4: the multi-workgroup Schur factorisation — SBA tests, then single vs multi per config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_sba.py -m gpu > $O/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 60 scripts/probe/xcd_probe > $O/xcd_probe.txt 2>&1 || exit 3
timeout -k 10 120 python3 scripts/ba_cumask.py > $O/ba_cumask.txt 2>&1 || exit 3
VX_SBA_FACTOR=single timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench_single.jsonl 2>&1 || exit 4
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench_multi.jsonl 2>&1 || exit 5
for g in 4 8 16 32; do
  VX_SBA_FACTOR_GROUPS=$g SBA_CFGS=C5-connected timeout -k 10 200 python3 scripts/sba_bench.py 10 >> $O/sba_groups.jsonl 2>&1 || exit 6
done
export TMPDIR=/tmp
SBA_CFGS=C5-connected timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d $O/pmc_sba -o pmc -- python3 scripts/sba_bench.py 2 > /dev/null 2>&1 || exit 7
python3 scripts/pmc_sba_summary.py "$(find $O/pmc_sba -name "*counter_collection.csv" | head -1)" > $O/pmc_sba_c5_connected_multi.txt 2>&1
