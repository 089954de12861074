#!/bin/bash
# round 4: everything new (resident BA, seq bench, connected C5, Schur plan from the resident map,
# compacted pose stage) — GPU tests, A/B of the compacted pose stage, a short bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_dmap.py \
    tests/test_cpp_adapters.py tests/test_gpu_sba.py tests/test_gpu_parity.py tests/test_gpu_fused_build.py \
    tests/test_gpu_sharded.py -m gpu > $O/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> $O/tests.log
# ordinary test failures (rc 1) go on to the measurements; a fault, abort or time limit ends the call
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    VX_BA_COMPACT=$v timeout -k 10 120 python -u scripts/ba_alone.py >> $O/ab_compact.txt 2>&1 || exit 4
  done
done
timeout -k 10 300 python -u scripts/sba_plan_time.py $O/sba_plan_time.json > $O/sba_plan_time.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 6
export TMPDIR=/tmp
for v in 1 0; do
  VX_BA_COMPACT=$v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt$v -o kt -- python3 scripts/ba_alone.py > /dev/null 2>&1 &&
  python3 scripts/ba_iter_durations.py $O/kt$v/kt_kernel_trace.csv 58120 24917 8590 3232 1320 > $O/ba_iter_durations_compact$v.txt 2>&1 || exit 7
done
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench.jsonl 2>&1 &&
SBA_CFGS=C5-connected timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d $O/pmc_sba -o pmc -- python3 scripts/sba_bench.py 2 > /dev/null 2>&1 &&
python3 scripts/pmc_sba_summary.py "$(find $O/pmc_sba -name "*counter_collection.csv" | head -1)" > $O/pmc_sba_c5_connected.txt 2>&1
