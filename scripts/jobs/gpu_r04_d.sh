#!/bin/bash
# round 4: the full GPU suite + smoke, then the seq-threads A/B, per-iteration k_ba_iter durations
# (default layout), the Schur bench and its MFMA counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 240 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 3
for i in 1 2; do
  for t in 1 4; do
    timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --seq-threads $t > $O/bench_t$t.$i.json 2> $O/bench_t$t.$i.err || exit 4
  done
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt0 -o kt -- python3 scripts/ba_alone.py > /dev/null 2>&1 || exit 5
python3 scripts/ba_iter_durations.py $O/kt0/kt_kernel_trace.csv 58120 24917 8590 3232 1320 > $O/ba_iter_durations_compact0.txt 2>&1
rm -f $O/kt0/kt_kernel_trace.csv
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench.jsonl 2>&1 || exit 6
SBA_CFGS=C5-connected timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d $O/pmc_sba -o pmc -- python3 scripts/sba_bench.py 2 > /dev/null 2>&1 || exit 7
python3 scripts/pmc_sba_summary.py "$(find $O/pmc_sba -name "*counter_collection.csv" | head -1)" > $O/pmc_sba_c5_connected.txt 2>&1
