#!/bin/bash
# round 5 (q): k_ba_iter with the padding loads dropped (landmark rows past B.x, pose-stage lanes past
# the entries' ends) + the Schur clearing in k_sba_update: parity subsets, durations, PMC traffic of
# the LocalBA window alone, back-substitution depth A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_dmap.py tests/test_gpu_sharded.py tests/test_gpu_fused_build.py tests/test_gpu_sba.py tests/test_cpp_adapters.py -m gpu > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 2; }
tail -1 $O/par.log
( timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/ba_alone.py > $O/kt.log 2>&1 ) || { tail -20 $O/kt.log; exit 5; }
python3 scripts/ba_iter_durations.py "$(find $O/kt -name 'kt_kernel_trace.csv' | head -1)" > $O/durations.txt 2>&1
rm -rf $O/kt
head -9 $O/durations.txt
for c in FETCH_SIZE WRITE_SIZE; do
  ( timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 scripts/ba_alone.py > $O/pmc_$c.log 2>&1 ) || { tail -20 $O/pmc_$c.log; exit 6; }
done
python3 scripts/pmc_summary.py "$(find $O/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1)" "$(find $O/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)" $O/pmc.json > $O/pmc.txt 2>&1 || { tail -20 $O/pmc.txt; exit 7; }
rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE
grep -E "k_ba_iter|k_ba_prologue" $O/pmc.txt
for d in 3 6; do
  ( export VX_SBA_BS_DEPTH=$d SBA_CFGS=C5-connected; timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/sba_bench.py 6 > $O/skt.log 2>&1 ) || { tail -20 $O/skt.log; exit 8; }
  echo "depth $d: $(python3 scripts/kt_avg.py "$(find $O/kt -name 'kt_kernel_trace.csv' | head -1)" k_sba_backsub k_sba_update k_sba_fac_blk | tr '\n' ' ') $(python3 -c "import json; d=json.loads(open('$O/skt.log').readlines()[-1]); print(d['ms_per_optimize'], d['kernel_us_per_iteration'].get('sba_solve'))")" | tee -a $O/bs_ab.txt
  rm -rf $O/kt
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-profile > $O/b.$rep.json 2> $O/b.$rep.err || { tail -20 $O/b.$rep.err; exit 9; }
  python3 -c "import json; d=json.load(open('$O/b.$rep.json')); print('bench', $rep, d['value'], d['latency_ms_per_frame'])" | tee -a $O/bench.txt
done
echo done
