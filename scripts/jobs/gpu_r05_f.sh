#!/bin/bash
# round 5 (f): the C3 pipeline against the matcher variants; the blocked Schur factor (k_sba_fac_blk): the SBA parity / bitwise tests, then the
# Schur bench (blocked against one column per launch) and a kernel trace of the connected C5 solve.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
# the C3 pipeline against the matcher's grid cap and load hoisting (session e: 0.1287 ms/frame with
# both, against 0.065 in session b without either)
for v in "VX_MATCH_GRID=0 VX_MATCH_HOIST=0" "VX_MATCH_HOIST=0" "VX_MATCH_GRID=0 VX_MATCH_HOIST=1" "VX_MATCH_HOIST=1"; do
  ( export $v; timeout -k 10 300 python -u bench.py --steps 500 --warmup 20 --no-cpu-baseline --no-profile > $O/b.json 2> $O/b.err ) || { tail -20 $O/b.err; exit 7; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('$v', d['value'], d['latency_ms_per_frame'], d['host_enqueue_ms_per_step'])" | tee -a $O/bench_match_ab.txt
done
timeout -k 10 120 python3 scripts/ba_alone.py > $O/alone.txt 2>&1 || exit 4
cut -c1-120 $O/alone.txt
timeout -k 10 400 $T tests/test_gpu_sba.py tests/test_gpu_dmap.py tests/test_gpu_sharded.py -m gpu -k "sba or schur" > $O/sba_tests.log 2>&1 || { tail -40 $O/sba_tests.log; exit 2; }
tail -1 $O/sba_tests.log
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench_blk.jsonl 2>&1 || { tail -20 $O/sba_bench_blk.jsonl; exit 6; }
VX_SBA_FACTOR=multi timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench_multi.jsonl 2>&1 || { tail -20 $O/sba_bench_multi.jsonl; exit 6; }
for f in blk multi; do
python3 -c "
import json
for l in open('$O/sba_bench_$f.jsonl'):
    d = json.loads(l); print('$f', d['config'], d['ms_per_optimize'], d['kernel_us_per_iteration'].get('sba_solve'), d['mfma_fp64'])"
done
( export SBA_CFGS=C5-connected; timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 scripts/sba_bench.py 4 > $O/kt.log 2>&1 ) || { tail -20 $O/kt.log; exit 5; }
python3 scripts/kt_avg.py "$(find $O/kt -name 'kt_kernel_trace.csv' | head -1)" k_sba_fac_blk k_sba_backsub k_sba_blocks k_sba_lm k_sba_update
cp "$(find $O/kt -name 'kt_kernel_stats.csv' | head -1)" $O/kernel_stats_sba_connected.csv
rm -f $(find $O/kt -name '*.csv')
echo done
