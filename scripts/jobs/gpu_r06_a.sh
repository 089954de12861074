#!/bin/bash
# round 6 (a): the GPU suite + smoke on the round's first changes; the committed C3 line and the
# rocprofv3 kernel statistics of the SAME command (its own JSON line kept, so the roofline check of
# tests/test_bench_contract.py compares one process with itself); C4 with its CPU baseline; the
# 256-observation fused packing cap A/B (VERDICT r5 #2b) alone and in the pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 2; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 3; }
timeout -k 10 300 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 4; }
cat $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_c3_rocprof.json 2> $O/prof.log || { tail -30 $O/prof.log; exit 5; }
rm -f $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_bench_c3.csv \;
head -4 $O/kernel_stats_bench_c3.csv | cut -c1-200
timeout -k 10 300 python bench.py --config C4 --steps 200 --warmup 10 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 6; }
cat $O/bench_c4.json | cut -c1-300
for r in 1 2; do
  for cap in 512 256; do
    VX_BA_FUSED_CAP=$cap timeout -k 10 120 python scripts/ba_alone.py >> $O/cap_alone.txt 2>&1 || exit 7
  done
done
cut -c1-160 $O/cap_alone.txt
timeout -k 10 900 bash scripts/ab_env.sh 2 VX_BA_FUSED_CAP 512 256 > $O/cap_bench.txt 2>&1 || { cat $O/cap_bench.txt; exit 8; }
cat $O/cap_bench.txt
echo done
