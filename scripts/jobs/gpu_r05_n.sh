#!/bin/bash
# round 5 (n): direct row reads without the first barrier (VX_BA_DROW): LocalBA parity subset,
# launch durations, LocalBA alone and the pipeline, A/B against the combine.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_dmap.py tests/test_gpu_sharded.py tests/test_gpu_fused_build.py tests/test_cpp_adapters.py -m gpu -k "ba_ or graph_replay or seq or shard or layout or dmap or adapter" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 2; }
tail -1 $O/par.log
for v in 1 0; do
  ( export VX_BA_DROW=$v; timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt$v -o kt -- python3 scripts/ba_alone.py > $O/kt$v.log 2>&1 ) || { tail -20 $O/kt$v.log; exit 5; }
  python3 scripts/ba_iter_durations.py "$(find $O/kt$v -name 'kt_kernel_trace.csv' | head -1)" > $O/durations_drow$v.txt 2>&1
  rm -f $(find $O/kt$v -name '*.csv')
  echo "== drow $v"; head -9 $O/durations_drow$v.txt
done
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_ba.py > $O/ktrace.txt 2>&1 || { tail -20 $O/ktrace.txt; exit 7; }
head -12 $O/ktrace.txt
for rep in 1 2; do
  for v in 1 0; do
    VX_BA_DROW=$v timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
    VX_BA_DROW=$v timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-profile > $O/b_$v.$rep.json 2> $O/b_$v.$rep.err || { tail -20 $O/b_$v.$rep.err; exit 6; }
    python3 -c "import json; d=json.load(open('$O/b_$v.$rep.json')); print('drow=$v', $rep, d['value'], d['latency_ms_per_frame'], d['host_enqueue_ms_per_step'])" | tee -a $O/bench_ab.txt
  done
done
cut -c1-100 $O/alone.txt
echo done
