#!/bin/bash
# Round-4 committed measurement (TAG): the whole GPU suite, smoke(), scripts/gpu_bench.sh (PMC
# traffic -> profiles/pmc_traffic.json, the default bench with its CPU baseline, rocprofv3 kernel
# stats), the driver's short command three times, a kernel trace of the resident one-call LocalBA,
# C2 / C4, the C5 rig and the Schur bench.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r04}
echo "tests"
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${TAG}.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
echo "smoke ok"
TAG=$TAG bash scripts/gpu_bench.sh || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_s20_$r.json 2> gpurun_out/bench_${TAG}_s20_$r.err || { echo "short bench failed"; tail -20 gpurun_out/bench_${TAG}_s20_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_s20_$r.json')); print('s20', d['value'], d['latency_ms_per_frame'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dmap_${TAG} -o run -- python3 scripts/dmap_optimize_loop.py 100 > gpurun_out/prof_dmap_${TAG}.log 2>&1 || { echo "dmap prof failed"; tail -20 gpurun_out/prof_dmap_${TAG}.log; exit 1; }
rm -f gpurun_out/prof_dmap_${TAG}/*kernel_trace.csv
for cfg in C2 C4; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo "$cfg bench failed"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$cfg.json')); print('$cfg', d['value'], d['latency_ms_per_frame'])"
done
timeout -k 10 300 python3 scripts/c5_rig_one_gpu.py > gpurun_out/c5_rig_${TAG}.jsonl 2> gpurun_out/c5_rig_${TAG}.err || { echo "c5 failed"; tail -20 gpurun_out/c5_rig_${TAG}.err; exit 1; }
timeout -k 10 300 python3 scripts/sba_bench.py 10 > gpurun_out/sba_bench_${TAG}.jsonl 2>&1 || { echo "sba bench failed"; exit 1; }
echo done
