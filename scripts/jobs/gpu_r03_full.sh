#!/bin/bash
# Round-3 committed measurement (TAG): the whole GPU suite, smoke(), the k_select_stl phase trace
# (C3, C4), then scripts/gpu_bench.sh (PMC traffic passes -> profiles/pmc_traffic.json, the default
# bench with its CPU baseline, rocprofv3 kernel stats) and the driver's short command three times.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${TAG}.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
echo "smoke ok"
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_select.py > gpurun_out/ktrace_select_${TAG}.txt 2>&1 || { echo "ktrace failed"; exit 1; }
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_select.py C4 >> gpurun_out/ktrace_select_${TAG}.txt 2>&1 || { echo "ktrace C4 failed"; exit 1; }
TAG=$TAG bash scripts/gpu_bench.sh || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_s20_$r.json 2> gpurun_out/bench_${TAG}_s20_$r.err || { echo "short bench failed"; tail -20 gpurun_out/bench_${TAG}_s20_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_s20_$r.json')); print('s20', d['value'], d['latency_ms_per_frame'])"
done
