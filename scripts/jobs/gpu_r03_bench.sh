#!/bin/bash
# Round-3 measurement session (TAG): default bench (2000 steps, CPU baseline), the driver's short
# command three times, and a rocprofv3 kernel-trace summary of the same pipeline.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_s20_$r.json 2> gpurun_out/bench_${TAG}_s20_$r.err || { echo "short bench failed"; tail -20 gpurun_out/bench_${TAG}_s20_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_s20_$r.json')); print('s20', d['value'], d['latency_ms_per_frame'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 300 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
f=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/kernel_stats_${TAG}.csv; head -40 gpurun_out/kernel_stats_${TAG}.csv
