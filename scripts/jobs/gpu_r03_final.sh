#!/bin/bash
# Final round-3 numbers (TAG): the default bench three more times (spread), C2 and C4 with the
# final code, and the C5 rig on one GPU.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-fin}
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_c3_$r.json 2> gpurun_out/bench_${TAG}_c3_$r.err || { echo "c3 bench failed"; tail -20 gpurun_out/bench_${TAG}_c3_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_c3_$r.json')); print('C3', d['value'], d['latency_ms_per_frame'])"
done
for cfg in C2 C4; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo "$cfg bench failed"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$cfg.json')); print('$cfg', d['value'], d['latency_ms_per_frame'])"
done
timeout -k 10 300 python3 scripts/c5_rig_one_gpu.py > gpurun_out/c5_rig_${TAG}.jsonl 2> gpurun_out/c5_rig_${TAG}.err || { echo "c5 failed"; tail -20 gpurun_out/c5_rig_${TAG}.err; exit 1; }
cat gpurun_out/c5_rig_${TAG}.jsonl
