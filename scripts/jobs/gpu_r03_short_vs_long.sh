#!/bin/bash
# The driver's short command (--steps 20 --warmup 5) three times against the 2000-step default
# (both without the CPU baseline), TAG.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-sl}
EXTRA=${EXTRA:-}
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $EXTRA > gpurun_out/${TAG}_s20_$r.json 2>/dev/null || { echo "short failed"; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline $EXTRA > gpurun_out/${TAG}_long_$r.json 2>/dev/null || { echo "long failed"; exit 1; }
  python3 -c "
import json
a = json.load(open('gpurun_out/${TAG}_s20_$r.json')); b = json.load(open('gpurun_out/${TAG}_long_$r.json'))
print('s20', a['value'], 'long', b['value'], 'ratio', round(a['value'] / b['value'], 3), 'fps', a['config']['frames_per_step'])"
done
