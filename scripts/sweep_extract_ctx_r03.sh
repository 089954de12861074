#!/bin/bash
# Extraction contexts x grid share with the STL-order select (r03): 2 alternating rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/sweep_ectx_${TAG:-a}.txt
: > $out
for rep in 1 2; do
  for cfg in "2 0.25" "3 0.25" "3 0.2" "4 0.2" "4 0.15"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --steps 2000 --no-cpu-baseline --no-profile --extract-ctx $1 --grid-share $2 > gpurun_out/ectx.json 2>/dev/null || { echo "bench failed $cfg"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ectx.json')); print('E=$1 share=$2', d['value'], d['latency_ms_per_frame'])" | tee -a $out
  done
done
