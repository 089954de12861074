#!/bin/bash
# A/B of pipeline / library variants (alternating, REPS rounds): each line "name value latency".
# VARIANTS: "name|ENV=..|bench args" entries separated by ';'.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/ab_${TAG:-a}.txt
: > $out
IFS=';' read -ra VS <<< "$VARIANTS"
for rep in $(seq 1 ${REPS:-3}); do
  for v in "${VS[@]}"; do
    IFS='|' read -r name envs args <<< "$v"
    env $envs timeout -k 10 150 python bench.py --steps 2000 --no-cpu-baseline --no-profile $args > gpurun_out/ab.json 2>/dev/null || { echo "bench failed: $v"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$name', d['value'], d['latency_ms_per_frame'])" | tee -a $out
  done
done
