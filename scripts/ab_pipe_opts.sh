#!/bin/bash
# bench.py value for two option sets, alternating: bash scripts/ab_pipe_opts.sh reps "opts A" "opts B"
set -o pipefail
reps=$1; A=$2; B=$3
for r in $(seq $reps); do
  for o in "$A" "$B"; do
    v=$(timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile $o 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['latency_ms_per_frame'])") || exit 1
    echo "[$o] $v"
  done
done
