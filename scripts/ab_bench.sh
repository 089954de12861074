#!/bin/bash
# bench.py value for the in-tree library vs others, alternating: bash scripts/ab_bench.sh reps lib...
set -o pipefail
reps=$1; shift
for r in $(seq $reps); do
  for lib in - "$@"; do
    if [ "$lib" = "-" ]; then unset VX_LIB; name=tree; else export VX_LIB=$lib; name=$(basename $lib .so); fi
    v=$(timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['latency_ms_per_frame'])") || exit 1
    echo "$name $v"
  done
done
