#!/bin/bash
# bench.py value (and the per-stage launch times) with an environment variable at each of several
# values, alternating: bash scripts/ab_env.sh reps VAR value...
set -o pipefail
reps=$1; var=$2; shift 2
summ='import json,sys
d = json.loads(sys.stdin.read()); s = d["stages_us"]
print(d["value"], d["latency_ms_per_frame"], {k: s[k] for k in s if k.startswith(("match", "ba"))})'
for r in $(seq $reps); do
  for val in "$@"; do
    export $var=$val
    v=$(timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null | python -c "$summ") || exit 1
    echo "$var=$val $v"
  done
done
