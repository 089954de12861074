#!/bin/bash
# bench.py value with Match on its own context vs on the extraction context of its frame, alternating.
set -o pipefail
for r in 1 2 3; do
  for opt in "--match-ctx own" "--match-ctx extract"; do
    v=$(timeout -k 10 300 python bench.py $opt 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['latency_ms_per_frame'])") || exit 1
    echo "opt=[$opt] value/latency: $v"
  done
done
