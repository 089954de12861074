#!/bin/bash
# bench.py value for 1..4 extraction contexts (frames alternate; Match on the frame's context), 3 runs each
set -o pipefail
for r in 1 2 3; do
  for e in ${EXTRACT_CTX:-2 3 4}; do
    v=$(timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --extract-ctx $e 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['latency_ms_per_frame'])") || exit 1
    echo "extract-ctx $e: $v"
  done
done
