#!/bin/bash
# bench.py value for 1 / 2 extraction contexts at several extraction grid shares
cd "$GRAFT_REPO_ROOT" || exit 1
for e in 1 2; do
  for g in 0.3333 0.5 1.0; do
    v=$(timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --extract-ctx $e --grid-share $g 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['latency_ms_per_frame'])") || exit 1
    echo "extract-ctx $e grid-share $g: $v"
  done
done
