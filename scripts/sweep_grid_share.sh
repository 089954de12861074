#!/bin/bash
# bench.py value vs the extraction contexts' grid share, for 2 and 3 extraction contexts, 2 runs each
set -o pipefail
for r in 1 2; do
  for e in 2 3; do
    for g in ${SHARES:-0.2 0.25 0.333 0.5}; do
      v=$(timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --extract-ctx $e --grid-share $g 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])") || exit 1
      echo "extract-ctx $e grid-share $g: $v"
    done
  done
done
