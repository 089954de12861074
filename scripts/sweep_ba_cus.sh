#!/bin/bash
# pipelined frame with LocalBA on a disjoint CU share (bench.py --ba-cus) vs shared CUs
cd "$GRAFT_REPO_ROOT" || exit 1
for cus in 0 0.5 0.3333 0.25; do
  for g in 0.3333 1.0; do
    v=$(timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --ba-cus $cus --grid-share $g 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])") || exit 1
    echo "ba-cus $cus grid-share $g: $v"
  done
done
