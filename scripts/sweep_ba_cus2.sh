#!/bin/bash
# pipelined C3 frame with LocalBA on most of the CUs (disjoint masks), 3 runs each
cd "$GRAFT_REPO_ROOT" || exit 1
for cus in 0 0.6667 0.75 0.8; do
  vals=""
  for rep in 1 2 3; do
    v=$(timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --ba-cus $cus 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 1
    vals="$vals $v"
  done
  echo "ba-cus $cus:$vals"
done
