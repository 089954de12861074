#!/bin/bash
# pipelined C3 frame with LocalBA on a disjoint CU share just above its workgroup count, against
# shared CUs, at two extraction grid shares; 2 runs each
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for cus in 0 0.54 0.6 0.667; do
    for g in 0.3333 0.5; do
      v=$(timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --ba-cus $cus --grid-share $g 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['host_enqueue_ms_per_step'])") || exit 1
      echo "ba-cus $cus grid-share $g: $v"
    done
  done
done
