#!/bin/bash
# pipelined C3 frame under scheduling options, 3 runs each (run-to-run spread ~3 %)
cd "$GRAFT_REPO_ROOT" || exit 1
for opt in "" "--ba-cus 0.25" "--ba-cus 0.5" "--ba-priority 1" "--ba-priority 1 --ba-cus 0.25"; do
  vals=""
  for rep in 1 2 3; do
    v=$(timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile $opt 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 1
    vals="$vals $v"
  done
  echo "[$opt]:$vals"
done
