#!/bin/bash
# which chain bounds the pipelined frame: bench.py with one stage left out (diagnostic), 2 runs each
cd "$GRAFT_REPO_ROOT" || exit 1
for e in ${EXTRACT_CTX:-1 2}; do
  for sk in "" ba match extract; do
    vals=""
    for rep in 1 2; do
      v=$(timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --extract-ctx $e ${sk:+--diag-skip $sk} 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 1
      vals="$vals $v"
    done
    echo "extract-ctx $e skip [$sk]:$vals"
  done
done
