#!/bin/bash
# k_pyramid tile / block against the 3-stream pipeline (default bench): does a smaller pyramid
# grid leave room for the concurrent LocalBA kernels?
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for tb in ${TBS:-"0 0" "64 1024" "80 1024" "96 1024" "64 512"}; do
  set -- $tb
  if [ "$1" = 0 ]; then unset VX_PYR_TILE VX_PYR_BLOCK; else export VX_PYR_TILE=$1 VX_PYR_BLOCK=$2; fi
  for rep in 1 2 3; do
    timeout -k 10 120 python bench.py --steps 200 --no-cpu-baseline --no-profile > gpurun_out/sp.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/sp.json')); print('tile $1 block $2', d['value'])"
  done
done
