#!/bin/bash
# round 5 (m): what the short command's gap depends on: warm-up length, step count.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
for rep in 1 2; do
  for a in "20 5" "20 100" "100 5" "20 5 late"; do
    set -- $a
    E=""; [ "$3" = late ] && E="VX_BENCH_GC_LATE=1"
    ( [ -n "$E" ] && export $E; timeout -k 10 300 python3 bench.py --gpus 1 --steps $1 --warmup $2 --no-cpu-baseline --no-profile > $O/r.json 2> $O/r.err ) || { tail -20 $O/r.err; exit 2; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('steps $1 warmup $2 $3', $rep, d['value'], d['host_enqueue_ms_per_step'])" | tee -a $O/summary.txt
  done
done
echo done
