#!/bin/bash
# round 4: recorded-sequence replay on one host thread vs one per context, alternating, 600 steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04l
mkdir -p $O
for rep in 1 2 3 4; do
  for t in 1 4; do
    timeout -k 10 300 python -u bench.py --steps 600 --warmup 20 --no-cpu-baseline --no-profile --seq-threads $t > $O/b_t$t.$rep.json 2> $O/b_t$t.$rep.err || exit 4
    python3 -c "import json; d=json.load(open('$O/b_t$t.$rep.json')); print('t$t', $rep, d['value'], d['host_enqueue_ms_per_step'], d['ms_per_step'])" >> $O/summary.txt
  done
done
cat $O/summary.txt
