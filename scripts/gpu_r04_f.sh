#!/bin/bash
# round 4: LocalBA on whole XCDs (its own L2s) against shared CUs — C3 pipelined bench, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 60 scripts/probe/xcd_probe > $O/xcd_probe.txt 2>&1 || exit 3
timeout -k 10 120 python3 scripts/ba_cumask.py > $O/ba_cumask.txt 2>&1 || exit 3
for rep in 1 2; do
  for cfg in "shared:" "rr4:--ba-xcds 4 --cu-xcd-map rr" "block4:--ba-xcds 4 --cu-xcd-map block" \
             "rr5:--ba-xcds 5 --cu-xcd-map rr" "block5:--ba-xcds 5 --cu-xcd-map block"; do
    name=${cfg%%:*}; flags=${cfg#*:}
    timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline $flags > $O/bench_$name.$rep.json 2> $O/bench_$name.$rep.err || exit 4
    python3 -c "import json,sys; d=json.load(open('$O/bench_$name.$rep.json')); print('$name', $rep, d['value'], d['host_enqueue_ms_per_step'], d['latency_ms_per_frame'])" >> $O/summary.txt
  done
done
