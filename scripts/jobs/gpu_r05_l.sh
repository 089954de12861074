#!/bin/bash
# round 5 (l): the driver's short command against a long run, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/s_$rep.json 2> $O/s_$rep.err || { tail -20 $O/s_$rep.err; exit 2; }
  python3 -c "import json; d=json.load(open('$O/s_$rep.json')); print('short', $rep, d['value'], d['host_enqueue_ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['pass_ms_per_step'])" | tee -a $O/summary.txt
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 1000 --warmup 5 --no-cpu-baseline --no-profile > $O/l_$rep.json 2> $O/l_$rep.err || { tail -20 $O/l_$rep.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/l_$rep.json')); print('long', $rep, d['value'], d['host_enqueue_ms_per_step'])" | tee -a $O/summary.txt
done
echo done
