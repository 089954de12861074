#!/bin/bash
# round 5 (r): padding loads skipped or not (VX_BA_PADSKIP), alternating on one box: launch durations,
# LocalBA alone, the C3 pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
for v in 1 0; do
  ( export VX_BA_PADSKIP=$v; timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt$v -o kt -- python3 scripts/ba_alone.py > $O/kt$v.log 2>&1 ) || { tail -20 $O/kt$v.log; exit 5; }
  python3 scripts/ba_iter_durations.py "$(find $O/kt$v -name 'kt_kernel_trace.csv' | head -1)" > $O/durations_padskip$v.txt 2>&1
  rm -rf $O/kt$v
  echo "== padskip $v"; head -9 $O/durations_padskip$v.txt
done
for rep in 1 2; do
  for v in 1 0; do
    VX_BA_PADSKIP=$v timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
    VX_BA_PADSKIP=$v timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-profile > $O/b_$v.$rep.json 2> $O/b_$v.$rep.err || { tail -20 $O/b_$v.$rep.err; exit 6; }
    python3 -c "import json; d=json.load(open('$O/b_$v.$rep.json')); print('padskip=$v', $rep, d['value'], d['latency_ms_per_frame'])" | tee -a $O/bench_ab.txt
  done
done
cut -c1-100 $O/alone.txt
echo done
