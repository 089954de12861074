#!/bin/bash
# round 5 (z): k_ba_iter with the entry records and rows issued ahead of the landmark loads (block
# records by scalar loads) against the previous build (VX_LIB=...head.so), alternating on one box:
# BA parity tests, launch durations, LocalBA alone, the C3 pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05z}
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_dmap.py tests/test_gpu_batch.py -m gpu > $O/ba_tests.log 2>&1 || { tail -40 $O/ba_tests.log; exit 2; }
tail -1 $O/ba_tests.log
HEADLIB=visionx-slam_amd/lib/libvxslam_head.so
for v in new head; do
  if [ $v = head ]; then export VX_LIB=$HEADLIB; else unset VX_LIB; fi
  ( timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt$v -o kt -- python3 scripts/ba_alone.py > $O/kt$v.log 2>&1 ) || { tail -20 $O/kt$v.log; exit 5; }
  python3 scripts/ba_iter_durations.py "$(find $O/kt$v -name 'kt_kernel_trace.csv' | head -1)" > $O/durations_$v.txt 2>&1
  rm -rf $O/kt$v
  echo "== $v"; head -9 $O/durations_$v.txt
done
for rep in 1 2; do
  for v in new head; do
    if [ $v = head ]; then export VX_LIB=$HEADLIB; else unset VX_LIB; fi
    timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
    timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-profile > $O/b_$v.$rep.json 2> $O/b_$v.$rep.err || { tail -20 $O/b_$v.$rep.err; exit 6; }
    python3 -c "import json; d=json.load(open('$O/b_$v.$rep.json')); print('$v', $rep, d['value'], d['latency_ms_per_frame'])" | tee -a $O/bench_ab.txt
  done
done
cut -c1-100 $O/alone.txt
echo done
