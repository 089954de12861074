#!/bin/bash
# round 5 (b): row sums by float atomics as the fused LocalBA's default (prologue included): the
# whole GPU suite, per-launch durations of atomic rows (512 and 256 threads) against the slot sums,
# LocalBA alone, and the C3 pipeline (1000-step bench runs, alternating atomic / slots).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
[ $rc -le 1 ] || { echo "gpu tests rc $rc"; tail -40 $O/gpu_tests.log; exit 2; }  # (1 = failed tests: go on)
tail -1 $O/gpu_tests.log
for v in atomic slots atomic256; do
  case $v in
    atomic) E="VX_BA_ATOMIC_ROWS=1" ;;
    slots) E="VX_BA_ATOMIC_ROWS=0" ;;
    atomic256) E="VX_BA_FUSED_THREADS=256" ;;
  esac
  ( export "$E"; timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/ba_alone.py > $O/kt_$v.log 2>&1 ) || { tail -20 $O/kt_$v.log; exit 5; }
  python3 scripts/ba_iter_durations.py "$(find $O/kt_$v -name 'kt_kernel_trace.csv' | head -1)" > $O/durations_$v.txt 2>&1
  rm -f $(find $O/kt_$v -name '*.csv')
  echo "== $v"; cat $O/durations_$v.txt
done
for rep in 1 2; do
  timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
  VX_BA_ATOMIC_ROWS=0 timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
done
cut -c1-120 $O/alone.txt
for rep in 1 2; do
  for v in 1 0; do
    VX_BA_ATOMIC_ROWS=$v timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-profile > $O/b_$v.$rep.json 2> $O/b_$v.$rep.err || { tail -20 $O/b_$v.$rep.err; exit 6; }
    python3 -c "import json; d=json.load(open('$O/b_$v.$rep.json')); print('atomic=$v', $rep, d['value'], d['latency_ms_per_frame'], d['host_enqueue_ms_per_step'])" | tee -a $O/bench_ab.txt
  done
done
echo done
