#!/bin/bash
# round 5 (a): k_ba_iter variants at C3 — the default 512-thread layout, the 256-thread layout
# ($VX_BA_FUSED_THREADS=256) and row sums by float atomics ($VX_BA_ATOMIC_ROWS=1): oracle parity of
# each, their pose-stage balance, LocalBA alone (alternating), and per-launch durations (rocprofv3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
K="ba_golden or ba_baseline or ba_variants or graph_replay"
timeout -k 10 300 $T tests/test_gpu_parity.py -m gpu -k "$K" > $O/par_default.log 2>&1 || { tail -30 $O/par_default.log; exit 2; }
tail -1 $O/par_default.log
VX_BA_FUSED_THREADS=256 timeout -k 10 300 $T tests/test_gpu_parity.py -m gpu -k "$K" > $O/par_256.log 2>&1 || { tail -30 $O/par_256.log; exit 2; }
tail -1 $O/par_256.log
VX_BA_ATOMIC_ROWS=1 timeout -k 10 300 $T tests/test_gpu_parity.py -m gpu -k "ba_golden or ba_baseline or ba_variants" > $O/par_atomic.log 2>&1 || { tail -30 $O/par_atomic.log; exit 2; }
tail -1 $O/par_atomic.log
timeout -k 10 120 python3 scripts/fused_balance.py > $O/balance_512.txt 2>&1 || exit 3
VX_BA_FUSED_THREADS=256 timeout -k 10 120 python3 scripts/fused_balance.py > $O/balance_256.txt 2>&1 || exit 3
cat $O/balance_512.txt $O/balance_256.txt
for rep in 1 2; do
  timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
  VX_BA_FUSED_THREADS=256 timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
  VX_BA_ATOMIC_ROWS=1 timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
done
cut -c1-160 $O/alone.txt
for v in default 256 atomic; do
  case $v in
    default) E="" ;;
    256) E="VX_BA_FUSED_THREADS=256" ;;
    atomic) E="VX_BA_ATOMIC_ROWS=1" ;;
  esac
  ( [ -n "$E" ] && export "$E"; timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/ba_alone.py > $O/kt_$v.log 2>&1 ) || { tail -20 $O/kt_$v.log; exit 5; }
  python3 scripts/ba_iter_durations.py "$(find $O/kt_$v -name 'kt_kernel_trace.csv' | head -1)" > $O/durations_$v.txt 2>&1
  rm -f $(find $O/kt_$v -name '*.csv')
  echo "== $v"; cat $O/durations_$v.txt
done
echo done
