#!/bin/bash
# round 5 (d): balanced pose-stage rounds (atomic row sums): LocalBA parity subset, per-launch
# durations, LocalBA alone, pipeline bench A/B against the slot sums
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_fused_build.py -m gpu -k "ba_ or graph_replay or seq or shard or layout" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 2; }
tail -1 $O/par.log
timeout -k 10 300 $T tests/test_gpu_stl_order.py tests/test_gpu_orb_stages.py tests/test_gpu_batch.py -m gpu > $O/orb.log 2>&1 || { tail -30 $O/orb.log; exit 2; }
tail -1 $O/orb.log
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_select.py > $O/ktrace_select.txt 2>&1 || { tail -20 $O/ktrace_select.txt; exit 9; }
VX_SEL_TAILN=0 VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_select.py > $O/ktrace_select_tailn0.txt 2>&1 || { tail -20 $O/ktrace_select_tailn0.txt; exit 9; }
head -10 $O/ktrace_select.txt
head -3 $O/ktrace_select_tailn0.txt
( timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/ba_alone.py > $O/kt.log 2>&1 ) || { tail -20 $O/kt.log; exit 5; }
python3 scripts/ba_iter_durations.py "$(find $O/kt -name 'kt_kernel_trace.csv' | head -1)" > $O/durations.txt 2>&1
rm -f $(find $O/kt -name '*.csv')
cat $O/durations.txt
for rep in 1 2; do
  timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
  VX_BA_ATOMIC_ROWS=0 timeout -k 10 120 python3 scripts/ba_alone.py >> $O/alone.txt 2>&1 || exit 4
done
cut -c1-100 $O/alone.txt
for rep in 1 2; do
  for v in 1 0; do
    VX_BA_ATOMIC_ROWS=$v timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-profile > $O/b_$v.$rep.json 2> $O/b_$v.$rep.err || { tail -20 $O/b_$v.$rep.err; exit 6; }
    python3 -c "import json; d=json.load(open('$O/b_$v.$rep.json')); print('atomic=$v', $rep, d['value'], d['latency_ms_per_frame'], d['host_enqueue_ms_per_step'])" | tee -a $O/bench_ab.txt
  done
done
for sh in 8x512 4x256 16x512 16x1024 8x512g256; do
  case $sh in
    8x512g256) E="VX_MATCH_GRID=256" ;;
    *) E="VX_MATCH_SHAPE=$sh" ;;
  esac
  ( export "$E"; timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/mt_$sh -o kt -- python3 scripts/match_alone.py 500 > $O/mt_$sh.log 2>&1 ) || { tail -20 $O/mt_$sh.log; exit 8; }
  echo "== $sh $(tail -1 $O/mt_$sh.log)"
  python3 scripts/kt_avg.py "$(find $O/mt_$sh -name 'kt_kernel_trace.csv' | head -1)" k_knn_rows k_knn_compact
  rm -f $(find $O/mt_$sh -name '*.csv')
done
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_ba.py > $O/ktrace.txt 2>&1 || { tail -20 $O/ktrace.txt; exit 7; }
head -30 $O/ktrace.txt
echo done
