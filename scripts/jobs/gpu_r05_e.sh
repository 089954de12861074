#!/bin/bash
# round 5 (e): after dropping the balanced rounds / direct row reads: k_ba_iter durations, select
# A/B (gather record batches; $VX_SEL_SPEC, $VX_SEL_TAILN opt-in), matcher grid cap, then the whole
# GPU suite + smoke, the new bench modes (C4 --scaling strong, C5 Schur rig) at N = 1, the Schur
# bench with its MFMA fraction, and the C3 bench line with the C++ drop-in costs.
# Stops at the first GPU failure (test failures are reported and the run goes on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
TR=visionx-slam_amd/lib/libvxslam_trace.so
( timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/ba_alone.py > $O/kt.log 2>&1 ) || { tail -20 $O/kt.log; exit 5; }
python3 scripts/ba_iter_durations.py "$(find $O/kt -name 'kt_kernel_trace.csv' | head -1)" > $O/durations.txt 2>&1
rm -f $(find $O/kt -name '*.csv')
head -12 $O/durations.txt
for v in "" VX_SEL_SPEC=1 VX_SEL_TAILN=1; do
  ( [ -n "$v" ] && export "$v"; VX_LIB=$TR timeout -k 10 120 python3 scripts/ktrace_select.py > $O/ktrace_select_${v:-base}.txt 2>&1 ) || { tail -20 $O/ktrace_select_${v:-base}.txt; exit 9; }
  echo "== select ${v:-base}"; head -3 $O/ktrace_select_${v:-base}.txt
done
for g in cap VX_MATCH_FUSE=1 VX_MATCH_GRID=0 VX_MATCH_SHAPE=4x256; do
  ( [ "$g" != cap ] && export "$g"; timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/mt_$g -o kt -- python3 scripts/match_alone.py 500 > $O/mt_$g.log 2>&1 ) || { tail -20 $O/mt_$g.log; exit 8; }
  echo "== match $g $(grep -h '^match' $O/mt_$g.log)"
  python3 scripts/kt_avg.py "$(find $O/mt_$g -name 'kt_kernel_trace.csv' | head -1)" k_knn_rows k_knn_compact k_select_stl
  rm -f $(find $O/mt_$g -name '*.csv')
done
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
[ $rc -le 1 ] || { echo "gpu tests rc $rc"; tail -40 $O/gpu_tests.log; exit 2; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --config C4 --scaling strong --steps 200 --warmup 10 --no-cpu-baseline > $O/bench_c4_strong.json 2> $O/bench_c4_strong.err || { tail -20 $O/bench_c4_strong.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/bench_c4_strong.json')); print('C4 strong', d['value'], d['config']['workload'])"
timeout -k 10 300 python bench.py --config C5 --steps 60 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 5; }
python3 -c "import json; d=json.load(open('$O/bench_c5.json')); print('C5', d['value'], d['ms_per_rig_step'], d['roofline'], d['cpu_baseline'])"
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench.jsonl 2>&1 || { tail -20 $O/sba_bench.jsonl; exit 6; }
python3 -c "
import json
for l in open('$O/sba_bench.jsonl'):
    d = json.loads(l); print(d['config'], d['ms_per_optimize'], d['kernel_us_per_iteration'].get('sba_solve'), d['mfma_fp64'])"
timeout -k 10 600 python bench.py --steps 1000 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 7; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('C3', d['value'], d['latency_ms_per_frame'], d['per_keyframe_ms'], d['roofline'], d['cpu_baseline']['value'])"
echo done
