#!/bin/bash
# Selection A/B (round 6, session 2): the STL-order / stage / ORB parity tests on the tree, then
# k_select_stl's average duration (rocprofv3 kernel stats) for the tree and lib/libvxslam_base.so,
# alternating: extraction alone (scripts/orb_loop.py, 300 extractions) and bench.py's C3 pipeline.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-sel}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stl_order.py \
  tests/test_gpu_orb_stages.py tests/test_gpu_parity.py -k "orb or extract or stl or stage or retain or match" \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
stat() {  # $1 = csv, $2 = label
  python3 - "$1" "$2" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_select_stl" in r["Name"] or "k_fast" in r["Name"] or "k_describe" in r["Name"]:
        print(f"{sys.argv[2]:14s} {r['Name'].split('(')[0].split('::')[-1][:16]:16s} {float(r['AverageNs']) / 1e3:7.3f} us  x{r['Calls']}")
PY
}
for r in 1 2; do
  for lib in tree base; do
    if [ $lib = base ]; then export VX_LIB=visionx-slam_amd/lib/libvxslam_base.so; else unset VX_LIB; fi
    d=gpurun_out/${TAG}_alone_${lib}_$r
    VX_ORB_LOOP_N=300 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/orb_loop.py > $d.log 2>&1 || { echo "alone $lib failed"; tail -20 $d.log; exit 1; }
    stat $d/run_kernel_stats.csv "alone-$lib"; rm -f $d/run_kernel_trace.csv
    d=gpurun_out/${TAG}_pipe_${lib}_$r
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-profile > $d.log 2>&1 || { echo "pipe $lib failed"; tail -20 $d.log; exit 1; }
    stat $d/run_kernel_stats.csv "pipe-$lib"; rm -f $d/run_kernel_trace.csv
  done
done
unset VX_LIB
for r in 1 2; do
  for lib in tree base; do
    if [ $lib = base ]; then export VX_LIB=visionx-slam_amd/lib/libvxslam_base.so; else unset VX_LIB; fi
    timeout -k 10 120 python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-profile > gpurun_out/${TAG}_bench_${lib}_$r.json 2> gpurun_out/${TAG}_bench_${lib}_$r.err || { echo "bench $lib failed"; tail -20 gpurun_out/${TAG}_bench_${lib}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'latency', d.get('latency_ms_per_frame'))" gpurun_out/${TAG}_bench_${lib}_$r.json $lib
  done
done
