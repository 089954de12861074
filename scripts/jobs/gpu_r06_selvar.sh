#!/bin/bash
# k_select_stl variants alone (rocprofv3 kernel stats of scripts/orb_loop.py, 300 C3 extractions),
# alternating over the libraries given as arguments ("-" = the tree), then the trace build's
# per-level phases (scripts/ktrace_select.py) and level 0's pass log (scripts/kpass_select.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-selvar}
for r in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset VX_LIB; name=tree; else export VX_LIB=visionx-slam_amd/lib/$lib.so; name=$lib; fi
    d=gpurun_out/${TAG}_${name}_$r
    VX_ORB_LOOP_N=300 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/orb_loop.py ${ORB_CFG} > $d.log 2>&1 || { echo "$name failed"; tail -20 $d.log; exit 1; }
    python3 - $d/run_kernel_stats.csv $name <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_select_stl" in r["Name"]:
        print(f"{sys.argv[2]:18s} k_select_stl {float(r['AverageNs']) / 1e3:7.3f} us (min {float(r['MinNs']) / 1e3:7.3f})  x{r['Calls']}")
PY
    rm -f $d/run_kernel_trace.csv
  done
done
unset VX_LIB
if [ -n "${TRACE}" ]; then
  VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_select.py ${ORB_CFG} || exit 1
  VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/kpass_select.py || exit 1
fi
