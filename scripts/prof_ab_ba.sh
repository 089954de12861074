#!/bin/bash
# k_ba_iter average duration (rocprofv3 --kernel-trace --stats) of LocalBA alone: the in-tree library
# vs ab/libvxslam_base.so, alternating.  usage: bash scripts/prof_ab_ba.sh [reps] [n_kf n_lm n_streams]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
reps=${1:-2}; shift
win=${*:-50 20000 1}
mkdir -p gpurun_out
for r in $(seq $reps); do
  for lib in tree base; do
    d=gpurun_out/pab_${lib}_$r
    if [ $lib = base ]; then export VX_LIB=ab/libvxslam_base.so; else unset VX_LIB; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/ba_alone.py $win > /dev/null 2>&1 || exit 1
    python3 - "$d/run_kernel_stats.csv" $lib <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_ba_iter" in r["Name"]:
        kind = "prologue" if "<true" in r["Name"] else "iter"
        print(f"{sys.argv[2]:5s} {kind:8s} {float(r['AverageNs']) / 1e3:7.3f} us  x{r['Calls']}")
PY
  done
done
