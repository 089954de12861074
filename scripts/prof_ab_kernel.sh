#!/bin/bash
# Average duration (rocprofv3 --kernel-trace --stats) of one kernel in bench.py's default pipeline:
# the in-tree library vs ab/libvxslam_base.so, alternating.
# usage: bash scripts/prof_ab_kernel.sh <kernel-name-substring> [reps]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
k=$1; reps=${2:-2}
mkdir -p gpurun_out
for r in $(seq $reps); do
  for lib in tree base; do
    d=gpurun_out/pabk_${lib}_$r
    if [ $lib = base ]; then export VX_LIB=ab/libvxslam_base.so; else unset VX_LIB; fi
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-profile > /dev/null 2>&1 || exit 1
    python3 - "$d/run_kernel_stats.csv" "$lib" "$k" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[3] in r["Name"]:
        print(f"{sys.argv[2]:5s} {r['Name'][:40]:40s} {float(r['AverageNs']) / 1e3:7.3f} us  x{r['Calls']}")
PY
  done
done
