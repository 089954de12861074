#!/bin/bash
# A/B of LocalBA alone: the in-tree library vs ab/libvxslam_base.so, alternating, per window.
# usage: bash scripts/ab_ba_alone.sh [reps]
set -o pipefail
reps=${1:-3}
for w in "50 20000 1" "100 50000 1" "400 160000 8"; do
  for r in $(seq $reps); do
    echo -n "new  "; timeout -k 10 120 python scripts/ba_alone.py $w | cut -c1-60 || exit 1
    echo -n "base "; VX_LIB=ab/libvxslam_base.so timeout -k 10 120 python scripts/ba_alone.py $w | cut -c1-60 || exit 1
  done
done
