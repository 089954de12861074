#!/bin/bash
# LocalBA alone for several builds of the library: bash scripts/ab_libs.sh "n_kf n_lm streams" reps lib...
# (a lib of "-" is the in-tree build)
set -o pipefail
w=$1; reps=$2; shift 2
for r in $(seq $reps); do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset VX_LIB; name=tree; else export VX_LIB=$lib; name=$(basename $lib .so); fi
    echo -n "$name "; timeout -k 10 120 python scripts/ba_alone.py $w | cut -c1-60 || exit 1
  done
done
