#!/bin/bash
# bench.py (C3) with the default library and the fused workgroup-size variants, twice each
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for lib in libvxslam.so libvxslam_ft512.so; do
    v=$(VX_LIB=visionx-slam_amd/lib/$lib timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stages_us'].get('ba_iter'), d['stages_us'].get('ba_prologue'))") || exit 1
    echo "$lib: frame, ba_iter us, prologue us = $v"
  done
done
VX_LIB=visionx-slam_amd/lib/libvxslam.so timeout -k 10 120 python scripts/ba_window_sweep.py 2>&1 | tail -14
