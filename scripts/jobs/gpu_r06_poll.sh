#!/bin/bash
# k_ba_win poll depth A/B: LocalBA parity tests on the tree, then LocalBA alone (scripts/ba_alone.py,
# best of 3 x 100 windows) and the C3 pipeline (bench.py 300 steps) for the libraries given
# ("-" = the tree), alternating, three rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-poll}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dmap.py tests/test_gpu_sharded.py -k "ba or dmap or shard or win" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for r in 1 2 3; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset VX_LIB; name=tree; else export VX_LIB=visionx-slam_amd/lib/$lib.so; name=$lib; fi
    timeout -k 10 120 python3 scripts/ba_alone.py > gpurun_out/${TAG}_a.txt 2>&1 || { echo "alone $name failed"; tail -5 gpurun_out/${TAG}_a.txt; exit 1; }; echo "$name alone: $(cut -c1-40 gpurun_out/${TAG}_a.txt)"
    timeout -k 10 120 python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-profile --no-drop-in > gpurun_out/${TAG}_b_${name}_$r.json 2> gpurun_out/${TAG}_b_${name}_$r.err || { echo "bench $name failed"; tail -20 gpurun_out/${TAG}_b_${name}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'pipeline', d['value'], 'latency', d.get('latency_ms_per_frame'))" gpurun_out/${TAG}_b_${name}_$r.json $name
  done
done
