#!/bin/bash
# round 4: everything new (resident BA, seq bench, connected C5, Schur plan from the resident map,
# compacted pose stage) — GPU tests, A/B of the compacted pose stage, a short bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_dmap.py \
    tests/test_cpp_adapters.py tests/test_gpu_sba.py tests/test_gpu_parity.py tests/test_gpu_fused_build.py \
    tests/test_gpu_sharded.py -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
for i in 1 2; do
  for v in 0 1; do
    VX_BA_COMPACT=$v timeout -k 10 120 python -u scripts/ba_alone.py >> $O/ab_compact.txt 2>&1 || break 2
  done
done
timeout -k 10 400 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
