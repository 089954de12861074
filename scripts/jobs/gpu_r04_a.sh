#!/bin/bash
# round 4: resident one-call LocalBA (ba_lean.hip) — its GPU tests, the adapter tests and a short bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_dmap.py \
    tests/test_cpp_adapters.py -m gpu > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
