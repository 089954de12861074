#!/bin/bash
# round 4: lean resident BA + seq bench (r04a) and the connected-C5 Schur solve
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_dmap.py \
    tests/test_cpp_adapters.py tests/test_gpu_sba.py -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
