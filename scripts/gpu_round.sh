#!/bin/bash
# Round-end style check: the whole GPU test suite as the driver runs it, then the committed
# measurements (scripts/gpu_bench.sh).  Stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash scripts/gpu_bench.sh
