set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dmap.py > gpurun_out/dmap_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_build_time.py > gpurun_out/plan_build_time.json 2> gpurun_out/plan_build_time.err
