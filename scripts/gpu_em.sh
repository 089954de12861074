set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_essential.py tests/test_gpu_ransac.py tests/test_cpp_adapters.py > gpurun_out/em_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 200 python -u scripts/em_bench.py 20 > gpurun_out/em_bench.json 2> gpurun_out/em_bench.err
