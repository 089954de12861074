#!/bin/bash
# k_describe change check (TAG): the ORB parity files, batched throughput with its kernel stats, and
# the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stl_order.py tests/test_gpu_batch.py tests/test_gpu_orb_stages.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/orb_tests_${TAG}.log 2>&1 || { echo "orb tests failed"; tail -30 gpurun_out/orb_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/orb_tests_${TAG}.log
timeout -k 10 300 python3 scripts/batch_throughput.py gpurun_out/batch_throughput_${TAG}.json > gpurun_out/batch_throughput_${TAG}.txt 2>&1 || { echo "batch failed"; tail -20 gpurun_out/batch_throughput_${TAG}.txt; exit 1; }
cat gpurun_out/batch_throughput_${TAG}.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_batch_${TAG} -o run -- python3 scripts/batch_throughput.py gpurun_out/bt_prof_${TAG}.json > gpurun_out/prof_batch_${TAG}.log 2>&1 || { echo "batch prof failed"; exit 1; }
rm -f gpurun_out/prof_batch_${TAG}/run_kernel_trace.csv
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}.json')); print(d['value'], d['stages_us'])"
