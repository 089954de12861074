#!/bin/bash
# One GPU session: bench (N=1), kernel-trace stats, and separate PMC passes for HBM traffic.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed $?"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof failed $?"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || { echo "pmc fetch failed $?"; tail -30 gpurun_out/pmc_fetch_${TAG}.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${TAG} -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/pmc_write_${TAG}.log 2>&1 || { echo "pmc write failed $?"; tail -30 gpurun_out/pmc_write_${TAG}.log; exit 1; }
find gpurun_out -name "*.csv" | head -20
