#!/bin/bash
# One GPU session for the committed measurements of a round (TAG):
#   1. two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) -> per-kernel HBM bytes
#      (scripts/pmc_summary.py, MI355X_MICROARCH.md corrections) -> profiles/pmc_traffic.json
#   2. bench.py (default N=1 command, with CPU baseline) -> the JSON line, traffic included
#   3. rocprofv3 --kernel-trace --stats of the same bench command -> per-kernel durations
# Every GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out profiles
TAG=${TAG:-r01}
P="--steps 20 --warmup 3 --no-cpu-baseline --no-profile"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o run -- python3 bench.py $P > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || { echo "pmc fetch failed"; tail -30 gpurun_out/pmc_fetch_${TAG}.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${TAG} -o run -- python3 bench.py $P > gpurun_out/pmc_write_${TAG}.log 2>&1 || { echo "pmc write failed"; tail -30 gpurun_out/pmc_write_${TAG}.log; exit 1; }
python3 scripts/pmc_summary.py "$(find gpurun_out/pmc_fetch_${TAG} -name '*counter_collection.csv' | head -1)" \
    "$(find gpurun_out/pmc_write_${TAG} -name '*counter_collection.csv' | head -1)" gpurun_out/pmc_traffic_${TAG}.json \
    > gpurun_out/pmc_traffic_${TAG}.txt || exit 1
cp gpurun_out/pmc_traffic_${TAG}.json profiles/pmc_traffic.json
rm -rf gpurun_out/pmc_fetch_${TAG} gpurun_out/pmc_write_${TAG}  # (raw counter CSVs: tens of MB)
cat gpurun_out/pmc_traffic_${TAG}.txt
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
rm -f gpurun_out/prof_${TAG}/*kernel_trace.csv  # (one row per launch: tens of MB; the stats stay)
find gpurun_out/prof_${TAG} -name "*kernel_stats.csv"
