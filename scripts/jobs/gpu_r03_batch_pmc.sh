#!/bin/bash
# HBM traffic of the batched extraction (TAG): FETCH_SIZE and WRITE_SIZE passes over
# scripts/batch_one.py 32 C3 (one launch per kernel for 32 frames) -> per-kernel bytes per launch.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-bp}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/bpmc_fetch_${TAG} -o run -- python3 scripts/batch_one.py 32 C3 10 > gpurun_out/bpmc_fetch_${TAG}.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/bpmc_fetch_${TAG}.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/bpmc_write_${TAG} -o run -- python3 scripts/batch_one.py 32 C3 10 > gpurun_out/bpmc_write_${TAG}.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/bpmc_write_${TAG}.log; exit 1; }
python3 scripts/pmc_summary.py "$(find gpurun_out/bpmc_fetch_${TAG} -name '*counter_collection.csv' | head -1)" \
    "$(find gpurun_out/bpmc_write_${TAG} -name '*counter_collection.csv' | head -1)" gpurun_out/batch_pmc_traffic_${TAG}.json \
    > gpurun_out/batch_pmc_traffic_${TAG}.txt || exit 1
rm -rf gpurun_out/bpmc_fetch_${TAG} gpurun_out/bpmc_write_${TAG}
cat gpurun_out/batch_pmc_traffic_${TAG}.txt
