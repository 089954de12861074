#!/bin/bash
# k_ba_iter HBM traffic per launch for LocalBA alone (C3): two --pmc passes (FETCH_SIZE, WRITE_SIZE)
# over scripts/ba_alone.py, summarised by scripts/pmc_summary.py.  usage: bash scripts/pmc_ba_alone.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-ba}
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$T -o run -- python3 scripts/ba_alone.py > gpurun_out/pmcf_$T.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$T -o run -- python3 scripts/ba_alone.py > gpurun_out/pmcw_$T.log 2>&1 || exit 1
python3 scripts/pmc_summary.py "$(find gpurun_out/pmcf_$T -name '*counter_collection.csv' | head -1)" \
    "$(find gpurun_out/pmcw_$T -name '*counter_collection.csv' | head -1)" gpurun_out/pmc_$T.json | grep k_ba_iter
