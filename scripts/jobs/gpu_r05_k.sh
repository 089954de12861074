#!/bin/bash
# round 5 (k): the C++ drop-in's phases (results read in place), the dmap parity subset.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_dmap.py tests/test_cpp_adapters.py -m gpu > $O/dmap.log 2>&1 || { tail -30 $O/dmap.log; exit 2; }
tail -1 $O/dmap.log
timeout -k 10 300 python3 scripts/adapter_timing.py 20 > $O/adapter_timing.txt 2>&1 || { tail -20 $O/adapter_timing.txt; exit 3; }
cat $O/adapter_timing.txt
echo done
