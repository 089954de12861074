#!/bin/bash
# round 6 (n): pinned snapshot arrays + single-sync fetch: the plan / adapter tests, then the phases
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${OUT:-r06n}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_adapters.py tests/test_gpu_dmap.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 2; }
tail -2 $O/t.txt
timeout -k 10 300 python3 -u scripts/adapter_timing.py 40 > $O/adapter_timing.txt 2>&1 || { tail -30 $O/adapter_timing.txt; exit 3; }
cat $O/adapter_timing.txt
