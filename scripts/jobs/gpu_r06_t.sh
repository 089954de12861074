#!/bin/bash
# round 6 (t): single-workgroup scan pairs in the lean build; 16 pool threads on the L3 slice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${OUT:-r06t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_adapters.py tests/test_gpu_dmap.py tests/test_gpu_sharded.py tests/test_gpu_sba.py -x -q --timeout 120 --timeout-method thread > $O/t.txt 2>&1 || { tail -40 $O/t.txt; exit 2; }
tail -2 $O/t.txt
timeout -k 10 400 python3 -u scripts/adapter_ab.py VX_LEAN_ROCPRIM_SCAN 6 100 1 > $O/ab_scan.txt 2>&1 || { tail -30 $O/ab_scan.txt; exit 3; }
tail -4 $O/ab_scan.txt
