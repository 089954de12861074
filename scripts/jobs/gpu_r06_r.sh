#!/bin/bash
# round 6 (r): vx_ba_optimize_map through the lean one-call build on the loaded view
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${OUT:-r06r}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_adapters.py tests/test_gpu_dmap.py tests/test_gpu_sharded.py tests/test_gpu_sba.py -x -q --timeout 120 --timeout-method thread > $O/t.txt 2>&1 || { tail -40 $O/t.txt; exit 2; }
tail -2 $O/t.txt
timeout -k 10 400 python3 -u scripts/adapter_ab.py VX_OPTMAP_LEAN 6 100 0 > $O/ab_lean.txt 2>&1 || { tail -30 $O/ab_lean.txt; exit 3; }
tail -4 $O/ab_lean.txt
timeout -k 10 300 python3 -u scripts/adapter_timing.py 40 > $O/adapter_timing.txt 2>&1 || { tail -30 $O/adapter_timing.txt; exit 4; }
cat $O/adapter_timing.txt
