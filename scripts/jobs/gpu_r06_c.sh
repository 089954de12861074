#!/bin/bash
# round 6 (c): the C++ drop-in's per-call phases on this box (resident and snapshot), for VERDICT r5 #5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06c}
mkdir -p $O
timeout -k 10 300 python scripts/adapter_timing.py 20 > $O/adapter_timing.txt 2>&1 || { tail -30 $O/adapter_timing.txt; exit 2; }
cat $O/adapter_timing.txt
