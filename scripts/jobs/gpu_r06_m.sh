#!/bin/bash
# round 6 (m): snapshot LocalBA::Optimize phases with the plan build's upload marks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${OUT:-r06m}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/adapter_timing.py 40 > $O/adapter_timing.txt 2>&1 || { tail -30 $O/adapter_timing.txt; exit 2; }
cat $O/adapter_timing.txt
