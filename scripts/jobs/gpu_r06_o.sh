#!/bin/bash
# round 6 (o): snapshot call with FlatMap's arrays page-locked vs pageable ($VX_HOST_PAGEABLE), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${OUT:-r06o}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 -u scripts/adapter_timing.py 40 > $O/pinned_$i.txt 2>&1 || { tail -30 $O/pinned_$i.txt; exit 2; }
  VX_HOST_PAGEABLE=1 timeout -k 10 300 python3 -u scripts/adapter_timing.py 40 > $O/pageable_$i.txt 2>&1 || { tail -30 $O/pageable_$i.txt; exit 3; }
  echo "round $i pinned:"; grep -A1 "^snapshot\|untimed\|flatten:\|optimize_map\|write-back" $O/pinned_$i.txt | grep -v "^--"
  echo "round $i pageable:"; grep -A1 "^snapshot\|untimed\|flatten:\|optimize_map\|write-back" $O/pageable_$i.txt | grep -v "^--"
done
