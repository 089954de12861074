#!/bin/bash
# round 5 (v): kernel trace of the connected C5 Schur bench — per-kernel durations and the gaps
# between the solve's launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05v}
mkdir -p $O
( export SBA_CFGS=C5-connected; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/sba_bench.py 3 > $O/prof.log 2>&1 ) || { tail -20 $O/prof.log; exit 3; }
python3 scripts/sba_gaps.py $O/prof > $O/sba_gaps.txt 2>&1 || { tail -20 $O/sba_gaps.txt; exit 4; }
cat $O/sba_gaps.txt
echo done
