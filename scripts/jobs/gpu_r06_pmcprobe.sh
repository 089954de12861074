#!/bin/bash
# round 6: does a rocprofv3 --pmc pass survive the persistent window?  LocalBA alone under one
# FETCH_SIZE pass, per-iteration launches first, then k_ba_win.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmcprobe
mkdir -p $O
VX_BA_PERSIST=0 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/a -o run -- python3 scripts/ba_alone.py > $O/a.log 2>&1; echo "persist=0 rc=$?"
tail -3 $O/a.log | cut -c1-200
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/b -o run -- python3 scripts/ba_alone.py > $O/b.log 2>&1; echo "persist=1 rc=$?"
tail -3 $O/b.log | cut -c1-200
grep -c k_ba_win $O/b/run_counter_collection.csv
rm -rf $O/a $O/b/*agent* 
echo done
