#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmcprobe2
mkdir -p $O
timeout -k 10 120 python3 scripts/perkf_probe.py > $O/plain.log 2>&1; echo "plain rc=$?"; tail -2 $O/plain.log
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/b -o run -- python3 scripts/perkf_probe.py > $O/b.log 2>&1; echo "pmc persist=1 rc=$?"
grep -v "^W\|^E" $O/b.log | tail -12 | cut -c1-200
VX_BA_PERSIST=0 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/a -o run -- python3 scripts/perkf_probe.py > $O/a.log 2>&1; echo "pmc persist=0 rc=$?"
grep -v "^W\|^E" $O/a.log | tail -4 | cut -c1-200
rm -rf $O/a $O/b
echo done
