#!/bin/bash
# round 5 (aq): HBM traffic per kernel of the connected C5 Schur bench (two separate rocprofv3 --pmc
# passes, FETCH_SIZE and WRITE_SIZE; MI355X_MICROARCH.md corrections applied by the summary).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05aq}
mkdir -p $O
export SBA_CFGS=C5-connected
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 scripts/sba_bench.py 2 > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 2; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 scripts/sba_bench.py 2 > $O/w.log 2>&1 || { tail -20 $O/w.log; exit 3; }
python3 scripts/pmc_kernel_bytes.py "$(find $O/f -name '*counter_collection.csv' | head -1)" "$(find $O/w -name '*counter_collection.csv' | head -1)" > $O/sba_pmc.txt 2>&1
rm -rf $O/f $O/w
cat $O/sba_pmc.txt
echo done
