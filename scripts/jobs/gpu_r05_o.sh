#!/bin/bash
# round 5 (o): k_knn_rows shape x grid sweep on the C3 frame pair (kernel trace, parity checked by
# match_alone.py on every run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
for sh in 8x512 4x256 8x256 4x128; do
  for g in 256 512 0; do
    ( export VX_MATCH_SHAPE=$sh VX_MATCH_GRID=$g; timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/mt -o kt -- python3 scripts/match_alone.py 500 > $O/mt.log 2>&1 ) || { tail -20 $O/mt.log; exit 8; }
    echo "$sh grid $g: $(python3 scripts/kt_avg.py "$(find $O/mt -name 'kt_kernel_trace.csv' | head -1)" k_knn_rows | tr '\n' ' ') $(grep -h '^match' $O/mt.log | sed 's/.*]: //')" | tee -a $O/sweep.txt
    rm -rf $O/mt
  done
done
echo done
