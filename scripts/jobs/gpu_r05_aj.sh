#!/bin/bash
# round 5 (aj): Schur kernels of the current build against the previous one (VX_LIB=...head.so),
# alternating on one box: rocprofv3 kernel statistics of the connected C5 Schur bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05aj}
mkdir -p $O
for rep in 1 2; do
  for v in new head; do
    if [ $v = head ]; then export VX_LIB=visionx-slam_amd/lib/libvxslam_head.so; else unset VX_LIB; fi
    ( export SBA_CFGS=C5-connected; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v$rep -o kt -- python3 scripts/sba_bench.py 4 > $O/sba_$v$rep.log 2>&1 ) || { tail -20 $O/sba_$v$rep.log; exit 3; }
    python3 scripts/sba_gaps.py $O/kt_$v$rep > $O/kernels_$v$rep.txt 2>&1
    rm -rf $O/kt_$v$rep
    echo "== $v $rep"; head -8 $O/kernels_$v$rep.txt
  done
done
echo done
