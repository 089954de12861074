#!/bin/bash
# round 5 (bb): Schur kernel statistics at C3 and C5 with the blocked factor as the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05bb}
mkdir -p $O
for cfg in C3 C5; do
  ( export SBA_CFGS=$cfg; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$cfg -o kt -- python3 scripts/sba_bench.py 4 > $O/sbak_$cfg.log 2>&1 ) || { tail -20 $O/sbak_$cfg.log; exit 3; }
  python3 scripts/sba_gaps.py $O/kt_$cfg > $O/kernels_$cfg.txt 2>&1
  rm -rf $O/kt_$cfg
  echo "== $cfg"; grep -v -- "->" $O/kernels_$cfg.txt | head -14
done
echo done
