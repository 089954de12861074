#!/bin/bash
# round 5 (p): back-substitution prefetch depth 3 vs 6 (connected C5; kernel trace + Schur bench).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
VX_SBA_BS_DEPTH=6 timeout -k 10 400 $T tests/test_gpu_sba.py -m gpu -k "sba" > $O/sba_tests.log 2>&1 || { tail -40 $O/sba_tests.log; exit 2; }
tail -1 $O/sba_tests.log
for d in 3 6 3 6; do
  ( export VX_SBA_BS_DEPTH=$d SBA_CFGS=C5-connected; timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/sba_bench.py 6 > $O/kt.log 2>&1 ) || { tail -20 $O/kt.log; exit 5; }
  echo "depth $d: $(python3 scripts/kt_avg.py "$(find $O/kt -name 'kt_kernel_trace.csv' | head -1)" k_sba_backsub k_sba_fac_blk | tr '\n' ' ') $(python3 -c "import json; d=json.loads(open('$O/kt.log').readlines()[-1]); print(d['ms_per_optimize'], d['kernel_us_per_iteration'].get('sba_solve'))")" | tee -a $O/ab.txt
  rm -rf $O/kt
done
echo done
