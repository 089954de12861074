#!/bin/bash
# round 5 (ar): the back-substitution with 32 tile groups a step (VX_SBA_BS_THREADS=512) against 16,
# alternating on one box: the bitwise test, then rocprofv3 kernel statistics and the plain bench of
# the connected C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ar}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sba.py -x -q --timeout 120 --timeout-method thread -k "multi_workgroup_factor_bitwise" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 2; }
tail -2 $O/test.log
for rep in 1 2; do
  for v in 512 256; do
    export VX_SBA_BS_THREADS=$v
    ( export SBA_CFGS=C5-connected; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v$rep -o kt -- python3 scripts/sba_bench.py 4 > $O/sbak_$v$rep.log 2>&1 ) || { tail -20 $O/sbak_$v$rep.log; exit 3; }
    python3 scripts/sba_gaps.py $O/kt_$v$rep > $O/kernels_$v$rep.txt 2>&1
    rm -rf $O/kt_$v$rep
    echo "== $v $rep"; grep -E "backsub|fac_blk|per iter|sba_solve" $O/kernels_$v$rep.txt | head -6
  done
done
for rep in 1 2; do
  for v in 512 256; do
    export VX_SBA_BS_THREADS=$v
    ( export SBA_CFGS=C5-connected; timeout -k 10 200 python3 scripts/sba_bench.py 20 > $O/sba_$v$rep.jsonl 2> $O/sba_$v$rep.err ) || { tail -20 $O/sba_$v$rep.err; exit 4; }
    echo "== bench $v $rep: $(grep -o '"ms_per_optimize": [0-9.]*' $O/sba_$v$rep.jsonl)"
  done
done
echo done
