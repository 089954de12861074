#!/bin/bash
# round 5 (av): tiles per look-ahead workgroup (VX_SBA_UPD_TILES, default 16) and per helper
# workgroup of the blocked factor (VX_SBA_BLK_TILES, default 32), swept on the connected C5,
# alternating; the bitwise factor test once with both changed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05av}
mkdir -p $O
( export VX_SBA_UPD_TILES=${TEST_UT:-8} VX_SBA_BLK_TILES=16 VX_SBA_UPD_THREADS=${TEST_TH:-512}; timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sba.py -x -q --timeout 120 --timeout-method thread -k "multi_workgroup_factor_bitwise" > $O/test.log 2>&1 ) || { tail -30 $O/test.log; exit 2; }
tail -1 $O/test.log
export SBA_CFGS=C5-connected
for rep in 1 2; do
  for v in ${SWEEP:-16:32 8:32 4:32 32:32 16:16 16:64}; do
    IFS=: read -r ut bt th <<< "$v"; export VX_SBA_UPD_TILES=$ut VX_SBA_BLK_TILES=$bt VX_SBA_UPD_THREADS=${th:-512}
    timeout -k 10 200 python3 scripts/sba_bench.py 20 > $O/sba_${v//:/_}_$rep.jsonl 2> $O/sba_${v//:/_}_$rep.err || { tail -20 $O/sba_${v//:/_}_$rep.err; exit 4; }
    echo "upd:blk $v rep $rep: $(grep -o '"ms_per_optimize": [0-9.]*' $O/sba_${v//:/_}_$rep.jsonl | tr '\n' ' ')"
  done
done
echo done
