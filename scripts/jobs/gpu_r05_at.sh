#!/bin/bash
# round 5 (at): the reduced-system assembly as two launches on two streams (VX_SBA_BLOCKS_SPLIT=2: diagonal blocks
# beside the off-diagonal ones at 156 VGPRs / three waves per SIMD) against one (208 VGPRs, two waves),
# alternating on one box: the bitwise test, kernel statistics and the Schur bench (C3 / C5 / connected).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05at}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sba.py -x -q --timeout 120 --timeout-method thread -k "blocks_split_launch or diagonal_block_split" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 2; }
tail -1 $O/test.log
for rep in 1 2; do
  for v in 2 0; do
    export VX_SBA_BLOCKS_SPLIT=$v
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v$rep -o kt -- python3 scripts/sba_bench.py 4 > $O/sbak_$v$rep.log 2>&1 || { tail -20 $O/sbak_$v$rep.log; exit 3; }
    python3 scripts/sba_gaps.py $O/kt_$v$rep > $O/kernels_$v$rep.txt 2>&1
    rm -rf $O/kt_$v$rep
    echo "== split=$v $rep"; grep -E "k_sba_blocks" $O/kernels_$v$rep.txt | grep -v -- "->" | head -3
    timeout -k 10 200 python3 scripts/sba_bench.py 20 > $O/sba_$v$rep.jsonl 2> $O/sba_$v$rep.err || { tail -20 $O/sba_$v$rep.err; exit 4; }
    echo "   bench: $(grep -o '"ms_per_optimize": [0-9.]*' $O/sba_$v$rep.jsonl | tr '\n' ' ')"
  done
done
echo done
