#!/bin/bash
# round 5 (as): k_sba_blocks at three waves per SIMD (__launch_bounds__(256, 3): 168 VGPRs, spills)
# against two (206 VGPRs), alternating on one box (VX_LIB=.../libvxslam_lb3.so): kernel statistics
# and the plain Schur bench over C3 / C5 / the connected C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05as}
mkdir -p $O
for rep in 1 2; do
  for v in lb3 cur; do
    if [ $v = lb3 ]; then export VX_LIB=visionx-slam_amd/lib/libvxslam_lb3.so; else unset VX_LIB; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v$rep -o kt -- python3 scripts/sba_bench.py 4 > $O/sbak_$v$rep.log 2>&1 || { tail -20 $O/sbak_$v$rep.log; exit 3; }
    python3 scripts/sba_gaps.py $O/kt_$v$rep > $O/kernels_$v$rep.txt 2>&1
    rm -rf $O/kt_$v$rep
    echo "== $v $rep"; grep -E "k_sba_blocks " $O/kernels_$v$rep.txt | head -3
    timeout -k 10 200 python3 scripts/sba_bench.py 20 > $O/sba_$v$rep.jsonl 2> $O/sba_$v$rep.err || { tail -20 $O/sba_$v$rep.err; exit 4; }
    echo "   bench: $(grep -o '"ms_per_optimize": [0-9.]*' $O/sba_$v$rep.jsonl | tr '\n' ' ')"
  done
done
echo done
