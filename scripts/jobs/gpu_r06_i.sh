#!/bin/bash
# round 6 (i): k_ba_win register budget: 2 vs 3 waves per SIMD (VX_BA_WIN_WAVES), alone and in the
# C3 pipeline, against the per-iteration launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "ba_ or frontend" > $O/t_parity.txt 2>&1 || { tail -40 $O/t_parity.txt; exit 2; }
tail -2 $O/t_parity.txt
for r in 1 2; do
  for v in 2 3; do
    VX_BA_WIN_WAVES=$v timeout -k 10 120 python scripts/ba_alone.py >> $O/alone.txt 2>&1 || { tail -5 $O/alone.txt; exit 4; }
  done
done
cut -c1-90 $O/alone.txt
timeout -k 10 900 bash scripts/ab_env.sh 3 VX_BA_WIN_WAVES 2 3 > $O/ab_bench.txt 2>&1 || { cat $O/ab_bench.txt; exit 5; }
cat $O/ab_bench.txt
echo done
