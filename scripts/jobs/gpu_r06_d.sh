#!/bin/bash
# round 6 (d): k_ba_win revisions — BA parity tests, LocalBA alone and the C3 pipeline vs the
# per-iteration launches (VX_BA_PERSIST=0), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "ba_ or frontend" > $O/t_parity.txt 2>&1 || { tail -40 $O/t_parity.txt; exit 2; }
tail -2 $O/t_parity.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_dmap.py tests/test_gpu_fused_build.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > $O/t_more.txt 2>&1 || { tail -40 $O/t_more.txt; exit 3; }
tail -2 $O/t_more.txt
for r in 1 2 3; do
  for v in 1 0; do
    VX_BA_PERSIST=$v timeout -k 10 120 python scripts/ba_alone.py >> $O/alone.txt 2>&1 || { tail -5 $O/alone.txt; exit 4; }
  done
done
cut -c1-90 $O/alone.txt
timeout -k 10 600 bash scripts/ab_env.sh 2 VX_BA_PERSIST 1 0 > $O/ab_bench.txt 2>&1 || { cat $O/ab_bench.txt; exit 5; }
cat $O/ab_bench.txt
echo done
