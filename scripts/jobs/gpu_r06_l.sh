#!/bin/bash
# round 6 (l): the persistent window launched directly vs through its one-node graph (VX_BA_WIN_GRAPH):
# C3 pipeline, alternating, and the window gaps from a kernel trace of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06l}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "ba_ or seq or frontend" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 2; }
tail -1 $O/t.txt
timeout -k 10 900 bash scripts/ab_env.sh 2 VX_BA_WIN_GRAPH 0 1 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 3; }
cat $O/ab.txt
for v in 0 1; do
  VX_BA_WIN_GRAPH=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt$v -o run -- python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-drop-in > $O/kt$v.json 2> $O/kt$v.log || { tail -20 $O/kt$v.log; exit 4; }
  python3 scripts/win_pipeline_gaps.py $O/kt$v > $O/win_gaps_graph$v.txt 2>&1 || { cat $O/win_gaps_graph$v.txt; exit 5; }
  rm -rf $O/kt$v
  echo "VX_BA_WIN_GRAPH=$v"; head -6 $O/win_gaps_graph$v.txt
done
echo done
