#!/bin/bash
# round 6 (h): the whole GPU suite + smoke on k_ba_win as the default, then the C3 pipeline with the
# persistent window vs the per-iteration launches, three alternating pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 2; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 3; }
tail -3 $O/smoke.txt
timeout -k 10 900 bash scripts/ab_env.sh 3 VX_BA_PERSIST 1 0 > $O/ab_bench.txt 2>&1 || { cat $O/ab_bench.txt; exit 5; }
cat $O/ab_bench.txt
echo done
