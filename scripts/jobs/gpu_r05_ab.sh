#!/bin/bash
# round 5 (ab): the C++ drop-in's landmark write-back with and without software prefetch
# (VX_WB_PREFETCH), alternating on one box: adapter GPU tests, per-call phases of both modes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ab}
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_cpp_adapters.py -m gpu > $O/adapter_tests.log 2>&1 || { tail -40 $O/adapter_tests.log; exit 2; }
tail -1 $O/adapter_tests.log
for rep in 1 2 3; do
  for v in 1 0; do
    echo "== prefetch $v rep $rep" >> $O/timing.txt
    VX_WB_PREFETCH=$v timeout -k 10 200 python3 scripts/adapter_timing.py 40 >> $O/timing.txt 2>&1 || { tail -20 $O/timing.txt; exit 3; }
  done
done
cat $O/timing.txt
echo done
