#!/bin/bash
# round 5 final (a): the whole GPU suite and smoke() on the committed tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05fa}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -le 1 ] || { echo "gpu tests rc $rc"; tail -40 $O/gpu_tests.log; exit 2; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
tail -2 $O/smoke.log
echo done
