#!/bin/bash
# round 5 (ay): one tile per look-ahead workgroup (the new default): the Schur GPU tests, the Schur
# bench over every config, and the connected C5's kernel statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ay}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sba.py -x -v --timeout 120 --timeout-method thread > $O/test_sba.log 2>&1 || { tail -30 $O/test_sba.log; exit 2; }
tail -1 $O/test_sba.log
timeout -k 10 300 python3 scripts/sba_bench.py > $O/sba_bench.jsonl 2> $O/sba_bench.err || { tail -20 $O/sba_bench.err; exit 3; }
python3 -c "
import json,sys
for l in open('$O/sba_bench.jsonl'):
    d=json.loads(l); print(d['config'], d['ms_per_optimize'], d.get('kernel_us_per_iteration'))"
( export SBA_CFGS=C5-connected; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 scripts/sba_bench.py 4 > $O/sbak.log 2>&1 ) || { tail -20 $O/sbak.log; exit 4; }
python3 scripts/sba_gaps.py $O/kt > $O/kernels.txt 2>&1
cp $O/kt/*kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || find $O/kt -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/kt
grep -v -- "->" $O/kernels.txt | head -14
echo done
