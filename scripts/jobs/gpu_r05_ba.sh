#!/bin/bash
# round 5 (ba): the blocked factor as the default at every size: the whole GPU suite, smoke(), the C5
# bench line and the Schur bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ba}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { echo "gpu tests rc $rc"; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit 2; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --config C5 --steps 60 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 5; }
python3 -c "import json; d=json.load(open('$O/bench_c5.json')); print('bench_c5', d['value'], d.get('ms_per_step'))"
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench.jsonl 2> $O/sba_bench.err || { tail -20 $O/sba_bench.err; exit 6; }
python3 -c "
import json
for l in open('$O/sba_bench.jsonl'):
    d = json.loads(l); print(d['config'], d['ms_per_optimize'], d['kernel_us_per_iteration'].get('sba_solve'), d['mfma_fp64']['fp64_frac'], d['factor'])"
echo done
