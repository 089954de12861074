#!/bin/bash
# round 6 (ag): the roofline's launch duration as the median of 5-step chunks: driver command x4 + contract tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${OUT:-r06ag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench_contract.py -x -q --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 2; }
tail -1 $O/t.txt
for i in 1 2 3 4; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || { tail -20 $O/driver_$i.err; exit 3; }
  python3 -c "import json; d=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$i', d['value'], r['avg_launch_us'], r['avg_launch_us_dominant_pass'], r['frac'], r['avg_launch_us_source'])"
done
