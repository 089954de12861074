#!/bin/bash
# round 6 (v): the whole GPU suite + smoke on the current tree, then the driver's own command x3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06v}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 2; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 3; }
tail -3 $O/smoke.txt
for i in 1 2 3; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || { tail -20 $O/driver_$i.err; exit 4; }
  python3 -c "import json; d=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1]); print('$i', d['value'], d.get('latency_ms_per_frame'), d['roofline']['frac'], d.get('per_keyframe_ms'))"
done
echo done
