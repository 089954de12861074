#!/bin/bash
# round 6 final check on the final tree: whole GPU suite + smoke, the driver's command x2, the C4 line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 2; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 3; }
tail -1 $O/smoke.txt
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || { tail -20 $O/driver_$i.err; exit 4; }
  python3 -c "import json; d=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1]); print('$i', d['value'], d.get('latency_ms_per_frame'), d['roofline']['frac'], d['per_keyframe_ms']['cpp_adapter'])"
done
timeout -k 10 600 python bench.py --config C4 --steps 200 --warmup 10 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 5; }
python3 -c "import json; d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1]); print('C4', d['value'], d['per_keyframe_ms'])" | cut -c1-400
echo done
