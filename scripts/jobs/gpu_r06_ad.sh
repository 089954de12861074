#!/bin/bash
# round 6 (ad): the driver's command with the drop-in subprocess on the whole affinity set
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${OUT:-r06ad}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || { tail -20 $O/driver_$i.err; exit 4; }
  python3 -c "import json; d=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1]); print('$i', d['value'], d.get('latency_ms_per_frame'), d['roofline']['frac'], d['per_keyframe_ms']['cpp_adapter'], d['config'].get('host_cpus'))" | cut -c1-400
done
