#!/bin/bash
# round 6: the default 2000-step command and the driver's 20-step command, three runs each, on the final tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${OUT:-r06dist}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 600 python3 bench.py --no-cpu-baseline > $O/long_$i.json 2> $O/long_$i.err || { tail -20 $O/long_$i.err; exit 2; }
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || { tail -20 $O/driver_$i.err; exit 3; }
  python3 -c "
import json
a=json.loads(open('$O/long_$i.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1])
print('$i 2000-step', a['value'], a['latency_ms_per_frame'], '| 20-step', b['value'], b['latency_ms_per_frame'], b['per_keyframe_ms']['cpp_adapter']['snapshot'], b['per_keyframe_ms']['cpp_adapter']['resident'])"
done
