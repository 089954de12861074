#!/bin/bash
# bench.py over --streams 1/2/3, each with and without the timed-region HIP-event bracket
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-m}
for s in 3 2 1; do
  timeout -k 10 300 python bench.py --streams $s --no-cpu-baseline > gpurun_out/mx_${TAG}_s${s}.json 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --streams $s --no-cpu-baseline --no-profile > gpurun_out/mx_${TAG}_s${s}_np.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import json, glob, os
tag = os.environ.get("TAG", "m")
for f in sorted(glob.glob(f"gpurun_out/mx_{tag}_*.json")):
    d = json.load(open(f))
    r = d.get("roofline") or {}
    print(f"{os.path.basename(f):24s} value {d['value']:.4f} latency {d.get('latency_ms_per_frame')} dom {r.get('kernel')} {r.get('avg_launch_us')}")
PY
