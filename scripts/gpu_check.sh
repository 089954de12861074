#!/bin/bash
# GPU parity tests, then a short bench with per-kernel stats.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-dev}
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/tests_${TAG}.log 2>&1
rc=$?; tail -15 gpurun_out/tests_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json; grep stage gpurun_out/bench_${TAG}.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
python3 - <<'PY'
import csv, os, re
tag = os.environ.get("TAG", "dev")
rows = list(csv.DictReader(open(f"gpurun_out/prof_{tag}/run_kernel_stats.csv")))
for r in rows:
    m = re.search(r"\b(k_[a-z0-9_]+)(?:<[^>(]*>)?\(", r["Name"]) 
    print(f"{(m.group(1) if m else r['Name'][:30]):22s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.2f} pct {float(r['Percentage']):6.2f}")
PY
