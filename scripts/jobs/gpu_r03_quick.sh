#!/bin/bash
# Quick loop: ORB order / stage parity tests, then a short bench + rocprofv3 kernel stats (TAG).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-q}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stl_order.py tests/test_gpu_orb_stages.py ${EXTRA_TESTS} > gpurun_out/quick_tests_${TAG}.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/quick_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/quick_tests_${TAG}.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 300 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
f=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/kernel_stats_${TAG}.csv
python3 - <<PY
import csv
for r in list(csv.DictReader(open("gpurun_out/kernel_stats_${TAG}.csv")))[:10]:
    n = r["Name"].split("(")[0].replace("vx::(anonymous namespace)::", "")[:40]
    print(f"{n:40s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} us")
PY
grep -o '"value": [0-9.]*' gpurun_out/prof_${TAG}.log | head -1
