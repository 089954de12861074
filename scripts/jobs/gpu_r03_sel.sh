#!/bin/bash
# Selection loop: the STL-order / stage parity tests, the retain primitive's kernel times per
# size (rocprofv3 stats of scripts/probe_retain.py, in call order), then the quick bench + stats.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-s}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stl_order.py tests/test_gpu_orb_stages.py ${EXTRA_TESTS} > gpurun_out/sel_tests_${TAG}.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sel_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/sel_tests_${TAG}.log
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/probe_${TAG} -o run -- python3 scripts/probe_retain.py > gpurun_out/probe_${TAG}.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/probe_${TAG}.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/probe_${TAG}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_test_retain" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sizes = ["64/40", "256/200", "307/244", "1024/500", "1868/868", "1868/868 u64"]
for i, sz in enumerate(sizes):
    d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[20 * i + 2:20 * i + 20])
    print(f"retain {sz:14s} median {d[len(d) // 2]:7.2f} us  min {d[0]:7.2f}")
PY
TAG=$TAG bash scripts/gpu_r03_quick_bench.sh
