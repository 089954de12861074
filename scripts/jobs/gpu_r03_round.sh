#!/bin/bash
# Round-3 session (TAG): the whole GPU suite, the k_select_stl phase trace (C3, C4), then the
# default bench, the driver's short command three times and a rocprofv3 kernel-stats pass.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -2 gpurun_out/gpu_tests_${TAG}.log
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_select.py > gpurun_out/ktrace_select_${TAG}.txt 2>&1 || { echo "ktrace failed"; tail -20 gpurun_out/ktrace_select_${TAG}.txt; exit 1; }
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_select.py C4 >> gpurun_out/ktrace_select_${TAG}.txt 2>&1 || { echo "ktrace C4 failed"; tail -20 gpurun_out/ktrace_select_${TAG}.txt; exit 1; }
cat gpurun_out/ktrace_select_${TAG}.txt
TAG=$TAG bash scripts/gpu_r03_bench.sh
