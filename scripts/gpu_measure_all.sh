#!/bin/bash
# One GPU session for a round's committed measurements (TAG): the GPU test suite, the PMC traffic
# passes + bench + rocprofv3 stats (scripts/gpu_bench.sh), the phase traces, the pipeline overlap
# probe, the LocalBA window sweep, extraction throughput, the C2 / C4 bench lines and the Schur BA
# bench.  Each GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
O=gpurun_out/m_${TAG}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
TAG=$TAG bash scripts/gpu_bench.sh > $O/gpu_bench.log 2>&1 || { echo "gpu_bench failed"; tail -30 $O/gpu_bench.log; exit 1; }
tail -3 $O/gpu_bench.log
export VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so
timeout -k 10 120 python -u scripts/ktrace_orb.py > $O/ktrace_orb_c3.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/ktrace_orb.py C4 > $O/ktrace_orb_c4.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/ktrace_ba.py > $O/ktrace_ba.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/ktrace_sba.py > $O/ktrace_sba.txt 2>&1 || exit 1
unset VX_LIB
timeout -k 10 300 python -u scripts/overlap_probe.py > $O/overlap_probe.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ba_window_sweep.py > $O/ba_window_sweep.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/extract_throughput.py > $O/extract_throughput_c3.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/extract_throughput.py C4 > $O/extract_throughput_c4.txt 2>&1 || exit 1
for c in C2 C4; do
  timeout -k 10 300 python bench.py --config $c --cpu-sample 10 > $O/bench_${c}.json 2> $O/bench_${c}.err || exit 1
done
timeout -k 10 300 python -u scripts/sba_bench.py > $O/sba_bench.json 2>&1 || exit 1
echo "all measurements done"
