#!/bin/bash
# round 6 (j): fault-path tests; the persistent window in the pipeline from a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06j}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dmap.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fault or dmap_plan or ba_base" > $O/t_fault.txt 2>&1 || { tail -30 $O/t_fault.txt; exit 2; }
tail -2 $O/t_fault.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-drop-in > $O/kt.json 2> $O/kt.log || { tail -20 $O/kt.log; exit 3; }
python3 scripts/win_pipeline_gaps.py $O/kt > $O/win_gaps.txt 2>&1 || { cat $O/win_gaps.txt; exit 4; }
rm -rf $O/kt
cat $O/win_gaps.txt
timeout -k 10 300 python scripts/adapter_timing.py 20 > $O/adapter_timing.txt 2>&1 || { tail -30 $O/adapter_timing.txt; exit 6; }
cat $O/adapter_timing.txt
echo done
