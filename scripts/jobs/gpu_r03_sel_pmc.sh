#!/bin/bash
# Where k_select_stl's / k_test_retain's cycles go: wave-cycle breakdown (SQ: waiting on memory,
# waiting for instruction fetch, issuing) over 30 synchronous C3 extractions (scripts/orb_loop.py)
# and the retain probe (scripts/probe_retain.py).  One counter set per rocprofv3 pass.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-p}
CNT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for prog in orb_loop probe_retain; do
  timeout -s KILL 90 rocprofv3 --pmc $CNT --output-format csv -d gpurun_out/pmc_${TAG}_${prog} -o run -- python3 scripts/${prog}.py > gpurun_out/pmc_${TAG}_${prog}.log 2>&1 || { echo "pmc pass failed ($prog)"; tail -20 gpurun_out/pmc_${TAG}_${prog}.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_${TAG}_${prog} -o run -- python3 scripts/${prog}.py > gpurun_out/kt_${TAG}_${prog}.log 2>&1 || { echo "kt pass failed ($prog)"; exit 1; }
  python3 scripts/pmc_sq.py $(find gpurun_out/pmc_${TAG}_${prog} -name "*counter_collection.csv" | head -1) $(find gpurun_out/kt_${TAG}_${prog} -name "*kernel_trace.csv" | head -1)
done
