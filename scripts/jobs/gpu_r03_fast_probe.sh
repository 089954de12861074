#!/bin/bash
# Where k_fast's time goes (TAG): phase timestamps (trace build) on one C3 / C4 frame, and the SQ
# wave-cycle breakdown of the batched extraction (scripts/batch_one.py 32 C3).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-fp}
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_orb.py > gpurun_out/ktrace_orb_${TAG}.txt 2>&1 || { echo "ktrace failed"; tail -20 gpurun_out/ktrace_orb_${TAG}.txt; exit 1; }
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_orb.py C4 >> gpurun_out/ktrace_orb_${TAG}.txt 2>&1 || { echo "ktrace C4 failed"; exit 1; }
cat gpurun_out/ktrace_orb_${TAG}.txt
CNT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $CNT --output-format csv -d gpurun_out/pmc_${TAG}_b32 -o run -- python3 scripts/batch_one.py 32 C3 10 > gpurun_out/pmc_${TAG}_b32.log 2>&1 || { echo "pmc pass failed"; tail -20 gpurun_out/pmc_${TAG}_b32.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_${TAG}_b32 -o run -- python3 scripts/batch_one.py 32 C3 10 > gpurun_out/kt_${TAG}_b32.log 2>&1 || { echo "kt pass failed"; exit 1; }
python3 scripts/pmc_sq.py $(find gpurun_out/pmc_${TAG}_b32 -name "*counter_collection.csv" | head -1) $(find gpurun_out/kt_${TAG}_b32 -name "*kernel_trace.csv" | head -1)
