#!/bin/bash
# round 5 (c): k_ba_iter phase trace (trace build) with the atomic row sums, C3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/r05c
mkdir -p $O
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_ba.py > $O/ktrace_atomic.txt 2>&1 || { tail -20 $O/ktrace_atomic.txt; exit 2; }
VX_BA_ATOMIC_ROWS=0 VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_ba.py > $O/ktrace_slots.txt 2>&1 || { tail -20 $O/ktrace_slots.txt; exit 2; }
head -40 $O/ktrace_atomic.txt
head -14 $O/ktrace_slots.txt
