#!/bin/bash
# round 5 (g): the blocked Schur factor's phases (trace build), the matcher / select parity subset
# and the match alone after the compaction's first loads moved ahead of the count.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_stl_order.py tests/test_gpu_orb_stages.py tests/test_gpu_batch.py -m gpu -k "match or orb or stl or select or batch" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 2; }
tail -1 $O/par.log
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_sba_blk.py > $O/ktrace_sba_blk.txt 2>&1 || { tail -20 $O/ktrace_sba_blk.txt; exit 9; }
cat $O/ktrace_sba_blk.txt
( timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/mt -o kt -- python3 scripts/match_alone.py 500 > $O/mt.log 2>&1 ) || { tail -20 $O/mt.log; exit 8; }
grep -h '^match' $O/mt.log
python3 scripts/kt_avg.py "$(find $O/mt -name 'kt_kernel_trace.csv' | head -1)" k_knn_rows k_knn_compact k_select_stl
rm -f $(find $O/mt -name '*.csv')
echo done
