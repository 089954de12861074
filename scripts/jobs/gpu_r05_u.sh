#!/bin/bash
# round 5 (u): potrf with row j's permutes ahead of the pivot's square root: bitwise / parity tests of
# the Schur forms, the blocked factor's phases (trace build), the connected C5 Schur bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05u}
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_sba.py -m gpu > $O/sba_tests.log 2>&1 || { tail -40 $O/sba_tests.log; exit 2; }
tail -1 $O/sba_tests.log
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_sba_blk.py > $O/ktrace_sba_blk.txt 2>&1 || { tail -20 $O/ktrace_sba_blk.txt; exit 9; }
cat $O/ktrace_sba_blk.txt
( export SBA_CFGS=${SBA_CFGS:-C5-connected}; timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench.jsonl 2>&1 ) || { tail -20 $O/sba_bench.jsonl; exit 6; }
python3 -c "
import json
for l in open('$O/sba_bench.jsonl'):
    d = json.loads(l); print(d['config'], d['ms_per_optimize'], d['kernel_us_per_iteration'], d['mfma_fp64']['fp64_frac'])"
echo done
