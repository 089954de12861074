#!/bin/bash
# round 5 (i): the blocked Schur factor with the pipelined look-ahead and the quad POTRF: bitwise / parity tests, its
# phases (trace build), the Schur bench blocked against one column per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_sba.py -m gpu -k "bitwise or connected" > $O/sba_tests.log 2>&1 || { tail -40 $O/sba_tests.log; exit 2; }
tail -1 $O/sba_tests.log
VX_LIB=visionx-slam_amd/lib/libvxslam_trace.so timeout -k 10 120 python3 scripts/ktrace_sba_blk.py > $O/ktrace_sba_blk.txt 2>&1 || { tail -20 $O/ktrace_sba_blk.txt; exit 9; }
cat $O/ktrace_sba_blk.txt
for f in block multi; do
  ( export VX_SBA_FACTOR=$f SBA_CFGS=C5-connected; timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench_$f.jsonl 2>&1 ) || { tail -20 $O/sba_bench_$f.jsonl; exit 6; }
  python3 -c "
import json
for l in open('$O/sba_bench_$f.jsonl'):
    d = json.loads(l); print('$f', d['config'], d['ms_per_optimize'], d['kernel_us_per_iteration'].get('sba_solve'), d['mfma_fp64']['fp64_frac'])"
done
echo done
