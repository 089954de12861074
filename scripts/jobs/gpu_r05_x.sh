#!/bin/bash
# round 5 (x): A/B of Schur factor builds on one box (alternating), the connected C5 Schur bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05x}
mkdir -p $O
for rep in 1 2; do
  for v in ${VARIANTS:-head en gate}; do
    ( export SBA_CFGS=C5-connected VX_LIB=visionx-slam_amd/lib/libvxslam_$v.so; timeout -k 10 200 python3 scripts/sba_bench.py 10 > $O/sba_$v.$rep.jsonl 2>&1 ) || { tail -20 $O/sba_$v.$rep.jsonl; exit 6; }
    python3 -c "
import json
for l in open('$O/sba_$v.$rep.jsonl'):
    d = json.loads(l); print('$v', $rep, d['ms_per_optimize'], d['kernel_us_per_iteration'])"
  done
done
echo done
