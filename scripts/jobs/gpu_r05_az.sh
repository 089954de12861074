#!/bin/bash
# round 5 (az): the blocked multi-workgroup factor (VX_SBA_FACTOR=block) against the default form at
# C3 (19 tile columns) and C5 (eight components of 10), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05az}
mkdir -p $O
export SBA_CFGS=C3,C5
for rep in 1 2; do
  for v in block default; do
    if [ $v = block ]; then export VX_SBA_FACTOR=block; else unset VX_SBA_FACTOR; fi
    timeout -k 10 200 python3 scripts/sba_bench.py 20 > $O/sba_${v}_$rep.jsonl 2> $O/sba_${v}_$rep.err || { tail -20 $O/sba_${v}_$rep.err; exit 4; }
    python3 -c "
import json
for l in open('$O/sba_${v}_$rep.jsonl'):
    d=json.loads(l); print('$v $rep', d['config'], d['ms_per_optimize'], d['kernel_us_per_iteration']['sba_solve'], d['factor'])"
  done
done
echo done
