#!/bin/bash
# round 6 (ab): the fused packing cap (landmark-stage observations per 512-thread workgroup) for the
# persistent window: LocalBA alone, then the C3 pipeline at the two best
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06ab}
mkdir -p $O
for i in 1 2; do
  for v in 512 496 480 464 448 416; do
    VX_BA_FUSED_CAP=$v timeout -k 10 120 python3 scripts/ba_alone.py 2>&1 | python3 -c "import sys,re; t=sys.stdin.read(); m=re.search(r'([0-9.]+) ms/run.*workgroups.: (\d+)', t); print('CAP=$v', m.group(1) if m else t[-300:], m.group(2) if m else '')"
  done
done | tee $O/alone.txt
timeout -k 10 900 bash scripts/ab_env.sh 3 VX_BA_FUSED_CAP 512 480 448 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 4; }
cat $O/ab.txt
