#!/bin/bash
# round 6 (g): k_ba_win hand-off variants, LocalBA alone: wave-by-wave vs barrier signalling x
# poll spacing (s_sleep naps), and the per-iteration launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06g}
mkdir -p $O
for r in 1 2; do
  for ws in 0 1; do
    for nap in 1 4 16; do
      VX_BA_WIN_WSIG=$ws VX_BA_WIN_NAPS=$nap timeout -k 10 120 python scripts/ba_alone.py >> $O/alone.txt 2>&1 || { tail -5 $O/alone.txt; exit 4; }
    done
  done
  VX_BA_PERSIST=0 timeout -k 10 120 python scripts/ba_alone.py >> $O/alone.txt 2>&1 || { tail -5 $O/alone.txt; exit 4; }
done
cut -c1-120 $O/alone.txt
echo done
