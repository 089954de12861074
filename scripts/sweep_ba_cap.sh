#!/bin/bash
# LocalBA alone at C3 for fused workgroup caps / sizes
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "50 20000 1" "100 50000 1"; do
  for env in "" "VX_BA_FUSED_CAP=384" "VX_BA_FUSED_CAP=256" "VX_BA_FUSED_THREADS=1024" "VX_BA_FUSED_THREADS=1024 VX_BA_FUSED_CAP=768" "VX_BA_FUSED=0"; do
    env $env timeout -k 10 60 python scripts/ba_alone.py $cfg || exit 1
  done
done
