#!/bin/bash
# LocalBA alone (ba_window_sweep's C3 line) and the pipelined frame for fused workgroup caps
cd "$GRAFT_REPO_ROOT" || exit 1
for cap in 512 384 320 256 192; do
  v=$(VX_BA_FUSED_CAP=$cap timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stages_us'].get('ba_iter'), d['stages_us'].get('ba_prologue'))") || exit 1
  echo "cap $cap: frame, ba_iter us, prologue us = $v"
done
