#!/bin/bash
# k_pyramid tile / block sweep: ORB parity at two non-default tiles, then per-config stage time
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for t in 32 48; do
  VX_PYR_TILE=$t timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "orb" -p no:cacheprovider > gpurun_out/sweep_tests_$t.log 2>&1 || { tail -20 gpurun_out/sweep_tests_$t.log; exit 1; }
  tail -1 gpurun_out/sweep_tests_$t.log
done
for t in 32 40 48 64 96; do for b in 512 1024; do
  VX_PYR_TILE=$t VX_PYR_BLOCK=$b timeout -k 10 120 python bench.py --streams 1 --steps 30 --no-cpu-baseline > gpurun_out/sweep_${t}_${b}.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sweep_${t}_${b}.json')); print('tile $t block $b', d['stages_us'].get('orb_pyramid'), d['value'])"
done; done
