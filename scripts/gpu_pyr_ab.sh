# the fused pyramid's shape in the pipeline: default (1024 threads, tile for 1/4 of the CUs) against
# 512-thread workgroups ($VX_PYR_BLOCK) and smaller tiles ($VX_PYR_TILE), alternating 1000-step C3
# runs; outputs under gpurun_out/$TAG
TAG=${TAG:-r04pyr}
mkdir -p gpurun_out/$TAG
for round in 1 2; do
  for v in ${VARIANTS:-def b512 t48 t40}; do
    unset VX_PYR_BLOCK VX_PYR_TILE
    case $v in b512) export VX_PYR_BLOCK=512;; t*) export VX_PYR_TILE=${v#t};; esac
    timeout -k 10 200 python -u bench.py --steps 1000 --no-cpu-baseline > gpurun_out/$TAG/${v}_$round.json 2> gpurun_out/$TAG/${v}_$round.err || exit 4
    python3 -c "
import json
b=json.load(open('gpurun_out/$TAG/${v}_$round.json'))
print('$v round $round', b['value'], b['latency_ms_per_frame'], b['stages_us'].get('orb_pyramid'), b['host_enqueue_ms_per_step'])"
  done
done
