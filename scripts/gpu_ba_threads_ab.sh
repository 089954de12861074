# LocalBA's fused workgroup size in the pipeline: the plan's choice (512 at C3) against 1024 threads
# ($VX_BA_FUSED_THREADS), alternating 1000-step C3 runs; outputs under gpurun_out/$TAG
TAG=${TAG:-r04bt}
mkdir -p gpurun_out/$TAG
for round in 1 2; do
  for t in auto 1024; do
    if [ $t = auto ]; then unset VX_BA_FUSED_THREADS; else export VX_BA_FUSED_THREADS=$t; fi
    timeout -k 10 200 python -u bench.py --steps 1000 --no-cpu-baseline --no-profile > gpurun_out/$TAG/c3_t${t}_$round.json 2> gpurun_out/$TAG/c3_t${t}_$round.err || exit 4
    python3 -c "
import json
b=json.load(open('gpurun_out/$TAG/c3_t${t}_$round.json'))
print('threads=$t round $round', b['value'], b['host_enqueue_ms_per_step'], b['ms_per_step'])"
  done
done
unset VX_BA_FUSED_THREADS
for t in 512 1024; do VX_BA_FUSED_THREADS=$t timeout -k 10 120 python3 scripts/ba_alone.py > gpurun_out/$TAG/alone_$t.txt 2>&1 || exit 4; tail -c 200 gpurun_out/$TAG/alone_$t.txt; echo; done
