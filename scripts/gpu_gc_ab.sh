# the driver's 20-step command with the cyclic collection before the pre-timing sync (default) or
# after it (VX_BENCH_GC_LATE=1, the earlier order), alternating; outputs under gpurun_out/$TAG
TAG=${TAG:-r04gc}
mkdir -p gpurun_out/$TAG
for round in 1 2 3 4; do
  for late in 0 1; do
    VX_BENCH_GC_LATE=$late timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/s20_late${late}_$round.json 2> gpurun_out/$TAG/s20_late${late}_$round.err || exit 4
    python3 -c "
import json
b=json.load(open('gpurun_out/$TAG/s20_late${late}_$round.json'))
print('late=$late round $round s20', b['value'], b['host_enqueue_ms_per_step'], b['ms_per_step'])"
  done
done
