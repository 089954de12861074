# bench.py --pin-host auto against off, alternating (C3 default 2000-step runs and the driver's 20-step
# command), outputs under gpurun_out/$TAG
TAG=${TAG:-r04pab}
mkdir -p gpurun_out/$TAG
for round in 1 2 3; do
  for pin in auto off; do
    timeout -k 10 200 python -u bench.py --pin-host $pin --no-cpu-baseline > gpurun_out/$TAG/c3_${pin}_$round.json 2> gpurun_out/$TAG/c3_${pin}_$round.err || exit 4
    timeout -k 10 200 python -u bench.py --pin-host $pin --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/s20_${pin}_$round.json 2> gpurun_out/$TAG/s20_${pin}_$round.err || exit 4
    python3 -c "
import json
a=json.load(open('gpurun_out/$TAG/c3_${pin}_$round.json')); b=json.load(open('gpurun_out/$TAG/s20_${pin}_$round.json'))
print('$pin round $round', 'C3 2000', a['value'], a['host_enqueue_ms_per_step'], '| s20', b['value'], b['host_enqueue_ms_per_step'], a.get('host_cpus'))"
  done
done
