# the driver's 20-step command with 12 (default) against 24 frames per step, alternating, and one
# 2000-step run each; outputs under gpurun_out/$TAG
TAG=${TAG:-r04fps}
mkdir -p gpurun_out/$TAG
for round in 1 2 3; do
  for f in 12 24; do
    timeout -k 10 200 python -u bench.py --frames-per-step $f --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/s20_f${f}_$round.json 2> gpurun_out/$TAG/s20_f${f}_$round.err || exit 4
    python3 -c "
import json
b=json.load(open('gpurun_out/$TAG/s20_f${f}_$round.json'))
print('F=$f round $round s20', b['value'], b['host_enqueue_ms_per_step'], b['ms_per_step'])"
  done
done
for f in 12 24; do
  timeout -k 10 300 python -u bench.py --frames-per-step $f --no-cpu-baseline --no-profile > gpurun_out/$TAG/long_f$f.json 2> gpurun_out/$TAG/long_f$f.err || exit 4
  python3 -c "
import json
b=json.load(open('gpurun_out/$TAG/long_f$f.json'))
print('F=$f 2000 steps', b['value'], b['host_enqueue_ms_per_step'], b['ms_per_step'])"
done
