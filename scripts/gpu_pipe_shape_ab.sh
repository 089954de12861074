# pipeline shape with the host pinned: extraction contexts E = 2 / 3 / 4 and the extraction grid
# share 0.2 / 0.25 / 0.33, alternating 1000-step C3 runs; outputs under gpurun_out/$TAG
TAG=${TAG:-r04shape}
mkdir -p gpurun_out/$TAG
for round in 1 2; do
  for v in e3 e2 e4 g20 g33; do
    case $v in e3) a="";; e2) a="--extract-ctx 2";; e4) a="--extract-ctx 4";; g20) a="--grid-share 0.2";; g33) a="--grid-share 0.33";; esac
    timeout -k 10 200 python -u bench.py --steps 1000 --no-cpu-baseline --no-profile $a > gpurun_out/$TAG/${v}_$round.json 2> gpurun_out/$TAG/${v}_$round.err || exit 4
    python3 -c "
import json
b=json.load(open('gpurun_out/$TAG/${v}_$round.json'))
print('$v round $round', b['value'], b['latency_ms_per_frame'], b['host_enqueue_ms_per_step'], b['ms_per_step'])"
  done
done
