#!/bin/bash
# bench.py C3 pipeline flag A/B on the final tree (300 steps each, alternating, three rounds):
# each argument is one flag set ("-" = defaults).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-flags}
for r in 1 2 3; do
  i=0
  for fl in "$@"; do
    i=$((i+1))
    [ "$fl" = "-" ] && fl=""
    timeout -k 10 150 python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-profile --no-drop-in $fl > gpurun_out/${TAG}_$i_$r.json 2> gpurun_out/${TAG}_$i_$r.err || { echo "bench [$fl] failed"; tail -20 gpurun_out/${TAG}_$i_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(f'{sys.argv[2]:28s}', d['value'], 'latency', d.get('latency_ms_per_frame'))" gpurun_out/${TAG}_$i_$r.json "[$fl]"
  done
done
