# the C3 pipeline with one element removed at a time (diagnostic lines, marked invalid): LocalBA not
# ordered after Match (--diag-nodep), without extraction / matching / LocalBA (--diag-skip), against
# the full pipeline; 1000-step runs, outputs under gpurun_out/$TAG
TAG=${TAG:-r04diag}
mkdir -p gpurun_out/$TAG
run() { name=$1; shift
  timeout -k 10 200 python -u bench.py --steps 1000 --no-cpu-baseline --no-profile "$@" > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || return 4
  python3 -c "
import json
b=json.load(open('gpurun_out/$TAG/$name.json'))
print('$name', b['value'], b['host_enqueue_ms_per_step'], b['ms_per_step'])"
}
run full && run nodep --diag-nodep && run skip_extract --diag-skip extract && run skip_match --diag-skip match && run skip_ba --diag-skip ba && run full2
