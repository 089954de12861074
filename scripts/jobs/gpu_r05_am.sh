#!/bin/bash
# round 5 (am): owned graphs (LocalBA / Schur plans) with two alternating instances against one
# (VX_GRAPH_INSTANCES=1), alternating on one box: graph / BA tests, the C3 pipeline with the host's
# per-call times (VX_SEQ_TIMING).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05am}
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_dmap.py tests/test_gpu_batch.py tests/test_gpu_sba.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in 2 1; do
    VX_GRAPH_INSTANCES=$v VX_SEQ_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-profile > $O/b_$v.$rep.json 2> $O/b_$v.$rep.err || { tail -20 $O/b_$v.$rep.err; exit 6; }
    python3 -c "import json; d=json.load(open('$O/b_$v.$rep.json')); print('instances=$v', $rep, d['value'], d['host_enqueue_ms_per_step'], d['latency_ms_per_frame'])" | tee -a $O/bench_ab.txt
    grep "ba_run" $O/b_$v.$rep.err | tail -1 | tee -a $O/bench_ab.txt
  done
done
echo done
