set -o pipefail
mkdir -p gpurun_out/r04o
run() { # name env...
  name=$1; shift
  env "$@" VX_SEQ_TIMING=1 timeout -k 10 150 python -u bench.py --config C2 --steps 400 --warmup 20 --no-cpu-baseline --no-profile > gpurun_out/r04o/$name.json 2> gpurun_out/r04o/$name.err || return 4
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r04o/$name.json')); print('$name', d['value'], d['host_enqueue_ms_per_step'], d['ms_per_step'])"
  grep '\[vx_seq\]' gpurun_out/r04o/$name.err | tr -s ' ' | cut -d' ' -f2,5 | tr '\n' ' '; echo
}
run base A=1 && run sigpool ROC_SIGNAL_POOL_SIZE=4096 && run aql ROC_AQL_QUEUE_SIZE=65536 && run batch DEBUG_CLR_MAX_BATCH_SIZE=64 DEBUG_CLR_BATCH_CPU_SYNC_SIZE=64 && run active ROC_ACTIVE_WAIT_TIMEOUT=0 && run cpwait GPU_STREAMOPS_CP_WAIT=1 && run base2 A=1
