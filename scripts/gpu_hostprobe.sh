# host CPU quota facts of a GPU box around C2 bench runs: cgroup throttling deltas and what else runs
set -o pipefail
mkdir -p gpurun_out/r04p
stat() { tr '\n' ' ' < /sys/fs/cgroup/cpu.stat | awk '{print $2, $12, $14}'; }
procs() { for p in $(cat /sys/fs/cgroup/cgroup.procs); do [ -r /proc/$p/stat ] && awk '{printf "%s %s %s %s | ", $1, $2, $14, $15}' /proc/$p/stat; done; echo; }
procs > gpurun_out/r04p/procs_start.txt
for i in 1 2 3; do
  a=$(stat)
  ( for k in $(seq 1 12); do sleep 0.5; procs; done ) > gpurun_out/r04p/procs_run$i.txt 2>&1 &
  sp=$!
  VX_SEQ_TIMING=1 timeout -k 10 150 python -u bench.py --config C2 --steps 400 --warmup 20 --no-cpu-baseline --no-profile > gpurun_out/r04p/c2_$i.json 2> gpurun_out/r04p/c2_$i.err || exit 4
  b=$(stat)
  wait $sp
  python3 -c "import json; d=json.load(open('gpurun_out/r04p/c2_$i.json')); print('run $i', d['value'], d['host_enqueue_ms_per_step'], 'cpu.stat usage/nr_throttled/throttled_usec before: $a after: $b')"
done
