# Host placement of the enqueueing process: C2 bench runs unpinned and pinned (taskset,
# before python starts) to the 8 least-busy logical CPUs of the whole host, of NUMA node 0 and of
# node 1 (busy = /proc/stat deltas over 0.5 s), two alternating rounds; per-call host costs from
# $VX_SEQ_TIMING.  Outputs under gpurun_out/$TAG.
TAG=${TAG:-r04pin}
mkdir -p gpurun_out/$TAG
pick() {  # pick NODE(-1 = any) -> comma list of the 8 idlest CPUs
python3 - "$1" <<'PY'
import sys, time
node = int(sys.argv[1])
def snap():
    d = {}
    for l in open("/proc/stat"):
        if l.startswith("cpu") and l[3].isdigit():
            f = l.split(); v = list(map(int, f[1:]))
            d[int(f[0][3:])] = (sum(v), v[3] + v[4])
    return d
a = snap(); time.sleep(0.5); b = snap()
busy = {c: 1 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) for c in b}
cpus = set(b)
if node >= 0:
    rng = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    cpus = set()
    for part in rng.split(","):
        x, _, y = part.partition("-"); cpus |= set(range(int(x), int(y or x) + 1))
best = sorted(cpus, key=lambda c: busy[c])[:8]
print(",".join(map(str, best)))
PY
}
for round in 1 2; do
  for mode in none any n0 n1; do
    if [ $mode = none ]; then pre=""; else
      n=-1; [ $mode = n0 ] && n=0; [ $mode = n1 ] && n=1
      cpus=$(pick $n); pre="taskset -c $cpus"; fi
    VX_SEQ_TIMING=1 timeout -k 10 150 $pre python -u bench.py --config C2 --steps 400 --warmup 20 --no-cpu-baseline --no-profile > gpurun_out/$TAG/${mode}_$round.json 2> gpurun_out/$TAG/${mode}_$round.err || exit 4
    python3 -c "
import json,re
d=json.load(open('gpurun_out/$TAG/${mode}_$round.json'))
t={}
for l in open('gpurun_out/$TAG/${mode}_$round.err'):
    m=re.match(r'\[vx_seq\] (\w+)\s+\d+ calls\s+([\d.]+)',l)
    if m: t.setdefault(m.group(1),[]).append(float(m.group(2)))
print('$mode round $round', '${pre}'[:40], d['value'], d['host_enqueue_ms_per_step'], {k: round(sum(v)/len(v),2) for k,v in t.items()})"
  done
done
