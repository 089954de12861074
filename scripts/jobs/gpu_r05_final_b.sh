#!/bin/bash
# round 5 final (b): committed measurements — PMC traffic passes, the bench line, the kernel-trace
# statistics of the same command (scripts/gpu_bench.sh, TAG=r05), then C4 --scaling strong, C5, the
# Schur bench and the LocalBA launch durations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ff}
mkdir -p $O
TAG=r05 bash scripts/gpu_bench.sh > $O/gpu_bench.log 2>&1 || { tail -30 $O/gpu_bench.log; exit 2; }
tail -5 $O/gpu_bench.log
timeout -k 10 300 python bench.py --config C4 --scaling strong --steps 200 --warmup 10 --no-cpu-baseline > $O/bench_c4_strong.json 2> $O/bench_c4_strong.err || { tail -20 $O/bench_c4_strong.err; exit 4; }
timeout -k 10 300 python bench.py --config C4 --steps 200 --warmup 10 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 4; }
timeout -k 10 300 python bench.py --config C5 --steps 60 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 5; }
timeout -k 10 300 python3 scripts/sba_bench.py 10 > $O/sba_bench.jsonl 2>&1 || { tail -20 $O/sba_bench.jsonl; exit 6; }
( timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/ba_alone.py > $O/kt.log 2>&1 ) || { tail -20 $O/kt.log; exit 7; }
python3 scripts/ba_iter_durations.py "$(find $O/kt -name 'kt_kernel_trace.csv' | head -1)" > $O/ba_iter_durations.txt 2>&1
rm -f $(find $O/kt -name '*.csv')
for f in bench_c4_strong bench_c4 bench_c5; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d.get('ms_per_step'))"; done
python3 -c "
import json
for l in open('$O/sba_bench.jsonl'):
    d = json.loads(l); print(d['config'], d['ms_per_optimize'], d['kernel_us_per_iteration'].get('sba_solve'), d['mfma_fp64']['fp64_frac'])"
head -9 $O/ba_iter_durations.txt
echo done
