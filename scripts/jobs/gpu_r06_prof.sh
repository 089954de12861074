#!/bin/bash
# round 6: the committed measurements on the current tree in ONE session:
#   1. PMC FETCH_SIZE / WRITE_SIZE passes (separate runs) -> profiles/pmc_traffic.json
#   2. bench.py, the default N = 1 command (CPU baseline included) -> the C3 line
#   3. rocprofv3 --kernel-trace --stats of bench.py -> per-kernel durations + that run's own line
#   4. C4 (with its CPU baseline) and C5 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r06}
O=gpurun_out/prof_$TAG
mkdir -p $O
P="--steps 20 --warmup 3 --no-cpu-baseline --no-profile --no-drop-in"
# (a heartbeat under gpurun_out/: the counter passes print nothing for minutes)
(while true; do sleep 30; date >> $O/heartbeat.txt; done) &
BEAT=$!
trap "kill $BEAT 2>/dev/null" EXIT
# (the bench's own passes with the per-iteration launches: rocprofv3's counter collection aborts on
# the pipelined bench with the persistent window; k_ba_win's bytes from LocalBA alone, below)
VX_BA_PERSIST=0 timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python3 bench.py $P > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -30 $O/pmc_fetch.log; exit 1; }
VX_BA_PERSIST=0 timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 bench.py $P > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -30 $O/pmc_write.log; exit 1; }
python3 scripts/pmc_summary.py "$(find $O/pf -name '*counter_collection.csv' | head -1)" \
    "$(find $O/pw -name '*counter_collection.csv' | head -1)" $O/pmc_traffic.json > $O/pmc_traffic.txt || exit 1
rm -rf $O/pf $O/pw
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/wf -o run -- python3 scripts/ba_alone.py > $O/pmc_win_fetch.log 2>&1 || { echo "pmc win fetch failed"; tail -30 $O/pmc_win_fetch.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/ww -o run -- python3 scripts/ba_alone.py > $O/pmc_win_write.log 2>&1 || { echo "pmc win write failed"; tail -30 $O/pmc_win_write.log; exit 1; }
(cd scripts && python3 pmc_merge_win.py "$(find ../$O/wf -name '*counter_collection.csv' | head -1)" "$(find ../$O/ww -name '*counter_collection.csv' | head -1)" ../$O/pmc_traffic.json) >> $O/pmc_traffic.txt || exit 1
rm -rf $O/wf $O/ww
cp $O/pmc_traffic.json profiles/pmc_traffic.json
grep -E "k_ba|k_select|k_fast|k_pyr|k_knn|k_desc" $O/pmc_traffic.txt
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench failed"; tail -20 $O/bench_c3.err; exit 2; }
cat $O/bench_c3.json | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline > $O/bench_c3_rocprof.json 2> $O/kt.log || { echo "rocprof failed"; tail -30 $O/kt.log; exit 3; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_bench_c3.csv \;
rm -rf $O/kt
head -5 $O/kernel_stats_bench_c3.csv | cut -c1-200
python3 -c "
import json,csv
d=json.loads(open('$O/bench_c3_rocprof.json').read().strip().splitlines()[-1]); rf=d['roofline']
rows=[r for r in csv.DictReader(open('$O/kernel_stats_bench_c3.csv')) if '::'+rf['hip_kernel']+'<' in r['Name'] or '::'+rf['hip_kernel']+'(' in r['Name']]
print('line', rf['kernel'], rf['avg_launch_us'], rf['frac'], 'profile', [(r['Name'][:60], float(r['AverageNs'])/1e3, rf['bytes_per_launch']/(float(r['AverageNs'])*1e-9)/8e12) for r in rows])
"
timeout -k 10 600 python bench.py --config C4 --steps 200 --warmup 10 > $O/bench_c4.json 2> $O/bench_c4.err || { echo "bench c4 failed"; tail -20 $O/bench_c4.err; exit 4; }
cat $O/bench_c4.json | cut -c1-300
timeout -k 10 600 python bench.py --config C5 --steps 60 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; tail -20 $O/bench_c5.err; exit 5; }
cat $O/bench_c5.json | cut -c1-300
echo done
