#!/bin/bash
# round 5 (ae): the lean call's read-back packed by k_lb_apply into one copy: resident-map tests,
# adapter per-call phases, the resident call's kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ae}
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_dmap.py tests/test_cpp_adapters.py tests/test_gpu_sba.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  echo "== rep $rep" >> $O/timing.txt
  timeout -k 10 200 python3 scripts/adapter_timing.py 40 >> $O/timing.txt 2>&1 || { tail -20 $O/timing.txt; exit 3; }
done
cat $O/timing.txt
python3 scripts/dump_c3_map.py /tmp/c3map && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- visionx-slam_amd/build/adapter_driver ba_calls /tmp/c3map 50 5 -1 40 resident > $O/drv.log 2>&1 || { tail -20 $O/drv.log; exit 4; }
cp $(find $O/kt -name 'kt_kernel_stats.csv' | head -1) $O/resident_kernel_stats.csv
rm -rf $O/kt
python3 -c "
import csv
for r in list(csv.reader(open('$O/resident_kernel_stats.csv')))[1:]:
    print(r[0].replace('vx::(anonymous namespace)::','')[:50], r[1], round(float(r[3])/1e3,2))"
echo done
