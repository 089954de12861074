#!/bin/bash
# round 4: kernel trace of the multi-workgroup Schur factor on the connected C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
SBA_CFGS=C5-connected timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/sba_bench.py 2 > /dev/null 2>&1 || exit 3
python3 scripts/sba_fac_trace.py $O/kt/kt_kernel_trace.csv > $O/sba_fac_trace.txt 2>&1
rm -f $O/kt/kt_kernel_trace.csv
cat $O/sba_fac_trace.txt
