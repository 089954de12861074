#!/bin/bash
# round 6: SQ counters of k_ba_win alone (LDS bank conflicts, LDS / VALU instruction mix, waits)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06lds}
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU --output-format csv -d $O/p1 -o run -- python3 scripts/ba_alone.py > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 2; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r06lds/p1/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "k_ba_win" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:24s} per launch {sum(v) / max(1, len(set(range(len(v))))) :.4g}  (n={len(v)})")
PY
