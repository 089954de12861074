#!/bin/bash
# Instruction-fetch share of the extraction kernels' L2->memory traffic: per-dispatch averages of
# SQC_TC_INST_REQ / SQC_TC_DATA_READ_REQ (SQ block) and FETCH_SIZE (separate pass) over
# scripts/orb_loop.py (30 C3 extractions, alone).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/sqc
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ --output-format csv -d $O/a -o run -- python3 scripts/orb_loop.py > $O/a.log 2>&1 || { echo "sqc pass failed"; tail -20 $O/a.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/b -o run -- python3 scripts/orb_loop.py > $O/b.log 2>&1 || { echo "fetch pass failed"; tail -20 $O/b.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections, re
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in ("a", "b"):
    f = glob.glob(f"{o}/{d}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        mm = re.search(r"\b(k_\w+)", r["Kernel_Name"])
        k = mm.group(1) if mm else r["Kernel_Name"][:20]
        per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, cn), v in per.items():
        acc[k][cn].append(v)
for k in sorted(acc):
    if not k.startswith("k_"):
        continue
    row = {cn: sum(v) / len(v) for cn, v in acc[k].items()}
    inst = row.get("SQC_TC_INST_REQ", 0.0)
    print(f"{k:16s} SQC_TC_INST_REQ {inst:9.0f} (x64 B = {inst * 64 / 1e3:7.1f} kB)  SQC_TC_DATA_READ_REQ {row.get('SQC_TC_DATA_READ_REQ', 0):8.0f}"
          f"  FETCH_SIZE {row.get('FETCH_SIZE', 0):8.1f} kB (x2 corrected {2 * row.get('FETCH_SIZE', 0):8.1f})")
PY
rm -rf $O/a $O/b
