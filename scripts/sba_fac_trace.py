"""Per-launch durations and gaps of the multi-workgroup Schur factor (k_sba_fac_begin /
k_sba_fac_step / k_sba_backsub) from a rocprofv3 kernel trace of scripts/sba_bench.py:

    SBA_CFGS=C5-connected rocprofv3 --kernel-trace --output-format csv -d D -o kt -- python3 scripts/sba_bench.py 2
    python3 scripts/sba_fac_trace.py D/kt_kernel_trace.csv"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps, gaps, begins, backs = [], [], [], []
prev_end = None
for r in rows:
    nm = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "k_sba_fac_step" in nm:
        steps.append((e - s) / 1e3)
        if prev_end is not None:
            gaps.append((s - prev_end) / 1e3)
    elif "k_sba_fac_begin" in nm:
        begins.append((e - s) / 1e3)
    elif "k_sba_backsub" in nm:
        backs.append((e - s) / 1e3)
    prev_end = e if any(k in nm for k in ("k_sba_fac_begin", "k_sba_fac_step")) else None
for name, v in (("k_sba_fac_begin", begins), ("k_sba_fac_step", steps), ("gap before a step", gaps),
                ("k_sba_backsub", backs)):
    if v:
        a = np.array(v)
        print(f"{name:20s} n {len(a):6d}  mean {a.mean():7.2f} us  median {np.median(a):7.2f}  p90 {np.percentile(a, 90):7.2f}")
