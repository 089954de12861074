"""Splits a rocprofv3 kernel trace of `python bench.py` into the bench's passes and prints one
kernel's per-dispatch duration per pass, so the HIP-event number bench.py reports
(roofline.avg_launch_us, measured in the roofline pass) can be compared with rocprof's view of
the same dispatches.  Passes, in dispatch order of the kernel (launches per step L):
profile (warmup * L) | timed (warmup + steps) * L | roofline steps * L | latency 20 * L.

    python3 scripts/trace_phases.py <run_kernel_trace.csv> <kernel> <launches_per_step> [steps] [warmup]
"""
import csv
import sys

import numpy as np

path, kernel, per = sys.argv[1], sys.argv[2], int(sys.argv[3])
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 300
warmup = int(sys.argv[5]) if len(sys.argv) > 5 else 5
rows = [r for r in csv.DictReader(open(path)) if kernel + "(" in r["Kernel_Name"] or kernel + "<" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows])
bounds = [("profile", warmup * per), ("timed", (warmup + steps) * per), ("roofline", steps * per), ("latency", 20 * per)]
a = 0
print(f"{kernel}: {len(d)} dispatches")
for name, n in bounds:
    seg = d[a:a + n]
    if len(seg):
        print(f"  {name:9s} {len(seg):5d} dispatches  mean {seg.mean():7.2f} us  median {np.median(seg):7.2f} us")
    a += n
