"""Durations of the LocalBA launches and the gaps between consecutive ones of the same run, from a
rocprofv3 --kernel-trace CSV (bench.py pipeline vs scripts/ba_alone.py): whether the pipeline's extra
LocalBA time is inside the kernels or between them.  `python scripts/ba_gap_trace.py run_kernel_trace.csv`"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_ba_iter" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = np.array([int(r["Start_Timestamp"]) for r in rows], np.int64)
en = np.array([int(r["End_Timestamp"]) for r in rows], np.int64)
pro = np.array(["true" in r["Kernel_Name"].split("<")[1][:8] if "<" in r["Kernel_Name"] else False for r in rows])
dur = (en - st) / 1e3
gap = (st[1:] - en[:-1]) / 1e3
# a gap belongs to a run when the next launch is not a prologue (runs start with the prologue)
inrun = ~pro[1:]
runs = np.flatnonzero(pro)
span = [(en[runs[i + 1] - 1] - st[runs[i]]) / 1e3 for i in range(len(runs) - 1)]
print(f"{len(rows)} launches, {pro.sum()} runs")
print(f"duration us: prologue median {np.median(dur[pro]):.2f}, iterations median {np.median(dur[~pro]):.2f} "
      f"p90 {np.percentile(dur[~pro], 90):.2f}")
print(f"gap inside a run us: median {np.median(gap[inrun]):.2f} p90 {np.percentile(gap[inrun], 90):.2f} "
      f"max {gap[inrun].max():.2f}")
print(f"run span (prologue start -> last end) us: median {np.median(span):.2f} p90 {np.percentile(span, 90):.2f}")
