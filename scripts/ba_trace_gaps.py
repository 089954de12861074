"""LocalBA launch gaps in the pipeline (round 4): from a rocprofv3 kernel trace of bench.py, the
k_ba_iter dispatches grouped into runs (a prologue starts one), each run's kernel time, the idle
time between its dependent launches, and the idle time between runs (the wait for Match).

    rocprofv3 --kernel-trace --output-format csv -d D -o kt -- python3 bench.py ...
    python3 scripts/ba_trace_gaps.py D/kt_kernel_trace.csv"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_ba_iter" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
runs, cur = [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3
    if "ILb1E" in r["Kernel_Name"] or "k_ba_iter<true" in r["Kernel_Name"]:
        cur = [(s, e)]
        runs.append(cur)
    elif cur is not None:
        cur.append((s, e))
L = max(len(r) for r in runs)
runs = [r for r in runs if len(r) == L][20:]
dur = np.array([[e - s for s, e in r] for r in runs])
gap = np.array([[r[i + 1][0] - r[i][1] for i in range(L - 1)] for r in runs])
span = np.array([r[-1][1] - r[0][0] for r in runs])
between = np.array([runs[i + 1][0][0] - runs[i][-1][1] for i in range(len(runs) - 1)])
period = np.array([runs[i + 1][0][0] - runs[i][0][0] for i in range(len(runs) - 1)])
print(f"{len(runs)} runs of {L} launches; microseconds (median, mean)")
for i in range(L):
    print(f"  launch {i} ({'prologue' if i == 0 else f'iteration {i - 1}'}): {np.median(dur[:, i]):6.2f} {dur[:, i].mean():6.2f}"
          + (f"   gap after: {np.median(gap[:, i]):5.2f} {gap[:, i].mean():5.2f}" if i < L - 1 else ""))
print(f"  kernel time per run {np.median(dur.sum(1)):6.2f} {dur.sum(1).mean():6.2f}")
print(f"  gaps within a run   {np.median(gap.sum(1)):6.2f} {gap.sum(1).mean():6.2f}")
print(f"  run span            {np.median(span):6.2f} {span.mean():6.2f}")
print(f"  idle between runs   {np.median(between):6.2f} {between.mean():6.2f}  (p10 {np.percentile(between, 10):.2f}, p90 {np.percentile(between, 90):.2f})")
print(f"  run period          {np.median(period):6.2f} {period.mean():6.2f}")
