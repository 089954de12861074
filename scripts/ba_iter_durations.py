"""Per-iteration k_ba_iter durations: the rocprofv3 kernel trace of
scripts/ba_alone.py, its k_ba_iter dispatches grouped by their place in a run (prologue, then
iterations 0 .. 4), against the valid pose-stage observations each launch's pose stage forms (that of
iteration it + 1; the last launch has none).

    rocprofv3 --kernel-trace --output-format csv -d D -o kt -- python3 scripts/ba_alone.py
    python3 scripts/ba_iter_durations.py D/kt_kernel_trace.csv [obs...]"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_ba_iter" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pro = [("ILb1E" in r["Kernel_Name"] or "k_ba_iter<true" in r["Kernel_Name"]) for r in rows]
dur = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows])
obs = [int(x) for x in sys.argv[2:]]
runs, cur = [], None
for p, d in zip(pro, dur):
    if p:
        cur = [d]
        runs.append(cur)
    elif cur is not None:
        cur.append(d)
L = max(len(r) for r in runs)
runs = [r for r in runs if len(r) == L][5:]  # (skip the warm-up runs)
a = np.array(runs)
print(f"{len(runs)} runs of {L} launches (prologue + {L - 1} iterations), microseconds:")
for i in range(L):
    name = "prologue" if i == 0 else f"iteration {i - 1}"
    nxt = f"  pose stage of iteration {i} ({obs[i]} valid observations)" if i < len(obs) and i < L - 1 else ""
    print(f"  {name:12s} mean {a[:, i].mean():7.3f}  median {np.median(a[:, i]):7.3f}{nxt}")
print(f"  run total   mean {a.sum(1).mean():7.3f}")
