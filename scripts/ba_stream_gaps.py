#!/usr/bin/env python3
"""The LocalBA stream inside the C3 pipeline, from a rocprofv3 kernel trace of bench.py: per window
(prologue + iterations) the span from the prologue's start to the last launch's end, the sum of its
launch durations, the gaps between its launches, and the time from one window's start to the next.

    python3 scripts/ba_stream_gaps.py <rocprofv3 output dir>
"""
import csv
import glob
import sys

import numpy as np


def main():
    tr = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
    ba = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
          if "k_ba_iter" in r["Kernel_Name"]]
    wins, cur = [], []
    for n, s, e in ba:
        if "k_ba_iter<true" in n.replace(" ", "") or "ILb1E" in n or "<true" in n:
            if cur:
                wins.append(cur)
            cur = [(s, e)]
        elif cur:
            cur.append((s, e))
    if cur:
        wins.append(cur)
    wins = [w for w in wins if len(w) >= 2][len(wins) // 10:]  # (skip the warm-up tenth)
    span = np.array([(w[-1][1] - w[0][0]) / 1e3 for w in wins])
    busy = np.array([sum(e - s for s, e in w) / 1e3 for w in wins])
    gaps = np.array([sum(max(0, w[i + 1][0] - w[i][1]) for i in range(len(w) - 1)) / 1e3 for w in wins])
    period = np.diff([w[0][0] for w in wins]) / 1e3
    nl = np.array([len(w) for w in wins])
    print(f"{len(wins)} windows, launches per window median {np.median(nl):.0f}")
    for name, v in (("span (prologue start -> last end)", span), ("sum of launch durations", busy),
                    ("sum of gaps between launches", gaps), ("window start -> next window start", period)):
        print(f"  {name:36s} median {np.median(v):7.2f}  mean {np.mean(v):7.2f}  p90 {np.percentile(v, 90):7.2f} us")
    per_launch = {}
    for w in wins:
        for i, (s, e) in enumerate(w):
            per_launch.setdefault(i, []).append((e - s) / 1e3)
    print("  launch durations (median us):", " ".join(f"{i}:{np.median(v):.2f}" for i, v in sorted(per_launch.items())))
    allk = {}
    for r in rows:
        n = r["Kernel_Name"].replace("vx::(anonymous namespace)::", "").split("(")[0]
        allk.setdefault(n[:40], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("kernels (calls, median us, total ms):")
    for n, v in sorted(allk.items(), key=lambda kv: -sum(kv[1]))[:16]:
        print(f"  {n:40s} {len(v):7d} {np.median(v):8.2f} {sum(v) / 1e3:9.2f}")


if __name__ == "__main__":
    main()
