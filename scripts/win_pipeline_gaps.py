#!/usr/bin/env python3
"""The persistent LocalBA window (k_ba_win) inside the C3 pipeline, from a rocprofv3 kernel trace of
bench.py: per window its duration, the gap after the previous window, and how long after its
dependencies were met it started — its Match (the k-th k_knn_compact pairs with the k-th window:
both run in frame order) and the previous window.  A start well after both means the window waited
for compute units (the extraction kernels' workgroups).

    python3 scripts/win_pipeline_gaps.py <rocprofv3 output dir>
"""
import csv
import glob
import sys

import numpy as np


def main():
    tr = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
    t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
    lo, hi = t0 + 0.35 * (t1 - t0), t0 + 0.65 * (t1 - t0)  # (the middle of the run: the timed steps)
    win = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "k_ba_win" in r["Kernel_Name"]]
    cmp_ = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "k_knn_compact" in r["Kernel_Name"]]
    wi = [i for i, (s, e) in enumerate(win) if lo <= s <= hi]
    if not wi:
        raise SystemExit("no windows in the middle of the trace")
    # pair: the compact that ended last before the first window of the region, then in lockstep
    s0 = win[wi[0]][0]
    j = max(k for k, (s, e) in enumerate(cmp_) if e <= s0)
    dur, gap, dep, wait_m, wait_w = [], [], [], [], []
    for n, i in enumerate(wi):
        if i == 0 or j + n >= len(cmp_):
            continue
        s, e = win[i]
        pe = win[i - 1][1]
        ce = cmp_[j + n][1]
        dur.append((e - s) / 1e3)
        gap.append((s - pe) / 1e3)
        dep.append((s - max(pe, ce)) / 1e3)
        wait_m.append(ce > pe)
    dur, gap, dep = map(np.array, (dur, gap, dep))
    print(f"{len(dur)} windows in the middle of the run")
    for name, v in (("window duration", dur), ("gap after the previous window", gap),
                    ("start after both dependencies met", dep)):
        print(f"  {name:36s} median {np.median(v):7.2f}  mean {np.mean(v):7.2f}  p10 {np.percentile(v, 10):7.2f}  p90 {np.percentile(v, 90):7.2f} us")
    print(f"  windows whose Match ended after the previous window: {np.mean(wait_m) * 100:.0f} %")
    period = np.diff([win[i][0] for i in wi]) / 1e3
    print(f"  window start -> next window start: median {np.median(period):.2f} us")
    kern = {}
    for r in rows:
        s = int(r["Start_Timestamp"])
        if lo <= s <= hi:
            n = r["Kernel_Name"].replace("vx::(anonymous namespace)::", "").split("(")[0][:40]
            kern.setdefault(n, []).append((int(r["End_Timestamp"]) - s) / 1e3)
    print("kernels in the same span (calls, median us):")
    for n, v in sorted(kern.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"  {n:40s} {len(v):6d} {np.median(v):8.2f}")


if __name__ == "__main__":
    main()
