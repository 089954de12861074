#!/usr/bin/env python3
"""Per-kernel durations of the Schur solve from a rocprofv3 kernel trace (scripts/jobs/gpu_r05_v.sh), and
the time between consecutive launches of the factor (end of one to the start of the next).

    python3 scripts/sba_gaps.py <rocprofv3 output dir>
"""
import csv
import glob
import sys
from collections import defaultdict

import numpy as np


def main():
    d = sys.argv[1]
    tr = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
    dur = defaultdict(list)
    seq = []
    for r in rows:
        n = r["Kernel_Name"].replace("vx::(anonymous namespace)::", "").split("(")[0]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[n].append((e - s) / 1e3)
        seq.append((n, s, e))
    print("kernel                      calls   avg us   total us")
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        if "sba" in n:
            print(f"{n[:28]:28s} {len(v):6d} {np.mean(v):8.2f} {sum(v):10.1f}")
    # gaps inside runs of solve kernels
    gaps = defaultdict(list)
    for (a, _, ea), (b, sb, _) in zip(seq, seq[1:]):
        if "sba" in a and "sba" in b and 0 <= sb - ea < 50_000:
            gaps[(a[:22], b[:22])].append((sb - ea) / 1e3)
    print("gap (end of a -> start of b)              n     median us")
    for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[0]:22s} -> {k[1]:22s} {len(v):6d} {np.median(v):8.2f}")


if __name__ == "__main__":
    main()
