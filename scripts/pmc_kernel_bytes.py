#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; KB units,
summed over the TCC instances), with the fetch counter doubled as MI355X_MICROARCH.md's gfx950
correction prescribes (the same convention as scripts/pmc_summary.py).

    python3 scripts/pmc_kernel_bytes.py <fetch counter_collection.csv> <write counter_collection.csv>"""
import collections
import csv
import sys


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if not r["Counter_Name"].startswith(counter):
            continue
        n = r["Kernel_Name"].replace("vx::(anonymous namespace)::", "").split("(")[0]
        tot[n] += float(r["Counter_Value"])
        disp[n].add(r["Dispatch_Id"])
    return {n: (tot[n] / len(disp[n]), len(disp[n])) for n in tot}


f = per_kernel(sys.argv[1], "FETCH_SIZE")
w = per_kernel(sys.argv[2], "WRITE_SIZE")
print(f"{'kernel':32s} {'launches':>8s} {'fetch KB (x2)':>14s} {'write KB':>10s} {'KB/launch':>10s}")
for n in sorted(f, key=lambda k: -(2 * f[k][0] + w.get(k, (0, 0))[0]) * f[k][1]):
    fk, cnt = f[n]
    wk = w.get(n, (0.0, 0))[0]
    print(f"{n[:32]:32s} {cnt:8d} {2 * fk:14.1f} {wk:10.1f} {2 * fk + wk:10.1f}")
