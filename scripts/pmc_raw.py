"""Mean per-dispatch value of every counter per kernel from rocprofv3 --pmc csv output(s).
Usage: pmc_raw.py counter_collection.csv [...]"""
import collections
import csv
import re
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        m = re.search(r"\b(k_[a-z0-9_]+)(?:<[^>(]*>)?\(", r["Kernel_Name"])
        if m:
            rows[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(rows.items()):
    print(k + ": " + ", ".join(f"{n}={sum(v) / len(v):.4g}" for n, v in sorted(c.items())))
