#!/usr/bin/env python3
"""Pipeline timeline from a rocprofv3 --kernel-trace CSV of bench.py.

    python3 scripts/pipe_timeline.py gpurun_out/<dir>/run_kernel_trace.csv

Per stream (queue): kernels, busy time and idle gaps over the steady-state window (frames between
the 25th and the 75th percentile of LocalBA prologue starts); per frame: the period between
consecutive LocalBA prologues, the LocalBA chain length (prologue start to last k_ba_iter end) and
the wait of each LocalBA run after its previous one."""
import collections
import csv
import re
import sys

import numpy as np


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


rows = list(csv.DictReader(open(sys.argv[1])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), short(r["Kernel_Name"]),
       r["Kernel_Name"]) for r in rows]
ev.sort()
pro = [e for e in ev if e[3] == "k_ba_iter" and "<true" in e[4]]
if len(pro) < 8:
    sys.exit("no fused LocalBA prologues in the trace")
t0 = pro[len(pro) // 4][0]
t1 = pro[3 * len(pro) // 4][0]
nfr = 3 * len(pro) // 4 - len(pro) // 4
print(f"window: {nfr} frames, {(t1 - t0) / 1e3:.1f} us, {(t1 - t0) / 1e3 / nfr:.2f} us/frame")
win = [e for e in ev if e[0] >= t0 and e[1] <= t1]
by_q = collections.defaultdict(list)
for e in win:
    by_q[e[2]].append(e)
for q, es in sorted(by_q.items()):
    busy = sum(e[1] - e[0] for e in es)
    kinds = collections.Counter(e[3] for e in es)
    per = {k: np.mean([e[1] - e[0] for e in es if e[3] == k]) / 1e3 for k in kinds}
    gaps = [es[i + 1][0] - es[i][1] for i in range(len(es) - 1)]
    print(f"queue {q}: busy {busy / (t1 - t0):.2f}, {busy / 1e3 / nfr:.1f} us/frame, gaps mean "
          f"{np.mean(gaps) / 1e3 if gaps else 0:.2f} us max {max(gaps) / 1e3 if gaps else 0:.1f} us; kernels "
          + ", ".join(f"{k} x{kinds[k] / nfr:.1f} {per[k]:.2f}us" for k in sorted(kinds)))
# LocalBA runs: prologue + following k_ba_iter on the same queue
qba = pro[0][2]
ba = [e for e in ev if e[2] == qba and e[3] == "k_ba_iter"]
runs, cur = [], []
for e in ba:
    if "<true" in e[4] and cur:
        runs.append(cur)
        cur = []
    cur.append(e)
runs.append(cur)
runs = [r for r in runs if r[0][0] >= t0 and r[-1][1] <= t1]
chain = [(r[-1][1] - r[0][0]) / 1e3 for r in runs]
waits = [(runs[i + 1][0][0] - runs[i][-1][1]) / 1e3 for i in range(len(runs) - 1)]
inner = [np.mean([(r[i + 1][0] - r[i][1]) / 1e3 for i in range(len(r) - 1)]) for r in runs]
print(f"LocalBA runs: chain {np.mean(chain):.1f} us (min {min(chain):.1f}), launch gaps inside {np.mean(inner):.2f} us, "
      f"wait before next run {np.mean(waits):.1f} us (max {max(waits):.1f})")
