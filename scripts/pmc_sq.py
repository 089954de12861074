"""Per-kernel SQ / GRBM counters from one rocprofv3 --pmc pass (csv): wave-cycle breakdown and
effective clock.  SQ_* cycle counters are in quad-cycles (MI355X_MICROARCH.md §PMC); GRBM_GUI_ACTIVE
is summed over the 8 XCDs.  Usage: pmc_sq.py run_counter_collection.csv run_kernel_trace.csv?"""
import collections
import csv
import re
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"\b(k_[a-z0-9_]+)(?:<[^>(]*>)?\(", r["Kernel_Name"])
    if not m:
        continue
    rows[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = collections.defaultdict(list)
if len(sys.argv) > 2:
    for r in csv.DictReader(open(sys.argv[2])):
        m = re.search(r"\b(k_[a-z0-9_]+)(?:<[^>(]*>)?\(", r["Kernel_Name"])
        if m:
            dur[m.group(1)].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':18s} {'waves':>7s} {'wave_us':>8s} {'wait%':>6s} {'instw%':>6s} {'active%':>7s} {'busy_us':>8s} {'clk_GHz':>7s}")
for k, c in sorted(rows.items()):
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) * 4
    waves = avg.get("SQ_WAVES", 0)
    pct = lambda n: 100.0 * avg.get(n, 0) * 4 / wc if wc else 0.0
    gui = avg.get("GRBM_GUI_ACTIVE", 0) / 8
    d = sum(dur[k]) / len(dur[k]) if dur.get(k) else 0
    clk = gui / (d * 1e3) if d else 0
    per_wave_us = (wc / waves / (clk * 1e3)) if waves and clk else 0
    print(f"{k:18s} {waves:7.0f} {per_wave_us:8.2f} {pct('SQ_WAIT_ANY'):6.1f} {pct('SQ_WAIT_INST_ANY'):6.1f} "
          f"{pct('SQ_ACTIVE_INST_ANY'):7.1f} {avg.get('SQ_BUSY_CYCLES', 0) / max(clk, 1e-9) / 1e3:8.2f} {clk:7.2f}")
