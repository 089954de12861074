"""Per-rebuild kernel and HIP API costs from scripts/gpu_rebuild_diff.sh's two runs (60 - 10 rebuilds).

    python3 scripts/rebuild_diff.py gpurun_out/TAG"""
import csv
import sys

d = sys.argv[1]
for k in ("hip_api_stats", "kernel_stats"):
    a = {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(f"{d}/{k}_10.csv"))}
    b = {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(f"{d}/{k}_60.csv"))}
    rows = []
    for n, (c, t) in b.items():
        c0, t0 = a.get(n, (0, 0.0))
        if c > c0:
            rows.append(((t - t0) / 50e3, (c - c0) / 50, n))
    rows.sort(reverse=True)
    print(f"{k}: per rebuild {sum(r[0] for r in rows):.1f} us in {sum(r[1] for r in rows):.0f} calls")
    for t, c, n in rows[:24]:
        print(f"   {n[:64]:64s} {c:6.2f} calls {t:8.2f} us")
