"""k_sba_solve MFMA counters (rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES) per window config, split by grid size (C3: 1
component workgroup, C5: 8) and keeping only launches that factored (MFMA count > 0; the last
iteration of a run only decides and exits)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if "k_sba_solve" not in r["Kernel_Name"]:
        continue
    key = (int(r["Grid_Size"]), r["Dispatch_Id"])
    by[key][r["Counter_Name"]] += float(r["Counter_Value"])
    by[key]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
agg = collections.defaultdict(list)
for (grid, _), v in by.items():
    if v.get("SQ_INSTS_VALU_MFMA_F64", 0) > 0:
        agg[grid].append(v)
for grid, vs in sorted(agg.items()):
    n = len(vs)
    mean = lambda k: sum(v.get(k, 0.0) for v in vs) / n
    flops = mean("SQ_INSTS_VALU_MFMA_MOPS_F64") * 512
    dur = mean("dur_ns") * 1e-9
    wgs = grid // 256
    print(f"k_sba_solve grid {grid} ({wgs} component workgroup(s)), {n} factoring launches: "
          f"MFMA_F64 instructions {mean('SQ_INSTS_VALU_MFMA_F64'):.0f}, MFMA FP64 flops {flops / 1e6:.2f} M, "
          f"MFMA busy cycles {mean('SQ_VALU_MFMA_BUSY_CYCLES'):.0f}, CU busy cycles {mean('SQ_BUSY_CU_CYCLES'):.0f}, "
          f"duration {dur * 1e6:.1f} us (profiled) -> {flops / dur / 1e12:.4f} TFLOP/s MFMA FP64")
