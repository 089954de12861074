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

# the multi-workgroup factorisation (k_sba_fac_begin, k_sba_fac_step x (nt - 1), k_sba_backsub): one
# group per solve, counters summed over its launches, duration = first start to last end
disp = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for r in rows:
    nm = r["Kernel_Name"]
    if not any(k in nm for k in ("k_sba_fac_begin", "k_sba_fac_step", "k_sba_fac_blk", "k_sba_backsub")):
        continue
    d = int(r["Dispatch_Id"])
    disp[d][r["Counter_Name"]] += float(r["Counter_Value"])
    meta[d] = (nm, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size"]))
groups, cur = [], None
for d in sorted(meta):
    nm = meta[d][0]
    if "k_sba_fac_begin" in nm:
        cur = [d]
        groups.append(cur)
    elif cur is not None:
        cur.append(d)
sols = []
for g in groups:
    tot = collections.defaultdict(float)
    for d in g:
        for k, v in disp[d].items():
            tot[k] += v
    if tot.get("SQ_INSTS_VALU_MFMA_F64", 0) <= 0:
        continue
    tot["span_ns"] = max(meta[d][2] for d in g) - min(meta[d][1] for d in g)
    tot["kern_ns"] = sum(meta[d][2] - meta[d][1] for d in g)
    tot["launches"] = len(g)
    tot["step_grid"] = max(meta[d][3] for d in g)
    sols.append(tot)
if sols:
    n = len(sols)
    mean = lambda k: sum(v.get(k, 0.0) for v in sols) / n
    flops = mean("SQ_INSTS_VALU_MFMA_MOPS_F64") * 512
    span = mean("span_ns") * 1e-9
    print(f"multi-workgroup factor ({mean('launches'):.0f} launches per solve, step grid {mean('step_grid') / 256:.0f} "
          f"workgroups), {n} factoring solves: MFMA_F64 instructions {mean('SQ_INSTS_VALU_MFMA_F64'):.0f}, "
          f"MFMA FP64 flops {flops / 1e6:.2f} M, MFMA busy cycles {mean('SQ_VALU_MFMA_BUSY_CYCLES'):.0f}, "
          f"CU busy cycles {mean('SQ_BUSY_CU_CYCLES'):.0f}, span {span * 1e6:.1f} us, kernel time "
          f"{mean('kern_ns') / 1e3:.1f} us (profiled) -> {flops / span / 1e12:.4f} TFLOP/s MFMA FP64 over the span")
