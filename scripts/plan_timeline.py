#!/usr/bin/env python3
"""Timeline of LocalBA plan builds (C3) from the resident map and from a snapshot: run under
`rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d DIR -o run --
python3 scripts/plan_timeline.py`, then `python3 scripts/plan_timeline.py DIR` summarises the last
build of each kind: wall time, kernel busy time, copies, synchronisations and host gaps."""
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))


def run():
    import vxslam
    from vxslam import synth
    nk, nl, _ = synth.ba_config("C3")
    m = synth.make_ba_map(0x5EED0003, nk, nl)
    o = vxslam.default_ba_options(window=nk)
    ctx = vxslam.Context(0)
    dm = vxslam.DMap(ctx)
    vxslam.dmap_load(dm, m)
    ctx.synchronize()
    for kind in ("dmap", "snapshot"):
        for i in range(8):
            time.sleep(0.005)
            t0 = time.perf_counter()
            p = dm.plan(o) if kind == "dmap" else ctx.ba_plan(m, o)
            t1 = time.perf_counter()
            p.close()
            print(f"{kind} build {i}: {1e3 * (t1 - t0):.3f} ms", flush=True)
    ctx.close()


def summarise(d):
    def load(pat):
        f = glob.glob(os.path.join(d, "**", pat), recursive=True)
        return list(csv.DictReader(open(f[0]))) if f else []
    ev = []
    for r in load("*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"].split("(")[0][-40:]))
    for r in load("*hip_api_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A", r["Function"]))
    for r in load("*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "copy")))
    ev.sort()
    # builds: API bursts separated by > 2 ms of silence
    groups, cur, last = [], [], None
    for e in ev:
        if last is not None and e[0] - last > 2_000_000:
            groups.append(cur)
            cur = []
        cur.append(e)
        last = max(last or 0, e[1])
    groups.append(cur)
    groups = [g for g in groups if sum(1 for e in g if e[2] == "K") > 5]
    for name, g in (("dmap (last)", groups[7] if len(groups) > 8 else groups[-1]), ("snapshot (last)", groups[-1])):
        t0 = min(e[0] for e in g)
        t1 = max(e[1] for e in g)
        kern = [e for e in g if e[2] == "K"]
        busy = sum(e[1] - e[0] for e in kern)
        sync = sum(e[1] - e[0] for e in g if e[2] == "A" and "Synchronize" in e[3])
        copies = [e for e in g if e[2] == "C"]
        print(f"{name}: wall {(t1 - t0) / 1e3:.1f} us, {len(kern)} kernels busy {busy / 1e3:.1f} us, "
              f"{len(copies)} copies {sum(e[1] - e[0] for e in copies) / 1e3:.1f} us, "
              f"{sum(1 for e in g if e[2] == 'A' and 'Synchronize' in e[3])} syncs {sync / 1e3:.1f} us")
        for e in g:
            if e[2] in "KC" or "Synchronize" in e[3] or "Memcpy" in e[3]:
                print(f"   {(e[0] - t0) / 1e3:8.1f} +{(e[1] - e[0]) / 1e3:7.1f}  {e[2]} {e[3]}")


if __name__ == "__main__":
    if len(sys.argv) > 1:
        summarise(sys.argv[1])
    else:
        run()
