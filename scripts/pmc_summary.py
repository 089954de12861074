"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs).

FETCH_SIZE / WRITE_SIZE are in KB.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports exactly
half the bytes of a wide coalesced streaming read (128-B requests tallied at 64 B), so the fetch
side is doubled; WRITE_SIZE is taken as reported.  Output: {"config", "n_gpus", "bytes_per_launch":
{stage: bytes per launch}}.  Usage: pmc_summary.py fetch.csv write.csv out.json [config] [n_gpus]
"""
import collections
import csv
import json
import re
import sys

# kernel -> the profiling stage (vx_prof_name) whose HIP-event bracket contains it
STAGE = {"k_gray": "orb_gray", "k_resize": "orb_resize", "k_pyramid": "orb_pyramid", "k_fast": "orb_fast_harris",
         "k_select": "orb_select", "k_select_stl": "orb_select", "k_blur": "orb_blur", "k_describe": "orb_describe",
         "k_knn_partial": "match_partial", "k_knn_rows": "match_partial", "k_knn_merge": "match_merge",
         "k_knn_compact": "match_merge", "k_ba_reset": "ba_reset",
         "k_pose_kf": "ba_pose_partial", "k_landmark_solve": "ba_landmark", "k_pose_solve_g": "ba_landmark",
         "k_landmark": "ba_landmark", "k_ba_iter": "ba_iter", "k_ba_prologue": "ba_prologue",
         "k_ba_win": "ba_window"}


def agg(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"\b(k_[a-z0-9_]+)(<[^>(]*>)?\(", r["Kernel_Name"])
        if m:
            name = m.group(1)
            if name == "k_ba_iter":  # the fused LocalBA: prologue (<true, ...>) vs iterations
                name = "k_ba_prologue" if "true" in (m.group(2) or "") else "k_ba_iter"
            d[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main(fetch_csv, write_csv, out_json, config="C3", n_gpus="1"):
    f = agg(fetch_csv, "FETCH_SIZE")
    w = agg(write_csv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        b = 2.0 * f.get(k, 0.0) * 1024 + w.get(k, 0.0) * 1024
        res[STAGE.get(k, k)] = int(b)
        print(f"{k:16s} fetch {f.get(k, 0):10.1f} KB (x2 corrected)  write {w.get(k, 0):10.1f} KB  -> {b / 1e3:10.1f} kB/launch")
    # bench.py reads the traffic only for the workload it was measured on
    json.dump({"config": config, "n_gpus": int(n_gpus), "bytes_per_launch": res}, open(out_json, "w"), indent=1,
              sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:6])
