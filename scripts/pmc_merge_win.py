"""Add k_ba_win's PMC bytes per launch (from rocprofv3 --pmc passes over scripts/ba_alone.py: the C3
window alone — the bench's own PMC passes run with VX_BA_PERSIST=0, since rocprofv3's counter
collection aborts on the pipelined bench with the persistent window, r06) to a pmc_traffic.json.

    pmc_merge_win.py fetch.csv write.csv pmc_traffic.json"""
import json
import sys

import pmc_summary


def main(fetch_csv, write_csv, out_json):
    f = pmc_summary.agg(fetch_csv, "FETCH_SIZE")
    w = pmc_summary.agg(write_csv, "WRITE_SIZE")
    d = json.load(open(out_json))
    if "k_ba_win" not in f:
        raise SystemExit("no k_ba_win dispatches in the counter files")
    b = 2.0 * f["k_ba_win"] * 1024 + w.get("k_ba_win", 0.0) * 1024
    d["bytes_per_launch"]["ba_window"] = int(b)
    d["ba_window_source"] = "rocprofv3 --pmc over scripts/ba_alone.py (C3 window, k_ba_win alone)"
    print(f"k_ba_win fetch {f['k_ba_win']:10.1f} KB (x2 corrected)  write {w.get('k_ba_win', 0):10.1f} KB  -> {b / 1e3:10.1f} kB/launch")
    json.dump(d, open(out_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:4])
