#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Units: rocprofv3 reports both counters in KiB. gfx950 correction (MI355X_MICROARCH.md
§HBM): FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane) coalesced streaming read,
so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.

    python tools/pmc_traffic.py gpurun_out/prof_r1b conv9 <grid_size>
"""
import csv
import json
import sys


def per_launch(path, grid):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if r["Grid_Size"] == str(grid)]
    return sum(v) / len(v), len(v)


def main(d, k, grid, algorithmic=None):
    f, nf = per_launch(f"{d}/pmc_{k}_FETCH_SIZE/pmc_counter_collection.csv", grid)
    w, nw = per_launch(f"{d}/pmc_{k}_WRITE_SIZE/pmc_counter_collection.csv", grid)
    rec = {"kernel": k, "grid_size": int(grid), "launches": [nf, nw], "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
           "fetch_bytes_corrected": 2 * f * 1024, "write_bytes": w * 1024,
           "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024, "correction": "FETCH_SIZE x2 (gfx950, 16B/lane reads)"}
    if algorithmic:
        rec["algorithmic_bytes"] = algorithmic
        rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / algorithmic
    print(json.dumps(rec, indent=1))
    return rec


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4]) if len(sys.argv) > 4 else None)
