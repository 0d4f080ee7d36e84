#!/usr/bin/env python3
"""Per-launch FETCH/WRITE traffic of one kernel from tools/profile.sh PMC passes: filters by a
kernel-name substring, takes the most frequent grid size, sums counter instances per dispatch.
Units: KiB counters; FETCH x2 (gfx950 16 B/lane read correction, MI355X_MICROARCH.md §HBM).
    python tools/pmc_kernel.py gpurun_out/prof_r1h conv9 conv_gemm_kernel [algorithmic_bytes] [out.json]"""
import collections
import csv
import json
import sys


def per_dispatch(path, pat):
    d, grid = collections.defaultdict(float), {}
    for r in csv.DictReader(open(path)):
        if pat in r["Kernel_Name"]:
            d[r["Dispatch_Id"]] += float(r["Counter_Value"])
            grid[r["Dispatch_Id"]] = r["Grid_Size"]
    g = collections.Counter(grid.values()).most_common(1)[0][0]
    v = [d[k] for k in d if grid[k] == g]
    return sum(v) / len(v), len(v), g


d, probe, pat = sys.argv[1], sys.argv[2], sys.argv[3]
f, nf, g = per_dispatch(f"{d}/pmc_{probe}_FETCH_SIZE/pmc_counter_collection.csv", pat)
w, nw, _ = per_dispatch(f"{d}/pmc_{probe}_WRITE_SIZE/pmc_counter_collection.csv", pat)
rec = {"probe": probe, "kernel": pat, "grid_size": int(g), "launches": [nf, nw], "FETCH_SIZE_KiB": f,
       "WRITE_SIZE_KiB": w, "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
       "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane reads); KiB units"}
if len(sys.argv) > 4:
    rec["algorithmic_bytes"] = float(sys.argv[4])
    rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / rec["algorithmic_bytes"]
print(json.dumps(rec, indent=1))
if len(sys.argv) > 5:
    json.dump(rec, open(sys.argv[5], "w"), indent=1)
