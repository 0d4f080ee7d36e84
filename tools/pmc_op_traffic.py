#!/usr/bin/env python3
"""HBM traffic per OP CALL (an op may be several launches, e.g. the decoder conv-k9 = the phased
256x256 kernel on whole rounds + the 128x128 kernel on the rows left) from separate rocprofv3
FETCH_SIZE / WRITE_SIZE passes over `tools/kernel_probe.py <op> --reps R`.

Units: KiB counters; gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE x2 for 16 B/lane
streaming reads; WRITE_SIZE exact for 16 B/lane stores.

    python tools/pmc_op_traffic.py gpurun_out/prof_r1e conv9 10 conv_gemm [algorithmic_bytes]
"""
import collections
import csv
import json
import sys


def per_call(path, name_sub, reps):
    tot = 0.0
    kern = collections.Counter()
    for r in csv.DictReader(open(path)):
        if name_sub in r["Kernel_Name"]:
            tot += float(r["Counter_Value"])
            kern[r["Kernel_Name"].split("(")[0][-60:] + f" grid={r['Grid_Size']}"] += 1
    return tot / reps, dict(kern)


def main(d, op, reps, name_sub, algorithmic=None):
    reps = int(reps)
    f, kf = per_call(f"{d}/pmc_{op}_FETCH_SIZE/pmc_counter_collection.csv", name_sub, reps)
    w, _ = per_call(f"{d}/pmc_{op}_WRITE_SIZE/pmc_counter_collection.csv", name_sub, reps)
    rec = {"op": op, "calls": reps, "dispatches": kf, "FETCH_SIZE_KiB_per_call": f, "WRITE_SIZE_KiB_per_call": w,
           "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
           "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane reads); KiB units; summed over the op's launches"}
    if algorithmic:
        rec["algorithmic_bytes"] = float(algorithmic)
        rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / float(algorithmic)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
