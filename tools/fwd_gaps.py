#!/usr/bin/env python3
"""One graph-replayed forward from a rocprofv3 kernel trace: kernels in order, duration, gap to
the previous kernel's end (us), averaged over the last N forwards (forward = cond_kernel .. next).

    python tools/fwd_gaps.py gpurun_out/trace/t/bench_kernel_trace.csv [--min-gap 1]
"""
import csv
import re
import sys


def main(path, min_gap=0.0):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    st = [i for i, r in enumerate(rows) if "cond_kernel" in r["Kernel_Name"]]
    segs = [rows[a:b] for a, b in zip(st[-11:-1], st[-10:])]
    n = len(segs[0])
    tot_d = tot_g = 0.0
    for i in range(n):
        d = sum(int(s[i]["End_Timestamp"]) - int(s[i]["Start_Timestamp"]) for s in segs) / len(segs) / 1e3
        g = 0.0 if i == 0 else sum(int(s[i]["Start_Timestamp"]) - int(s[i - 1]["End_Timestamp"]) for s in segs) / len(segs) / 1e3
        tot_d += d
        tot_g += g
        r = segs[0][i]
        if g >= min_gap:
            name = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", r["Kernel_Name"])[:40]
            print(f"{i:3d} {name:40s} {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):6d} {d:8.1f} gap {g:5.1f}")
    print(f"kernels {n}: busy {tot_d:.1f} us, gaps {tot_g:.1f} us")


if __name__ == "__main__":
    mg = float(sys.argv[sys.argv.index("--min-gap") + 1]) if "--min-gap" in sys.argv else -1e9
    main(sys.argv[1], mg)
