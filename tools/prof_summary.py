#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv by (kernel, grid): calls, mean/min duration (us).

    python tools/prof_summary.py gpurun_out/prof_r1/trace/bench_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)(I[^E]*E)?", name)
    base = m.group(1) if m else name[:40]
    tmpl = ""
    if "ILi" in name:
        tmpl = "<" + ",".join(re.findall(r"Li(\d+)E", name)) + (",bf16" if "DF16b" in name.split("EEv")[0][-8:] else "") + ">"
    return base + tmpl


def main(path, top=40):
    rows = list(csv.DictReader(open(path)))
    g = collections.defaultdict(list)
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = (short(r["Kernel_Name"]), f"{int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}")
        g[key].append(d)
    tot = sum(sum(v) for v in g.values())
    print(f"{'kernel':44s} {'grid(WGs)':>14s} {'calls':>6s} {'mean_us':>9s} {'min_us':>9s} {'share':>6s}")
    for (k, grid), v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{k:44s} {grid:>14s} {len(v):6d} {sum(v)/len(v):9.2f} {min(v):9.2f} {100*sum(v)/tot:5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1])
