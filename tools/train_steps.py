#!/usr/bin/env python3
"""Per-step GPU time of a graphed train-step trace (rocprofv3 kernel_trace.csv of
`bench.py --mode train`): steps are delimited by the optimizer's last launch (fused Adam or torch's
multi_tensor_apply); prints kernels / busy / span per step and the top kernels of the last step.

    python tools/train_steps.py gpurun_out/r4d_train/trace/train_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def main(path, top=30):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    is_opt = lambda n: "adam_kernel" in n or "multi_tensor_apply" in n
    ends = []
    for i, r in enumerate(rows):
        if is_opt(r["Kernel_Name"]) and (i + 1 == len(rows) or not is_opt(rows[i + 1]["Kernel_Name"])):
            ends.append(i)
    steps = []
    for a, b in zip(ends[:-1], ends[1:]):
        seg = rows[a + 1:b + 1]
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
        span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
        steps.append((len(seg), busy, span, seg))
    for n, busy, span, _ in steps:
        print(f"step: {n:5d} kernels  busy {busy:8.0f} us  span {span:8.0f} us")
    seg = steps[-1][3]
    g = collections.defaultdict(list)
    for r in seg:
        m = re.search(r"(\w+_kernel\w*?)(I|E|\(|$)", r["Kernel_Name"])
        g[(m.group(1) if m else r["Kernel_Name"])[:56]].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"\nlast step: {len(seg)} kernels, busy {sum(sum(v) for v in g.values()):.0f} us")
    for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{k:58s} {len(v):4d} {sum(v):8.1f} {sum(v) / len(v):7.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
