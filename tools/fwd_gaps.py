#!/usr/bin/env python3
"""Graph-replayed forwards from a rocprofv3 kernel trace of bench.py: kernels in order, duration,
gap to the previous kernel's end (us), averaged over the timed graph replays.

A forward starts at its two length-mask launches (or, with the masks written by the first encoder
block, at the conditioning launch / that block). The bench's trace also holds eager forwards
(warm-up, and the roofline's HIP-event-timed forwards, whose host-bound launches leave gaps); the
graph replays are the forwards with (almost) no internal gaps, so those are the ones averaged.

    python tools/fwd_gaps.py gpurun_out/trace/t/bench_kernel_trace.csv [--min-gap 1] [--start embed_pe]
"""
import csv
import re
import sys


def forwards(rows, start=None):
    """Cut the trace into calls: at each `start` kernel (name substring) when given, else at the two
    length-mask launches a teacher-forced forward begins with."""
    if start:
        st = [i for i, r in enumerate(rows) if start in r["Kernel_Name"]]
    else:
        st = [i for i, r in enumerate(rows) if "length_mask" in r["Kernel_Name"] and i + 1 < len(rows)
              and "length_mask" in rows[i + 1]["Kernel_Name"]]
        # round 5: the first encoder block writes the masks (fs2_enc_embed_attn_block); a forward
        # then starts at the conditioning launch, or at that block when there is none
        for marker in ("cond_kernel", "enc_attn_block_kernel<true", "enc_attn_block_kernelILb1"):
            if len(st) < 2:
                st = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    return [rows[a:b] for a, b in zip(st, st[1:])]


def main(path, min_gap=0.0, start=None):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    fw = forwards(rows, start)
    n = max(set(len(f) for f in fw), key=lambda k: sum(len(f) == k for f in fw))  # the usual launch count
    inner = lambda f: sum(int(f[i]["Start_Timestamp"]) - int(f[i - 1]["End_Timestamp"]) for i in range(1, len(f))) / 1e3
    graphed = [f for f in fw if len(f) == n and inner(f) < 5.0]
    segs = graphed[-8:] if graphed else [f for f in fw if len(f) == n][-8:]
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
    walls = [(int(f[-1]["End_Timestamp"]) - int(f[0]["Start_Timestamp"])) / 1e3 for f in segs]
    print(f"kernels {n}: busy {tot_d:.1f} us, gaps {tot_g:.1f} us; {len(segs)} graph-replayed forwards averaged "
          f"(wall {min(walls):.1f}..{max(walls):.1f} us)")


if __name__ == "__main__":
    mg = float(sys.argv[sys.argv.index("--min-gap") + 1]) if "--min-gap" in sys.argv else -1e9
    main(sys.argv[1], mg, sys.argv[sys.argv.index("--start") + 1] if "--start" in sys.argv else None)
