#!/usr/bin/env python3
"""Per-kernel ISA summary from a hipcc -save-temps .s file: registers, spills, MFMA count,
waitcnt list inside the function (to check that a pipelined loop has no stray vmcnt(0))."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):\s*; @", s, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    body = s[m.end():]
    body = body[:body.index(".Lfunc_end")]
    tail = s[m.end():]
    stats = {k: (re.search(r"; " + k + r": (\d+)", tail) or [None, None])[1]
             for k in ("NumVgprs", "NumAgprs", "TotalNumVgprs", "NumSgprs", "ScratchSize", "Occupancy")}
    waits = re.findall(r"s_waitcnt\s+(vmcnt\(\d+\))", body)
    print(name[:90])
    print("  ", stats, "lines", body.count("\n"), "mfma", body.count("v_mfma"),
          "s_barrier", body.count("s_barrier"), "glds", body.count("lds\n") + body.count(" lds "))
    print("   vmcnt:", " ".join(waits[:80]))
