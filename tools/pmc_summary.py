#!/usr/bin/env python3
"""Summarise tools/pmc_cmd.sh output: per-dispatch mean of every counter for the kernels whose
name matches a pattern (optionally a grid size), plus derived ratios.
    python tools/pmc_summary.py gpurun_out/pmc_c9_8p conv_gemm [grid]"""
import csv
import glob
import sys
from collections import defaultdict

d, pat = sys.argv[1], sys.argv[2]
grid = sys.argv[3] if len(sys.argv) > 3 else None
vals = defaultdict(list)
for f in sorted(glob.glob(f"{d}/g*/pmc_counter_collection.csv")):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"] or (grid and r["Grid_Size"] != grid):
            continue
        per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (c, _), v in per.items():
        vals[c].append(v)
m = {c: sum(v) / len(v) for c, v in vals.items()}
for c in sorted(m):
    print(f"{c:32s} {m[c]:16.1f}  (n={len(vals[c])})")
g = m.get("GRBM_GUI_ACTIVE")
if g:
    print("--- derived")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (kernel cycles = GRBM / 8); the MFMA busy
        # cycles are summed over all 1,024 SIMDs (MI355X_MICROARCH.md, PMC units)
        print(f"MFMA busy per SIMD = busy / (1024 x GRBM/8)  {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g / 8):.3f}")
        print(f"kernel cycles (GRBM/8)                      {g / 8:.0f}")
    if "SQ_WAIT_ANY" in m and "SQ_BUSY_CYCLES" in m:
        print(f"WAIT_ANY / WAVE-cycles-ish          {m['SQ_WAIT_ANY'] / max(1, m.get('SQ_WAVE_CYCLES', m['SQ_BUSY_CYCLES'])):.3f}")
