#!/usr/bin/env python3
"""Per-launch PMC table of a whole forward from tools/pmc_cmd.sh passes over tools/fwd_probe.py.

Dispatches are ordered by id and cut into forwards at their two leading length-mask launches (or
the conditioning launch / the first encoder block, as tools/fwd_gaps.py); counters are averaged per launch position over the forwards of the most
common launch count. Units and corrections (MI355X_MICROARCH.md):
* FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is doubled (gfx950 reports half the bytes of a
  16 B/lane streaming read). hbm_MB = 2 * FETCH + WRITE.
* GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel cycles = GRBM / 8.
* SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over every SIMD: MFMA busy = busy / (1024 SIMDs x
  GRBM / 8).

    python tools/pmc_fwd.py gpurun_out/pmc_<tag> [--json out.json]
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

N_SIMD = 1024
N_XCD = 8


def dispatches(d):
    """{dispatch_id: {"name", "grid", "wg", counter: value}} over every pass directory."""
    out = {}
    for f in sorted(glob.glob(f"{d}/g*/**/*counter_collection.csv", recursive=True)):
        per = defaultdict(float)
        meta = {}
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            per[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            meta[k] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]))
        tag = f  # one pass per file: dispatch ids are per process, so key by (pass, id)
        for (k, c), v in per.items():
            e = out.setdefault((tag, k), {"name": meta[k][0], "grid": meta[k][1], "wg": meta[k][2]})
            e[c] = v
    return out


def forwards(seq):
    st = [i for i in range(len(seq) - 1) if "length_mask" in seq[i]["name"] and "length_mask" in seq[i + 1]["name"]]
    # round 5: the first encoder block writes the masks; a forward starts at the conditioning
    # launch, or at that block when there is none (as tools/fwd_gaps.py)
    for marker in ("cond_kernel", "enc_attn_block_kernel<true", "enc_attn_block_kernelILb1"):
        if len(st) < 2:
            st = [i for i in range(len(seq)) if marker in seq[i]["name"]]
    return [seq[a:b] for a, b in zip(st, st[1:] + [len(seq)])]


def main(d, out_json=None):
    ds = dispatches(d)
    passes = defaultdict(list)
    for (tag, k), e in ds.items():
        passes[tag].append((k, e))
    tables = []
    for tag, lst in passes.items():
        seq = [e for _, e in sorted(lst, key=lambda t: t[0])]
        fws = forwards(seq)
        if not fws:
            continue
        n = max(set(len(f) for f in fws), key=lambda m: sum(len(f) == m for f in fws))
        tables.append([f for f in fws if len(f) == n])
    if not tables:
        raise SystemExit(f"no forwards found under {d}")
    n = len(tables[0][0])
    rows = []
    for i in range(n):
        rec = {"pos": i, "name": re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", tables[0][0][i]["name"]),
               "workgroups": tables[0][0][i]["grid"] // max(1, tables[0][0][i]["wg"])}
        for fws in tables:
            if len(fws[0]) != n:
                continue
            keys = [k for k in fws[0][i] if k not in ("name", "grid", "wg")]
            for k in keys:
                rec[k] = sum(f[i].get(k, 0.0) for f in fws) / len(fws)
        g = rec.get("GRBM_GUI_ACTIVE")
        if "FETCH_SIZE" in rec and "WRITE_SIZE" in rec:
            rec["hbm_MB"] = (2 * rec["FETCH_SIZE"] + rec["WRITE_SIZE"]) * 1024 / 1e6
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in rec:
            rec["mfma_busy"] = rec["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * g / N_XCD)
        if g:
            rec["kernel_kcycles"] = g / N_XCD / 1e3
        rows.append(rec)
    cols = [("hbm_MB", "{:8.1f}"), ("mfma_busy", "{:6.3f}"), ("kernel_kcycles", "{:8.1f}")]
    print(f"{'pos':>3} {'kernel':40s} {'WGs':>6} " + " ".join(f"{c:>14s}" for c, _ in cols))
    for r in rows:
        vals = " ".join(f"{(fmt.format(r[c]) if c in r else '-'):>14s}" for c, fmt in cols)
        print(f"{r['pos']:3d} {r['name'][:40]:40s} {r['workgroups']:6d} {vals}")
    if out_json:
        with open(out_json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None)
