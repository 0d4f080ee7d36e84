#!/usr/bin/env python3
"""profiles/ffn_pre_traffic.json (read by bench.py for the roofline's `traffic`) from a per-launch
PMC table of eager cfg2 forwards (tools/pmc_fwd.sh -> table.json): the decoder's last fused
fc + FFN launch (the roofline launch) and the five that also project the next block's Q|K|V.

    python tools/pre_traffic.py gpurun_out/pmcf_<tag>/table.json profiles/<round>/pmc_forward.json [out.json]
"""
import json
import sys

FRAMES, D = 24883, 256


def main(table, source):
    rows = json.load(open(table))
    ffn = [r for r in rows if "ffn_fused_kernel<9, 4, 7, true>" in r["name"]]  # the decoder PRE launches
    last, rest = ffn[-1], ffn[:-1]
    algo = {"att_rows_in": FRAMES * D * 2, "x_rows_in": FRAMES * D * 2, "y_rows_out": FRAMES * D * 2,
            "weights_once": 2 * (256 * 256 + 256 * 9 * 1024 + 1024 * 256)}
    hbm = (2 * last["FETCH_SIZE"] + last["WRITE_SIZE"]) * 1024
    out = {
        "kernel": "ffn_fused_kernel<9,4,7,PRE=true> (decoder's last block: fc + residual + LN prologue, FFN, LN "
                  "epilogue; the bench line's roofline launch)",
        "launch_position": last["pos"],
        "FETCH_SIZE_KiB": last["FETCH_SIZE"],
        "WRITE_SIZE_KiB": last["WRITE_SIZE"],
        "hbm_bytes_per_launch": hbm,
        "correction": "FETCH_SIZE x2 (gfx950 reports half the bytes of 16 B/lane streaming reads); KiB units",
        "algorithmic_bytes": sum(algo.values()),
        "traffic_over_algorithmic": hbm / sum(algo.values()),
        "algorithmic_breakdown": algo,
        "mfma_busy_per_simd": last.get("mfma_busy"),
        "with_next_qkv_launches": {
            "positions": [r["pos"] for r in rest],
            "hbm_bytes_per_launch": sum((2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024 for r in rest) / max(1, len(rest)),
            "mfma_busy_per_simd": sum(r.get("mfma_busy", 0.0) for r in rest) / max(1, len(rest)),
        },
        "note": "the excess over algorithmic is the weights fetched once per XCD L2 (8 x 5.4 MB): every workgroup "
                "streams all weights for its 112 rows and the 8 L2s are not shared; FETCH counts Infinity-Cache hits too",
        "source": f"{source} (tools/pmc_fwd.sh over tools/fwd_probe.py: eager cfg2 forwards, one rocprofv3 --pmc "
                  "pass per counter group)",
    }
    dst = sys.argv[3] if len(sys.argv) > 3 else "profiles/ffn_pre_traffic.json"
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("launch_position", "hbm_bytes_per_launch", "traffic_over_algorithmic",
                                          "mfma_busy_per_simd")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
