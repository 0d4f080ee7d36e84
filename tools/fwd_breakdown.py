#!/usr/bin/env python3
"""Per-launch-group time of the cfg2 forward (bench.forward_timers_graph: event nodes inside one
captured graph, replayed; falls back to eager HIP events), the FFT-block GEMM fraction and the LR
fraction, plus the graph-replayed step time. For A/B runs under FS2_* switches:
    FS2_LR_STORE=plain python tools/fwd_breakdown.py [--tag name]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    import bench
    from fs2amd.data import synth_batch, to_device

    tag = sys.argv[sys.argv.index("--tag") + 1] if "--tag" in sys.argv else "default"
    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    bc = synth_batch(64, 64, seed=1)
    b = to_device(bc, dev)
    el = bench.timed_steps(model, b, dev, 50, 20, True)
    try:
        fwd = bench.forward_timers_graph(model, b)
        how = "graph"
    except Exception as e:  # noqa: BLE001
        print(f"in-graph timing failed ({e!r}); eager events", file=sys.stderr)
        fwd = bench.forward_timers(model, b)
        how = "eager"
    brk = bench.forward_breakdown(fwd, bc, bench.BF16_PEAK_TFLOPS)
    print(json.dumps({"tag": tag, "timing": how, "ms_per_step": round(el / 50 * 1e3, 4),
                      "fft_gemm_frac": brk.get("fft_gemm", {}).get("frac"), "lr_frac": brk.get("lr", {}).get("frac"),
                      "us": brk["us_per_forward"]}))


if __name__ == "__main__":
    main()
