#!/usr/bin/env python3
"""bf16 vs fp32 HIP path, free-running cfg2: how many discrete decisions flip (rounded
durations, pitch/energy buckets) — and how many of those the f32 VariancePredictors prevent."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    import bench
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "fp32")
    args = to_device(synth_batch(64, 64, seed=1, teacher=False), dev)
    va = model.variance_adaptor
    res = {}
    for prec, vp in (("fp32", "fp32"), ("bf16", "fp32"), ("bf16vp", "bf16"), ("bf16x3vp", "bf16x3")):
        model.set_precision(prec[:4], vp)
        with torch.no_grad():
            out = model(**args)
        torch.cuda.synchronize()
        res[prec] = out
    for tag in ("bf16", "bf16vp", "bf16x3vp"):
        report(res["fp32"], res[tag], va, tag)


def report(f, b, va, tag):
    valid = ~f[6]
    dflip = int(((f[5] != b[5]) & valid).sum())
    pb = torch.bucketize(f[2], va.pitch_bins), torch.bucketize(b[2], va.pitch_bins)
    eb = torch.bucketize(f[3], va.energy_bins), torch.bucketize(b[3], va.energy_bins)
    n = int(valid.sum())
    print(f"[{tag}] phonemes {n}: duration flips {dflip} ({100*dflip/n:.2f}%), pitch bucket flips "
          f"{int(((pb[0] != pb[1]) & valid).sum())}, energy bucket flips {int(((eb[0] != eb[1]) & valid).sum())}; "
          f"log_d max|d| {float((f[4]-b[4]).abs().max()):.4f}, mel_len equal {bool(torch.equal(f[9], b[9]))}")


if __name__ == "__main__":
    main()
