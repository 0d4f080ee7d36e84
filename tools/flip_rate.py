#!/usr/bin/env python3
"""bf16 vs fp32 HIP path, free-running cfg2 (committed reference inputs): how many discrete
decisions flip (rounded durations, pitch/energy buckets), how large the prediction differences
are relative to the bucket width, and how the VariancePredictor precision changes that."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    from fs2amd.data import to_device
    from fs2amd.model import FastSpeech2
    from _common import configs, load_case, oracle_state_dict

    dev = torch.device("cuda:0")
    pc, mc, _ = configs()
    model = FastSpeech2(pc, mc)
    model.load_state_dict(oracle_state_dict())
    model = model.to(dev).eval()
    args, _, _, _ = load_case("cfg2_free")
    args = to_device(args, dev)
    va = model.variance_adaptor
    res = {}
    for tag, prec, vp in (("fp32", "fp32", "fp32"), ("bf16/vp32", "bf16", "fp32"), ("bf16/vp16", "bf16", "bf16"),
                          ("bf16/vpx3", "bf16", "bf16x3")):
        model.set_precision(prec, vp)
        with torch.no_grad():
            res[tag] = model(**args)
        torch.cuda.synchronize()
    f = res["fp32"]
    valid = ~f[6]
    print(f"p_pred range [{float(f[2][valid].min()):.3f}, {float(f[2][valid].max()):.3f}], bin width "
          f"{float(va.pitch_bins[1] - va.pitch_bins[0]):.4f}; e_pred range [{float(f[3][valid].min()):.3f}, "
          f"{float(f[3][valid].max()):.3f}], bin width {float(va.energy_bins[1] - va.energy_bins[0]):.4f}")
    for tag in ("bf16/vp32", "bf16/vp16", "bf16/vpx3"):
        report(f, res[tag], va, tag)
    # energy prediction error with the pitch embedding pinned to the fp32 buckets (p_targets):
    model.set_precision("bf16", "bf16x3")
    pinned = dict(args, p_targets=f[2])
    model.set_precision("fp32", "fp32")
    with torch.no_grad():
        f2 = model(**pinned)
    model.set_precision("bf16", "bf16x3")
    with torch.no_grad():
        b2 = model(**pinned)
    torch.cuda.synchronize()
    report(f2, b2, va, "bf16/vpx3, pitch pinned")


def report(f, b, va, tag):
    valid = ~f[6]
    n = int(valid.sum())
    dflip = int(((f[5] != b[5]) & valid).sum())
    pb = torch.bucketize(f[2], va.pitch_bins), torch.bucketize(b[2], va.pitch_bins)
    eb = torch.bucketize(f[3], va.energy_bins), torch.bucketize(b[3], va.energy_bins)
    dp, de = (f[2] - b[2]).abs()[valid], (f[3] - b[3]).abs()[valid]
    print(f"[{tag}] {n} phonemes: duration flips {dflip} ({100 * dflip / n:.2f}%), pitch bucket flips "
          f"{100 * int(((pb[0] != pb[1]) & valid).sum()) / n:.2f}% (max |db| {int((pb[0] - pb[1]).abs().max())}), "
          f"energy bucket flips {100 * int(((eb[0] != eb[1]) & valid).sum()) / n:.2f}% (max |db| "
          f"{int((eb[0] - eb[1]).abs().max())}); |dp| mean {float(dp.mean()):.2e} max {float(dp.max()):.2e}, "
          f"|de| mean {float(de.mean()):.2e} max {float(de.max()):.2e}, log_d max|d| "
          f"{float((f[4] - b[4]).abs()[valid].max()):.4f}")


if __name__ == "__main__":
    main()
