#!/usr/bin/env python3
"""Eager cfg2 forwards of the bench batch, for rocprofv3 PMC passes over a whole forward
(tools/pmc_fwd.py turns the counters into a per-launch table).

    python tools/fwd_probe.py [--fwd 4] [--dtype bf16] [--free]
--free: the free-running synthesis batch (durations predicted, one host read) instead of the
teacher-forced bench batch.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fwd", type=int, default=4)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--free", action="store_true")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--phonemes", type=int, default=64)
    ap.add_argument("--lmax", type=int, default=None)
    a = ap.parse_args()
    import bench
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, a.dtype)
    b = to_device(synth_batch(a.batch, a.phonemes, a.lmax, seed=1, teacher=not a.free), dev)
    if a.dtype == "fp8":
        model.calibrate_fp8(**to_device(synth_batch(a.batch, a.phonemes, a.lmax, seed=1000), dev))
    with torch.no_grad():
        for _ in range(2):
            model(**b)
        torch.cuda.synchronize()
        for _ in range(a.fwd):
            model(**b)
    torch.cuda.synchronize()
    print("fwd_probe done", a.fwd)


if __name__ == "__main__":
    main()
