#!/usr/bin/env python3
"""Time one conv launch shape over a sweep of row counts M (B=1, T=M): exposes wave
quantisation (tile rounds over 256 CUs x workgroups-per-CU). HIP events, mean of --reps."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "expressive-fastspeech2-mandarin_amd"))
from fs2amd import _lib as L, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cin", type=int, default=256)
ap.add_argument("--n", type=int, default=1024)
ap.add_argument("--ks", type=int, default=9)
ap.add_argument("--epi", default="relu")
ap.add_argument("--ms", default="8192,12288,16384,20480,24576,24704,24883,25600,27520,28672,32768")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
w = ops.pack_conv_weight(torch.randn(a.n, a.cin, a.ks, device=dev, generator=g) * 0.02, L.FS2_BF16)
bias = torch.zeros(a.n, device=dev)
ln = (torch.ones(a.n, device=dev), torch.zeros(a.n, device=dev), 1e-5)
for M in [int(x) for x in a.ms.split(",")]:
    x = torch.randn(1, M, a.cin, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(1, M, a.n, device=dev, dtype=torch.bfloat16)
    kw = dict(cin=a.cin, ks=a.ks, pad=(a.ks - 1) // 2, compute=L.FS2_BF16, out=out)
    if a.epi == "res_ln":
        res = torch.randn(1, M, a.n, device=dev, generator=g).to(torch.bfloat16)
        fn = lambda: ops.conv1d(x, w, bias, epilogue=L.EPI_RES_LN, residual=res, ln=ln, **kw)
    else:
        fn = lambda: ops.conv1d(x, w, bias, epilogue=L.EPI_BIAS_RELU if a.epi == "relu" else L.EPI_BIAS, **kw)
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.reps
    fl = 2.0 * M * a.cin * a.ks * a.n
    print(f"M={M:6d} {us:8.2f} us  {fl / us / 1e6:7.1f} TF/s  us/krow={us / M * 1e3:.3f}", flush=True)
