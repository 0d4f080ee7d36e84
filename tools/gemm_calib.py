#!/usr/bin/env python3
"""Calibration: hipBLASLt (torch.matmul) on the conv-k9 GEMM shape vs our implicit-GEMM kernel.

The decoder FFN Conv1d(256->1024, k=9) is a [M, 9*256] x [9*256, 1024] GEMM after im2col; this
times the library GEMM on an explicit im2col matrix (bf16, f32 accumulate) with HIP events, so
the conv kernel's TFLOP/s has a same-box reference point. Not part of the product path.
"""
import sys
import torch

M = int(sys.argv[1]) if len(sys.argv) > 1 else 24883
dev = torch.device("cuda:0")
for (m, k, n) in ((M, 2304, 1024), (32768, 2304, 1024), (M, 1024, 256), (M, 256, 768), (8192, 8192, 8192)):
    a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"hipblaslt bf16 M={m} K={k} N={n}: {us:.1f} us  {2*m*k*n/us/1e6:.0f} TFLOP/s", flush=True)
