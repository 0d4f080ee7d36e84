#!/usr/bin/env python3
"""Run the HiFi-GAN generator (bf16, random-init V1 weights) on a cfg2-shaped mel batch
[64, 430, 80] a few times (profiling target: tools/prof_voc.sh)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
import torch  # noqa: E402


def main():
    from fs2amd.synth_weights import fill_vocoder
    from fs2amd.vocoder import V1_CONFIG, Generator, flops_per_frame

    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    B, T = int(os.environ.get("VB", 64)), int(os.environ.get("VT", 430))
    dev = torch.device("cuda:0")
    g = Generator(V1_CONFIG)
    fill_vocoder(g, V1_CONFIG)
    g = g.to(dev).eval().set_precision(prec)
    mel = torch.randn(B, T, 80, generator=torch.Generator().manual_seed(0)).to(dev) * 2 - 5
    with torch.no_grad():
        for _ in range(2):
            g.forward_btc(mel)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 3
        for _ in range(n):
            g.forward_btc(mel)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"vocoder {prec} B={B} T={T}: {dt*1e3:.2f} ms, {flops_per_frame()*B*T/dt/1e12:.1f} TFLOP/s, "
          f"{B*T/dt/1e6:.2f} M frames/s")


if __name__ == "__main__":
    main()
