#!/usr/bin/env python3
"""Attention launch-shape A/B at the cfg2 decoder shape (packed valid frames): run the variant
FS2_ATTN_VARIANT selects (read once per process), save its output, and if a saved output of another
variant is given, require bit-identical results.

    FS2_ATTN_VARIANT=2 python tools/attn_ab.py out2.pt
    FS2_ATTN_VARIANT=8 python tools/attn_ab.py out8.pt --against out2.pt
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
    ap.add_argument("out")
    ap.add_argument("--against", default=None)
    a = ap.parse_args()
    import bench
    from fs2amd import ops
    from fs2amd.data import synth_batch

    dev = torch.device("cuda:0")
    bc = synth_batch(64, 64, seed=1)
    T = int(bc["max_mel_len"])
    lens = bc["mel_lens"].to(dev)
    lay = ops.SeqLayout(lens, T)
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(64 * T, 768, generator=g).to(dev, torch.bfloat16)
    outs = [ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay)]
    # padded rows with key lengths too (the non-packed launch)
    qkv_p = torch.randn(16, T, 768, generator=g).to(dev, torch.bfloat16)
    lens_p = torch.randint(0, T + 1, (16,), generator=g).to(dev)
    lens_p[0] = T
    outs.append(ops.attention(qkv_p, lens_p, 2, 128, 128 ** 0.5))
    torch.cuda.synchronize()
    R = int(lay.cu[-1])
    res = [outs[0][:R].cpu(), outs[1].cpu()]
    t = bench._graph_mean_s(lambda: ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay), dev, 20)
    print(f"variant {os.environ.get('FS2_ATTN_VARIANT', 'default')}: {t * 1e6:.2f} us per call (graph)", flush=True)
    torch.save(res, a.out)
    if a.against:
        ref = torch.load(a.against, weights_only=True)
        valid = torch.arange(T, device="cpu")[None, :] < lens_p.cpu()[:, None]
        ok0 = torch.equal(res[0], ref[0])
        ok1 = torch.equal(res[1][valid], ref[1][valid])
        print(f"bit-identical vs {a.against}: packed {ok0}, padded valid rows {ok1}", flush=True)
        if not (ok0 and ok1):
            d = (res[0].float() - ref[0].float()).abs().max()
            print(f"max |d| packed {float(d):.3e}", flush=True)
            sys.exit(1)


if __name__ == "__main__":
    main()
