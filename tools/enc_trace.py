#!/usr/bin/env python3
"""Phase timing inside fs2_enc_attn_block from a trace build (FS2_LIB=abl/libfs2hip_enctrace.so,
enc_block.hip under -DENC_TRACE=1, FS2_ENC_TRACE=1): wave 0 of every workgroup stamps the shader
clock at each phase boundary into the split-K workspace's tail. Prints per-phase mean / max
cycles over the cfg2 encoder's 64 workgroups."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)
os.environ["FS2_ENC_TRACE"] = "1"
import torch  # noqa: E402


def main():
    import bench
    from fs2amd import ops
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    b = to_device(synth_batch(64, 64, seed=1), dev)
    P = model.packed(dev)
    lp = P.enc_layers[1]
    x = torch.randn(64, 64, 256, generator=torch.Generator().manual_seed(0)).to(dev, torch.bfloat16)
    for _ in range(3):
        ops.enc_attn_block(x, b["src_lens"], lp.wqf, lp.bqkv, lp.wfcf, lp.bfc, lp.ln1, 2, 128, 128 ** 0.5)
    torch.cuda.synchronize()
    ws = ops.splitk_workspace(dev)
    tail = ws[ws.numel() - 65536:].view(torch.int64).reshape(-1, 16)[:64].cpu().double()
    n = int(tail[0, 15])
    names = ["prologue (x tile, vectors, k-step 0) + barrier", "Q|K|V GEMM (8 k-steps)", "Q|K|V epilogue + fc weight loads",
             "attention", "o barrier + o write + barrier", "fc GEMM", "+ bias + x, LayerNorm", "stores"]
    print(f"workgroups 64, stamps {n}; total mean {float((tail[:, n - 1] - tail[:, 0]).mean()):.0f} cycles")
    for i in range(1, n):
        d = tail[:, i] - tail[:, i - 1]
        print(f"{names[i - 1] if i - 1 < len(names) else i:48s} mean {float(d.mean()):8.0f} max {float(d.max()):8.0f}")
    t0 = float(tail[:, 0].min())
    print(f"start skew {float(tail[:, 0].max()) - t0:.0f} cycles; span {float(tail[:, n - 1].max()) - t0:.0f} cycles")


if __name__ == "__main__":
    main()
