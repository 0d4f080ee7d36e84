#!/usr/bin/env python3
"""Phase timing inside fs2_ffn_wide from a trace build (ffn_wide.hip under -DWIDE_TRACE=1, loaded
through FS2_LIB; `python tools/wide_trace.py build` makes tracelib/libfs2hip_widetrace.so here):
thread 0 of every workgroup stamps the shader clock at each phase boundary into the split-K
workspace's tail. Prints per-phase mean / max cycles of both launches.

    FS2_LIB=$PWD/tracelib/libfs2hip_widetrace.so python tools/wide_trace.py [--rows N]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)

NAMES = {1: ["prologue: x tile DMA, weight ring, row positions, barrier", "conv-k GEMM (main loop) + drain",
             "H staging + stores (drained)"],
         2: ["operand loads (drained)", "GEMM + partial exchange through LDS", "+ b2 + x, z stores (drained) + barrier",
             "arrival counter", "LayerNorm + stores (last arriver only)"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="run")
    ap.add_argument("--rows", type=int, default=0, help="packed decoder rows (0: the cfg2 encoder's 64 x 64 padded rows)")
    a = ap.parse_args()
    if a.what == "build":
        import __graft_entry__ as g
        os.makedirs(os.path.join(REPO, "tracelib"), exist_ok=True)
        g.build_hip(extra_flags=["-DWIDE_TRACE=1"], out=os.path.join(REPO, "tracelib", "libfs2hip_widetrace.so"))
        return
    import torch
    import bench
    from fs2amd import ops
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    b = to_device(synth_batch(64, 64, seed=1), dev)
    P = model.packed(dev)
    g = torch.Generator().manual_seed(0)
    if a.rows:
        lp = P.dec_layers[0]
        l3 = torch.full((64,), a.rows // 64, dtype=torch.int64)
        l3[: a.rows - int(l3.sum())] += 1
        lay = ops.SeqLayout(l3.to(dev), 959)
        lay.rows_hint = a.rows
        h = torch.randn(lay.capacity, 256, generator=g).to(dev, torch.bfloat16)
        fn = lambda: ops.ffn_wide(h, lp.w12, lp.b1, lp.b2, ks=9, pad=4, ln=lp.ln2, layout=lay)
    else:
        el = P.enc_layers[0]
        xe = torch.randn(64, 64, 256, generator=g).to(dev, torch.bfloat16)
        fn = lambda: ops.ffn_wide(xe, el.w12, el.b1, el.b2, ks=9, pad=4, ln=el.ln2, lens=b["src_lens"])
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ws = ops.splitk_workspace(dev)
    tail = ws[ws.numel() - 65536:].view(torch.int64).reshape(2, 512, 8).cpu().double()
    for k in (1, 2):
        t = tail[k - 1]
        n = t[:, 7]
        used = n > 0
        t, n = t[used], n[used]
        print(f"launch {k}: {int(used.sum())} workgroups traced (of <= 512)")
        for nn in sorted(set(int(v) for v in n.tolist())):
            tt = t[n == nn]
            tot = tt[:, nn - 1] - tt[:, 0]
            print(f"  {tt.shape[0]} workgroups with {nn} stamps: total mean {float(tot.mean()):.0f} max {float(tot.max()):.0f}")
            for i in range(1, nn):
                d = tt[:, i] - tt[:, i - 1]
                nm = NAMES[k][i - 1] if i - 1 < len(NAMES[k]) else str(i)
                print(f"    {nm:60s} mean {float(d.mean()):8.0f} max {float(d.max()):8.0f}")
        t0 = float(t[:, 0].min())
        print(f"  start skew {float(t[:, 0].max()) - t0:.0f}; span {float((t[:, 6] * 0 + t.max(1).values).max()) - t0:.0f} cycles")


if __name__ == "__main__":
    main()
