#!/usr/bin/env python3
"""Phase timing inside the fused FFN from a trace build (FS2_LIB=abl/libfs2hip_trace.so, ffn.hip
under -DFFN_TRACE=1): wave 0 of every workgroup stamps the shader clock at kernel start, after
the prologue, around each chunk's H hand-off, before and after the LN epilogue; the stamps
go to the packed buffer's spare tail rows. Prints per-phase mean / max cycles over workgroups."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    import bench
    from fs2amd import ops
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    bc = synth_batch(64, 64, seed=1)
    b = to_device(bc, dev)
    P = model.packed(dev)
    B, T = 64, int(bc["max_mel_len"])
    lp = P.dec_layers[0]
    lay = ops.SeqLayout(b["mel_lens"], T)
    h = torch.randn(B * T, 256, generator=torch.Generator().manual_seed(0)).to(dev, torch.bfloat16)
    out = torch.empty_like(h)
    for _ in range(3):
        ops.ffn(h, lp.w12, lp.b1, lp.b2, ks=9, pad=4, ln=lp.ln2, layout=lay, out=out)
    torch.cuda.synchronize()
    R = int(lay.cu[-1])
    nwg = (R + 111) // 112
    assert B * T - nwg >= R, "no spare capacity rows for the stamps"
    st = out.view(torch.int64).reshape(B * T, -1)[B * T - nwg:].flip(0)[:, :32].cpu()
    print("raw wg0:", st[0, :13].tolist())
    n = int(st[0, 31])
    t = st[:, :n].double()
    t0 = t[:, 0].min()
    names = ["prologue"] + [f"c{c}:{p}" for c in range(4) for p in ("gemm1", "h_handoff", "gemm2")] + ["epilogue"]
    # stamps: 0 start, 1 after prologue, per chunk: before write_h, after write_h; then before / after epilogue
    edges = [0, 1]
    for c in range(4):
        edges += [2 + 2 * c, 3 + 2 * c]
    edges += [10, 11]
    print(f"workgroups {t.shape[0]}, stamps {n}; total mean {float((t[:, 11] - t[:, 0]).mean()):.0f} cycles")
    seg = []
    for i in range(1, 12):
        d = t[:, i] - t[:, i - 1]
        seg.append((i, float(d.mean()), float(d.max())))
    labels = ["prologue"]
    for c in range(4):
        labels += [f"c{c} gemm1 (+prev gemm2)" if c else "c0 gemm1", f"c{c} write_h"]
    labels += ["c3 gemm2", "epilogue (all)"]
    for (i, mean, mx), lab in zip(seg[:10], labels):
        print(f"{lab:28s} mean {mean:9.0f}  max {mx:9.0f} cycles")
    # epilogue split: 10 before drain, 12 after drain + barrier, 13 after E writes, 11 end
    for lab, i0, i1 in (("  drain vmcnt + barrier", 10, 12), ("  epilogue: v + partial sums", 12, 14),
                        ("  epilogue: mean reduce", 14, 15), ("  epilogue: var partials", 15, 16),
                        ("  epilogue: var reduce", 16, 17), ("  epilogue: y + staging + sync", 17, 18),
                        ("  epilogue: stores", 18, 13), ("  after", 13, 11)):
        d = t[:, i1] - t[:, i0]
        print(f"{lab:28s} mean {float(d.mean()):9.0f}  max {float(d.max()):9.0f} cycles")


def main_enc(nsplit=4, tile_rows=64, with_qkv=True):
    """The encoder's split-hidden FFN (64 x 64 padded rows, the forward's launch form): per-workgroup
    phase stamps from the split-K workspace (past the partials), every split included."""
    import bench
    from fs2amd import ops
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    b = to_device(synth_batch(64, 64, seed=1), dev)
    P = model.packed(dev)
    el, nx = P.enc_layers[0], P.enc_layers[1]
    x = torch.randn(64, 64, 256, generator=torch.Generator().manual_seed(0)).to(dev, torch.bfloat16)
    kw = dict(ks=9, pad=4, ln=el.ln2, lens=b["src_lens"], nsplit=nsplit, tile_rows=tile_rows)
    if with_qkv:
        kw["next_qkv"] = (nx.wqf, nx.bqkv)
    for _ in range(3):
        ops.ffn(x, el.w12, el.b1, el.b2, **kw)
    torch.cuda.synchronize()
    ws = ops.splitk_workspace(dev)
    MB = tile_rows // 16
    ntiles = 4096 // tile_rows
    part = ntiles * nsplit * 4 * 4 * MB * 64 * 16
    nwg = (ntiles * nsplit + 7) & ~7
    st = ws[4096 + part: 4096 + part + 256 * nwg].view(torch.int64).reshape(nwg, 32).cpu()
    ok = st[:, 31] >= 21
    st = st[ok].double()
    last = st[:, 30] == 1
    t0 = st[:, 0].min()
    lab = {1: "prologue (x tile)", 2: "gemm1", 3: "write_h", 10: "gemm2 (+ drain start)", 19: "partials stored + counter",
           20: "partial sums loaded (last)", 18: "LN epilogue to staging (last)", 13: "stores + Q|K|V (last)"}
    print(f"workgroups traced {int(ok.sum())}, last arrivers {int(last.sum())}; start skew "
          f"{float((st[:, 0] - t0).max()):.0f} cycles")

    def seg(rows, a, b_):
        d = rows[:, b_] - rows[:, a]
        return float(d.mean()), float(d.max())
    for a, b_, name in ((0, 1, "prologue: x tile, first units"), (1, 2, "gemm1 (1 chunk)"), (2, 3, "write_h"),
                        (3, 10, "gemm2"), (10, 19, "partial store + counter")):
        m, mx = seg(st, a, b_)
        print(f"{name:32s} mean {m:9.0f} max {mx:9.0f} cycles")
    L = st[last]
    for a, b_, name in ((19, 20, "last: partial loads + sum"), (20, 18, "last: LN epilogue"),
                        (18, 13, "last: stores + next Q|K|V"), (0, 13, "last: total")):
        m, mx = seg(L, a, b_)
        print(f"{name:32s} mean {m:9.0f} max {mx:9.0f} cycles")
    end_all = float((L[:, 13] - t0).max())
    print(f"kernel span (first start -> last end) {end_all:.0f} cycles")


def main_dec_pre():
    """The decoder's in-forward launch: fc + residual + LN prologue, the FFN, the LN epilogue and
    the next block's Q|K|V (packed 112-row tiles, one per CU)."""
    import bench
    from fs2amd import ops
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    bc = synth_batch(64, 64, seed=1)
    b = to_device(bc, dev)
    P = model.packed(dev)
    B, T = 64, int(bc["max_mel_len"])
    lp, nx = P.dec_layers[0], P.dec_layers[1]
    lay = ops.SeqLayout(b["mel_lens"], T)
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(B * T, 256, generator=gen).to(dev, torch.bfloat16)
    att = torch.randn(B * T, 256, generator=gen).to(dev, torch.bfloat16)
    out = torch.empty_like(x)
    kw = dict(ks=9, pad=4, ln=lp.ln2, layout=lay, out=out, pre=(att, lp.wfcf, lp.bfc, lp.ln1))
    if "--no-qkv" not in sys.argv:
        kw["next_qkv"] = (nx.wqf, nx.bqkv)
    for _ in range(3):
        ops.ffn(x, lp.w12, lp.b1, lp.b2, **kw)
    torch.cuda.synchronize()
    R = int(lay.cu[-1])
    nwg = (R + 111) // 112
    assert B * T - nwg >= R, "no spare capacity rows for the stamps"
    st = out.view(torch.int64).reshape(B * T, -1)[B * T - nwg:].flip(0)[:, :32].cpu()
    ok = st[:, 31] >= 21
    t = st[ok].double()
    print(f"workgroups traced {int(ok.sum())}")
    t[:, 27] = t[:, 28]  # kernel entry (slot 28) as column 27 for the table below
    if int(st[0, 31]) >= 25:  # PRE sub-stamps: 21 loads issued, 22 landed, 23 / 24 row passes
        for a, b_, name in ((27, 21, "  PRE: row masks, loads issued"), (21, 22, "  PRE: tiles + fc weights landed"),
                            (22, 23, "  PRE: pass 0 (GEMM0 + LN, 64 rows)"), (23, 24, "  PRE: pass 1"),
                            (24, 0, "  PRE: vectors + ring start")):
            d = t[:, b_] - t[:, a]
            print(f"{name:36s} mean {float(d.mean()):9.0f} max {float(d.max()):9.0f} cycles")
    segs = [(27, 0, "entry -> PRE prologue done"), (0, 1, "x tile landed / first units"), (1, 2, "c0 gemm1"), (2, 3, "c0 write_h"),
            (3, 4, "c0 gemm2 + c1 gemm1"), (4, 5, "c1 write_h"), (5, 6, "c1 gemm2 + c2 gemm1"), (6, 7, "c2 write_h"),
            (7, 8, "c2 gemm2 + c3 gemm1"), (8, 9, "c3 write_h"), (9, 10, "c3 gemm2"), (10, 12, "drain + barrier"),
            (12, 18, "LN epilogue to staging"), (18, 13, "stores + next Q|K|V"), (27, 13, "total")]
    for a, b_, name in segs:
        d = t[:, b_] - t[:, a]
        print(f"{name:36s} mean {float(d.mean()):9.0f} max {float(d.max()):9.0f} cycles")


if __name__ == "__main__":
    if "--dec-pre" in sys.argv:
        main_dec_pre()
    elif "--enc" in sys.argv:
        main_enc(with_qkv="--no-qkv" not in sys.argv)
    else:
        main()
