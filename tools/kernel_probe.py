#!/usr/bin/env python3
"""Launch ONE hot-path kernel repeatedly at the bench's cfg2 shapes (for rocprofv3 PMC passes).

    python tools/kernel_probe.py conv9 --reps 20
kernels: ffn (decoder fused FFN, fs2_ffn), enc_ffn_wide / ffn_wide_rows (fs2_ffn_wide at the encoder shape /
on --rows packed decoder rows), ffn_rows / ffn2_rows (decoder FFN fused / two launches on --rows
packed rows), enc_ffn (encoder FFN fused, --nsplit), conv9 (decoder FFN Conv1d k=9 256->1024), conv1 (FFN k=1 1024->256 + res + LN),
qkv, attn, lr (LengthRegulator gather + PE), lr_pad / lr_pad4 (fs2_length_regulate at cfg2 / cfg4), lr_fused / lr_proj (the forward's LR launch without / with
the first Q|K|V), postnet (512->512 k=5 + tanh), vpf / vpf_dp / vpf_en
(fs2_vp_fused sets). --flush MB writes that much before each launch (cold caches).
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
    ap.add_argument("kernel")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--time", action="store_true", help="print mean duration (HIP events) instead of profiling")
    ap.add_argument("--nsplit", type=int, default=None, help="ffn / enc_ffn / ffn_rows: fs2_ffn split-hidden workgroups per tile")
    ap.add_argument("--tile-rows", type=int, default=None, help="ffn / enc_ffn / ffn_rows: fs2_ffn tile rows (112 / 64)")
    ap.add_argument("--rows", type=int, default=11141, help="ffn_rows / ffn2_rows: packed decoder rows (free-running cfg2: 11141)")
    ap.add_argument("--flush", type=int, default=0, help="MB written before each launch (cold L2 / MALL); --time subtracts it")
    a = ap.parse_args()
    import bench
    from fs2amd import _lib as L, ops
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, a.dtype)
    bc = synth_batch(64, 64, seed=1)
    b = to_device(bc, dev)
    if a.dtype == "fp8":
        model.calibrate_fp8(**to_device(synth_batch(64, 64, seed=1000), dev))
    P = model.packed(dev)
    B, T = 64, int(bc["max_mel_len"])
    dt = ops.torch_dtype(P.act_dtype)
    lp = P.dec_layers[0]
    g = torch.Generator().manual_seed(0)
    rnd = lambda *s: torch.randn(*s, generator=g).to(dev, dt)
    lens = b["mel_lens"]
    # decoder kernels run on packed valid frames, as in the forward (runtime._stage2)
    lay = ops.SeqLayout(lens, T)
    if a.kernel == "conv9" and lp.fp8 is not None:
        h = rnd(B * T, 256).to(torch.float8_e4m3fn)
        fn = lambda: ops.conv1d(h, lp.fp8.w1, lp.b1, cin=256, ks=9, pad=4, compute=L.FS2_FP8,
                                epilogue=L.EPI_BIAS_RELU, out_dtype=L.FS2_FP8, out_scale=1.0 / lp.fp8.s_f,
                                col_scale=lp.fp8.cs1, layout=lay)
    elif a.kernel == "conv9":
        h = rnd(B * T, 256)
        fn = lambda: ops.conv1d(h, lp.w1, lp.b1, cin=256, ks=9, pad=4, compute=P.compute, epilogue=L.EPI_BIAS_RELU,
                                out_dtype=P.act_dtype, layout=lay)
    elif a.kernel == "ffn":  # fused FFN (fs2_ffn): conv-k9 + ReLU + conv-k1 + res + LN, packed rows
        h = rnd(B * T, 256)
        out = torch.empty_like(h)
        fn = lambda: ops.ffn(h, lp.w12, lp.b1, lp.b2, ks=9, pad=4, ln=lp.ln2, layout=lay, out=out, nsplit=a.nsplit, tile_rows=a.tile_rows)
    elif a.kernel in ("ffn_rows", "ffn2_rows"):  # decoder FFN on fewer packed rows (free-running), fused / two launches
        T2 = 959
        l2 = torch.full((64,), a.rows // 64, dtype=torch.int64)
        l2[: a.rows - int(l2.sum())] += 1
        lay2 = ops.SeqLayout(l2.to(dev), T2)
        lay2.rows_hint = a.rows
        h = rnd(lay2.capacity, 256)
        out = torch.empty_like(h)
        if a.kernel == "ffn_rows":
            fn = lambda: ops.ffn(h, lp.w12, lp.b1, lp.b2, ks=9, pad=4, ln=lp.ln2, layout=lay2, out=out, nsplit=a.nsplit,
                                 tile_rows=a.tile_rows)
        else:
            def fn():
                f = ops.conv1d(h, lp.w1, lp.b1, cin=256, ks=9, pad=4, compute=P.compute, epilogue=L.EPI_BIAS_RELU,
                               out_dtype=P.act_dtype, layout=lay2)
                ops.conv1d(f, lp.w2, lp.b2, cin=1024, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_RES_LN,
                           out_dtype=P.act_dtype, residual=h, ln=lp.ln2, layout=lay2, out=out)
    elif a.kernel == "enc_ffn":  # encoder FFN fused (split-hidden), padded 64 x 64 rows with lens
        el = P.enc_layers[0]
        xe = rnd(64, 64, 256)
        fn = lambda: ops.ffn(xe, el.w12, el.b1, el.b2, ks=9, pad=4, ln=el.ln2, lens=b["src_lens"], nsplit=a.nsplit,
                              tile_rows=a.tile_rows)
    elif a.kernel == "enc_ffn_wide":  # encoder FFN as fs2_ffn_wide (two wide-tile launches)
        el = P.enc_layers[0]
        xe = rnd(64, 64, 256)
        fn = lambda: ops.ffn_wide(xe, el.w12, el.b1, el.b2, ks=9, pad=4, ln=el.ln2, lens=b["src_lens"])
    elif a.kernel == "ffn_wide_rows":  # decoder FFN as fs2_ffn_wide on --rows packed rows
        l3 = torch.full((64,), a.rows // 64, dtype=torch.int64)
        l3[: a.rows - int(l3.sum())] += 1
        lay3 = ops.SeqLayout(l3.to(dev), 959)
        lay3.rows_hint = a.rows
        h3 = rnd(lay3.capacity, 256)
        out3 = torch.empty_like(h3)
        fn = lambda: ops.ffn_wide(h3, lp.w12, lp.b1, lp.b2, ks=9, pad=4, ln=lp.ln2, layout=lay3, out=out3)
    elif a.kernel == "mel":  # mel_linear: packed decoder rows -> padded [B, T, 80] f32 + the bf16 copy
        h = rnd(B * T, 256)
        mel_bf = torch.empty(B, T, 80, device=dev, dtype=torch.bfloat16)
        fn = lambda: ops.conv1d(h, P.mel_w, P.mel_b, cin=256, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_BIAS,
                                out_dtype=L.FS2_F32, src_layout=lay, out2=mel_bf)
    elif a.kernel == "conv1":
        f, h = rnd(B * T, 1024), rnd(B * T, 256)
        fn = lambda: ops.conv1d(f, lp.w2, lp.b2, cin=1024, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_RES_LN,
                                out_dtype=P.act_dtype, residual=h, ln=lp.ln2, layout=lay)
    elif a.kernel == "fc":  # attention output projection + residual + LN (decoder, packed rows)
        o, h = rnd(B * T, 256), rnd(B * T, 256)
        fn = lambda: ops.conv1d(o, lp.wfc, lp.bfc, cin=256, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_RES_LN,
                                out_dtype=P.act_dtype, residual=h, ln=lp.ln1, layout=lay)
    elif a.kernel == "qkv":
        h = rnd(B * T, 256)
        fn = lambda: ops.conv1d(h, lp.wqkv, lp.bqkv, cin=256, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_BIAS,
                                out_dtype=P.act_dtype, layout=lay)
    elif a.kernel == "attn":
        qkv = rnd(B * T, 768)
        fn = lambda: ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay)
    elif a.kernel == "attn_free":  # free-running-like packed attention: 63 short sequences + one of 959 frames
        lf = torch.randint(60, 300, (64,), generator=g)
        lf[7] = 959
        layf = ops.SeqLayout(lf.to(dev), 960)
        layf.rows_hint = ops.rows_bucket(int(lf.sum()), 64 * 960)
        qkvf = rnd(layf.capacity, 768)
        fn = lambda: ops.attention(qkvf, None, 2, 128, 128 ** 0.5, layout=layf)
    elif a.kernel == "lr":
        x = rnd(B, 64, 256)
        cum, ml, _ = ops.lr_durations(b["d_targets"])
        fn = lambda: ops.lr_expand(x, cum, ml, T, pe=P.dec_pe, out_dtype=P.act_dtype, out_layout=lay)
    elif a.kernel == "lr4":  # LR stress shape (cfg4: B=256, L 16..160, T ~1000), bf16 + PE
        b4 = to_device(synth_batch(256, 16, 160, seed=1), dev)
        x4 = torch.randn(256, b4["texts"].shape[1], 256, generator=g).to(dev, dt)
        cum4, ml4, _ = ops.lr_durations(b4["d_targets"])
        fn = lambda: ops.lr_expand(x4, cum4, ml4, int(b4["max_mel_len"]), pe=P.dec_pe, out_dtype=P.act_dtype)
    elif a.kernel in ("lr_pad", "lr_pad4"):  # fs2_length_regulate: the padded contract in one launch
        bb = b if a.kernel == "lr_pad" else to_device(synth_batch(256, 16, 160, seed=1), dev)
        xq = torch.randn(*bb["texts"].shape, 256, generator=g).to(dev, dt)
        Tq = int(bb["max_mel_len"])
        fn = lambda: ops.length_regulate(xq, bb["d_targets"], Tq)
    elif a.kernel in ("lr_fused", "lr_fused4"):  # the forward's one-launch LR (scan + layout + gather + PE)
        bb = b if a.kernel == "lr_fused" else to_device(synth_batch(256, 16, 160, seed=1), dev)
        Bq, Lq = bb["texts"].shape
        xq = torch.randn(Bq, Lq, 256, generator=g).to(dev, dt)
        Tq = int(bb["max_mel_len"])
        fn = lambda: ops.lr_fused(xq, bb["mel_lens"], Tq, pe=P.dec_pe, out_dtype=P.act_dtype, dur=bb["d_targets"])
    elif a.kernel == "lr_proj":  # lr_fused + the decoder's first Q|K|V by linearity (fs2_lr_fused_proj)
        from fs2amd.runtime import _qkv_pe
        Lq = b["texts"].shape[1]
        xq = torch.randn(B, Lq, 256, generator=g).to(dev, dt)
        xw = torch.randn(B * Lq, 768, generator=g).to(dev)
        tab = _qkv_pe(P, T)
        fn = lambda: ops.lr_fused(xq, b["mel_lens"], T, pe=P.dec_pe, out_dtype=P.act_dtype, dur=b["d_targets"],
                                  proj=(xw, tab))
    elif a.kernel == "postnet":
        y = rnd(B, T, 512)
        pl = P.postnet[1]
        fn = lambda: ops.conv1d(y, pl.w, pl.b, cin=512, ks=5, pad=2, compute=P.compute, epilogue=L.EPI_BIAS_TANH,
                                out_dtype=P.act_dtype)
    elif a.kernel == "wconv":  # the same PostNet conv on the weight-streamed kernel (fs2_wconv)
        y = rnd(B, T, 512)
        pl = P.postnet[1]
        fn = lambda: ops.wconv(y, pl.wfr, pl.b, ks=5, pad=2)
    elif a.kernel in ("pn_tail_fused", "pn_tail"):  # PostNet layers 3 + 4 in one launch / the N = 80 tail alone
        y = rnd(B, T, 512)
        pl, pt = P.postnet[3], P.postnet[4]
        res = torch.randn(B, T, 80, generator=g).to(dev)
        if a.kernel == "pn_tail":
            fn = lambda: ops.wconv_tail(y, pt.wtail, pt.b, res)
        else:
            fn = lambda: ops.wconv(y, pl.wfr, pl.b, ks=5, pad=2, tail=(pt.wtail, pt.b, res))
    elif a.kernel in ("postnet_first", "postnet_first_bf", "postnet_last"):
        # PostNet 80->512 (f32 mel in, or its bf16 copy) / 512->80 + residual
        mel = torch.randn(B, T, 80, generator=g).to(dev)
        if a.kernel == "postnet_first_bf":
            mel = mel.to(torch.bfloat16)
        if a.kernel.startswith("postnet_first"):
            pl = P.postnet[0]
            fn = lambda: ops.conv1d(mel, pl.w, pl.b, cin=pl.cin, ks=pl.k, pad=pl.p, compute=P.compute,
                                    epilogue=L.EPI_BIAS_TANH, out_dtype=P.act_dtype)
        else:
            y = rnd(B, T, 512)
            pl = P.postnet[-1]
            fn = lambda: ops.conv1d(y, pl.w, pl.b, cin=pl.cin, ks=pl.k, pad=pl.p, compute=P.compute,
                                    epilogue=L.EPI_BIAS_RES, out_dtype=L.FS2_F32, residual=mel)
    elif a.kernel == "cond":  # speaker + emotion/arousal/valence conditioning vectors
        fn = lambda: ops.cond_vectors(b["speakers"], P.spk_table, b["emotions"], b["arousals"], b["valences"],
                                      P.emo_table, P.aro_table, P.val_table, P.emo_w, P.emo_b, P.d_model)
    elif a.kernel == "layout":  # packed-sequence layout of the decoder frames
        fn = lambda: ops.SeqLayout(lens, T)
    elif a.kernel in ("vp_c1", "vp_c2", "vpcols"):  # column-split duration + pitch predictors
        from fs2amd.runtime import variance_predictors
        F = P.vpcols.dp
        xe = rnd(64, 64, 256)
        le = b["src_lens"]
        y1 = torch.randn(64, 64, 512, generator=g).to(dev)
        h = rnd(64, 64, 1024)
        if a.kernel == "vp_c1":
            fn = lambda: ops.conv1d(xe, F.w1, F.b1, cin=2 * F.c, ks=F.k, pad=F.p, compute=L.FS2_BF16,
                                    epilogue=L.EPI_BIAS_RELU, out_dtype=L.FS2_F32, cin_block=F.c, cin_src=(0, 0))
        elif a.kernel == "vp_c2":
            fn = lambda: ops.conv1d(h, F.w2, F.b2, cin=3 * F.c, ks=F.k, pad=F.p, compute=L.FS2_BF16,
                                    epilogue=L.EPI_BIAS_RELU, out_dtype=L.FS2_F32, cin_block=F.c,
                                    cin_src=(0, 0, F.c), group=(F.c, 2 * F.c))
        else:
            fn = lambda: variance_predictors(F, xe, le)
    elif a.kernel in ("enc_conv9", "enc_ln", "vp"):
        Be, Le = 64, 64
        xe = rnd(Be, Le, 256)
        le = b["src_lens"]
        el = P.enc_layers[0]
        if a.kernel == "enc_conv9":
            fn = lambda: ops.conv1d(xe, el.w1, el.b1, cin=256, ks=9, pad=4, compute=P.compute,
                                    epilogue=L.EPI_BIAS_RELU, out_dtype=P.act_dtype)
        elif a.kernel == "enc_ln":
            fe = rnd(Be, Le, 1024)
            fn = lambda: ops.conv1d(fe, el.w2, el.b2, cin=1024, ks=1, pad=0, compute=P.compute,
                                    epilogue=L.EPI_RES_LN, out_dtype=P.act_dtype, residual=xe, ln=el.ln2, lens=le)
        else:
            from fs2amd.runtime import variance_predictor
            fn = lambda: variance_predictor(P.vp["pitch"], xe, le)
    elif a.kernel in ("vpf", "vpf_dp", "vpf_en"):  # fs2_vp_fused: duration + pitch set, energy set (both: vpf)
        V = P.vpfused
        xe = rnd(64, 64, 256)
        le = b["src_lens"]
        emb_p = (1, b.get("p_targets"), 1.0, P.bins["pitch"], P.var_table["pitch"])
        emb_e = (0, b.get("e_targets"), 1.0, P.bins["energy"], P.var_table["energy"])

        def fn():
            x = xe
            if a.kernel != "vpf_en":
                _, x = ops.vp_fused(x, V.dp, le, embed=emb_p)
            if a.kernel != "vpf_dp":
                ops.vp_fused(x, V.energy, le, embed=emb_e)
    elif a.kernel == "cond_bwd":  # the training conditioning backward (fs2_cond_bwd) at cfg3's B = 16, L = 64
        m = model
        Bq, Lq = 16, 64
        ids = [torch.randint(0, n, (Bq,), generator=g).to(dev) for n in
               (m.speaker_emb.num_embeddings, m.emotion_emb.num_embeddings, m.arousal_emb.num_embeddings,
                m.valence_emb.num_embeddings)]
        tabs = [m.speaker_emb.weight, m.emotion_emb.weight, m.arousal_emb.weight, m.valence_emb.weight]
        lw, lb = m.emotion_linear[0].weight, m.emotion_linear[0].bias
        _, emo_o = ops.cond_vectors(ids[0], tabs[0], ids[1], ids[2], ids[3], tabs[1], tabs[2], tabs[3], lw, lb, 256)
        dyq = torch.randn(Bq, Lq, 256, generator=g).to(dev)
        grads = [torch.zeros_like(t) for t in tabs] + [torch.zeros_like(lw), torch.zeros_like(lb)]
        fn = lambda: ops.cond_bwd(dyq, ids[0], tabs[0], ids[1], ids[2], ids[3], tabs[1], tabs[2], tabs[3], lw, emo_o,
                                  *grads)
    elif a.kernel == "reduce_ln":  # 8 LayerNorm-parameter partial sets (256 partial blocks x 768) in one launch
        parts = [torch.randn(256 * 768, generator=g).to(dev) for _ in range(8)]
        outs = [[torch.empty(256, device=dev) for _ in range(3)] for _ in range(8)]

        def fn():
            q = []
            for p, o in zip(parts, outs):
                ops._defer_add(q, p, M=768, S=256, kind=0, split=256, accumulate=1, outs=o)
            ops.reduce_flush(q, parts[0])
    elif a.kernel in ("reduce_w1", "reduce_w2", "reduce_qkv"):
        # deferred split-partial reductions (fs2_reduce_batch_launch) as the training backward queues
        # them: 8 layers' weight gradients in one launch (partials past the 256 MB MALL, as in a step)
        KS, N, C, S = {"reduce_w1": (9, 1024, 256, 4), "reduce_w2": (1, 256, 1024, 16),
                       "reduce_qkv": (1, 768, 256, 16)}[a.kernel]
        M = KS * N * C
        parts = [torch.randn(S * M, generator=g).to(dev) for _ in range(8)]
        outs = [torch.empty(N, C, KS, device=dev) for _ in range(8)]
        print(f"bytes per launch {8 * (S + 1) * M * 4 / 1e6:.1f} MB")

        def fn():
            q = []
            for p, o in zip(parts, outs):
                ops._defer_add(q, p, M=M, S=S, kind=1, KS=KS, N=N, C=C, split=N, accumulate=1, outs=(o,))
            ops.reduce_flush(q, parts[0])
    else:
        raise SystemExit(f"unknown kernel {a.kernel}")
    flush_buf = torch.empty(a.flush << 18, device=dev, dtype=torch.float32) if a.flush else None
    if flush_buf is not None:
        fn0 = fn

        def fn():
            flush_buf.zero_()
            fn0()
    if a.time:
        # the reps are captured as one HIP graph and replayed: small launches are host-bound when
        # issued from Python one by one (~15 us of ctypes / allocator work per call)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
            torch.cuda.synchronize(dev)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for _ in range(a.reps):
                    fn()
            gr.replay()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(3):
                gr.replay()
            e1.record(s)
            e1.synchronize()
        t = e0.elapsed_time(e1) * 1e3 / (3 * a.reps)
        if flush_buf is not None:  # the flush alone, to subtract
            with torch.cuda.stream(s):
                gf = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gf, stream=s):
                    for _ in range(a.reps):
                        flush_buf.zero_()
                gf.replay()
                torch.cuda.synchronize(dev)
                e0.record(s)
                for _ in range(3):
                    gf.replay()
                e1.record(s)
                e1.synchronize()
            tf = e0.elapsed_time(e1) * 1e3 / (3 * a.reps)
            print(f"{a.kernel}: {t - tf:.2f} us/launch (graph, after a {a.flush} MB flush: {t:.2f} - {tf:.2f})")
            return
        print(f"{a.kernel}: {t:.2f} us/launch (graph)")
        return
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    print("probe done", a.kernel, a.reps)


if __name__ == "__main__":
    main()
