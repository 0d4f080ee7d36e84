"""Training forward of FastSpeech2 (train.py step, cfg3) on the fs2hip kernels + autograd.

Same train-mode semantics as the reference (model/fastspeech2.py:73-148 with ``self.training``):
dropout after the attention output projection and after the FFN (transformer/SubLayers.py:54,90,
p = encoder/decoder_dropout), VariancePredictor dropout (model/modules.py:223,235), the PostNet's
hard-coded ``F.dropout(0.5)`` (transformer/Layers.py:133-134), BatchNorm1d on batch statistics
(running buffers updated), decoder crop to ``max_seq_len`` (transformer/Models.py:154-162), PE
tables never recomputed in training (Models.py:82,145).

Where the arithmetic runs:
  * every Conv1d / Linear with >= 4 outputs: :class:`Conv1dFn` — forward and input-gradient on
    ``fs2_conv1d`` (MFMA; the input gradient is the same per-sequence conv with the taps flipped
    and the weight transposed), weight gradient as ONE hipBLASLt GEMM over the tap-unfolded input;
  * self-attention: :class:`AttentionFn` — forward ``fs2_attention``, backward
    ``fs2_attention_bwd`` (flash-style dQ and dK/dV kernels, no T x T tensor);
  * LengthRegulator: the duration scan and source-index map on ``fs2_lr_durations`` /
    ``fs2_lr_expand`` (+ the decoder PE), its gradient a deterministic segmented sum
    (``fs2_lr_backward``, LengthRegulatorFn); bucketize + pitch / energy embedding on
    ``fs2_variance_embed_ex`` with the table gradient on ``fs2_embedding_bwd`` (VarianceEmbedFn);
  * LayerNorm, dropout, BatchNorm, embeddings, losses: torch on the device.
Parity: tests/test_gpu_train.py against the reference's own gradients (train_grads.npz).
"""
import ctypes
import os

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib as L
from . import ops


def _act(x, compute):
    return x.contiguous() if compute == L.FS2_F32 else x.to(torch.bfloat16).contiguous()


class Conv1dFn(torch.autograd.Function):
    """y[b,t] = sum_k W_k x[b, t+k-pad] + bias over padded sequences [B, T, C] (zero outside
    [0, T) per sequence, as nn.Conv1d on the [B, C, T] transpose). w: nn.Conv1d [N, Cin, KS] or
    nn.Linear [N, Cin]. f32 in / f32 out; ``compute`` is the MFMA operand type."""

    @staticmethod
    def forward(ctx, x, w, b, pad, compute):
        w3 = (w if w.dim() == 3 else w.unsqueeze(-1)).detach()
        N, Cin, KS = w3.shape
        xc = _act(x, compute)
        y = ops.conv1d(xc, ops.pack_conv_weight(w3, compute), None if b is None else b.detach().float().contiguous(),
                       cin=Cin, ks=KS, pad=pad, compute=compute, epilogue=L.EPI_BIAS, out_dtype=L.FS2_F32)
        ctx.save_for_backward(xc, w3)
        ctx.pad, ctx.compute, ctx.linear, ctx.has_bias = pad, compute, w.dim() == 2, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w3 = ctx.saved_tensors
        N, Cin, KS = w3.shape
        pad, compute = ctx.pad, ctx.compute
        dyc = _act(dy, compute)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # dx[s] = sum_k W_k^T dy[s + pad - k]: a conv of dy with taps flipped, W transposed
            if N == ops.cin_pad(N, compute):  # packed [Cin][KS][N] = w[n, c, KS-1-k]: one copy
                wtp = torch.empty(Cin, KS, N, dtype=ops.torch_dtype(compute), device=w3.device).copy_(
                    w3.flip(-1).permute(1, 2, 0))
            else:
                wtp = ops.pack_conv_weight(w3.flip(-1).transpose(0, 1), compute)
            dx = ops.conv1d(dyc, wtp, None, cin=N, ks=KS, pad=KS - 1 - pad,
                            compute=compute, epilogue=L.EPI_BIAS, out_dtype=L.FS2_F32)
        if ctx.needs_input_grad[1] and _wgrad_kernel_ok(compute, N, Cin, KS, xc):
            # fs2_conv_wgrad: no unfolded copy of x, the bias gradient from the same pass
            dw, db = ops.conv_wgrad(dyc, xc, KS, pad, want_db=ctx.has_bias and ctx.needs_input_grad[2])
            dw = dw.view(N, Cin) if ctx.linear else dw
            return dx, dw, db, None, None
        if ctx.needs_input_grad[1]:
            B, T, _ = xc.shape
            if KS == 1:
                xu = xc.reshape(B * T, Cin)
            else:
                xu = F.pad(xc, (0, 0, pad, KS - 1 - pad)).unfold(1, KS, 1).reshape(B * T, Cin * KS)
            dw = _wgrad(dyc.reshape(B * T, N), xu, B).view(N, Cin, KS)
            if ctx.linear:
                dw = dw.view(N, Cin)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.sum((0, 1))
        return dx, dw, db, None, None


def _wgrad_kernel_ok(compute, N, Cin, KS, xc):
    import os
    return (compute == L.FS2_BF16 and xc.is_cuda and xc.dim() == 3 and KS in (1, 3, 5, 9) and N % 8 == 0
            and Cin % 8 == 0 and xc.shape[-1] == Cin and os.environ.get("FS2_WGRAD_KERNEL", "1") != "0")


def _wgrad_chunks(rows, B, N, K):
    """Row chunks of the weight-gradient GEMM: a small dW (fc 256 x 256, FFN w_2 256 x 1024, VP)
    reduced over ~7k rows as one GEMM runs on a handful of workgroups; split into C batched GEMMs
    (C | B, f32 partials of <= 4 MiB in total) summed afterwards. FS2_WGRAD_SPLIT=0: one GEMM."""
    import os
    if os.environ.get("FS2_WGRAD_SPLIT", "1") == "0":
        return 1
    c = 1
    while c * 2 <= B and B % (c * 2) == 0 and (c * 2) * N * K * 4 <= (4 << 20) and rows // (c * 2) >= 128:
        c *= 2
    return c


def _wgrad(dy2, xu, B):
    """dW [N, K] = dy2^T xu over the rows (dy2 [rows, N], xu [rows, K], same dtype), f32 out."""
    rows, N = dy2.shape
    K = xu.shape[1]
    c = _wgrad_chunks(rows, B, N, K)
    if c == 1 or not dy2.is_cuda:
        return torch.matmul(dy2.t(), xu).float()
    r = rows // c
    out = torch.bmm(dy2.view(c, r, N).transpose(1, 2), xu.view(c, r, K), out_dtype=torch.float32) \
        if dy2.dtype != torch.float32 else torch.bmm(dy2.view(c, r, N).transpose(1, 2), xu.view(c, r, K))
    return out.sum(0)


def conv1d(x, conv, pad, compute):
    return Conv1dFn.apply(x, conv.weight, conv.bias, pad, compute)


def linear(x, lin, compute):
    if lin.out_features % 4:
        return F.linear(x, lin.weight, lin.bias)
    return Conv1dFn.apply(x, lin.weight, lin.bias, 0, compute)


class AttentionFn(torch.autograd.Function):
    """Key-padding-masked multi-head attention over the fused [B, T, 3*H*dk] projection
    (transformer/Modules.py:14-25 + SubLayers.py:42-52). A sequence of length 0 gives zeros and
    zero gradients (the reference gives NaN there)."""

    @staticmethod
    def forward(ctx, qkv, lens, n_head, d_k, temperature, compute):
        qa = _act(qkv, compute)
        out = ops.attention(qa, lens, n_head, d_k, temperature)
        ctx.save_for_backward(qa, out, lens)
        ctx.n_head, ctx.d_k, ctx.temperature = n_head, d_k, temperature
        return out.float()

    @staticmethod
    def backward(ctx, dout):
        # flash-style HIP backward (fs2_attention_bwd): no [B, H, T, T] tensor
        qa, out, lens = ctx.saved_tensors
        dqkv = ops.attention_bwd(qa, out, dout, lens, ctx.n_head, ctx.d_k, ctx.temperature)
        return dqkv, None, None, None, None, None


def _layer_norm(x, ln):
    return F.layer_norm(x, ln.normalized_shape, ln.weight, ln.bias, ln.eps)


def fft_block(blk, x, mask, lens, p_drop, training, compute):
    """transformer/Layers.py:21-30 with SubLayers.py:29-57 (MHA) and :85-93 (FFN)."""
    a, f = blk.slf_attn, blk.pos_ffn
    H, dk = a.n_head, a.d_k
    w = torch.cat([a.w_qs.weight, a.w_ks.weight, a.w_vs.weight], 0)
    bqkv = torch.cat([a.w_qs.bias, a.w_ks.bias, a.w_vs.bias], 0)
    qkv = Conv1dFn.apply(x, w, bqkv, 0, compute)
    att = AttentionFn.apply(qkv, lens, H, dk, float(np.power(dk, 0.5)), compute)
    o = F.dropout(linear(att, a.fc, compute), p_drop, training)
    h = _layer_norm(o + x, a.layer_norm).masked_fill(mask.unsqueeze(-1), 0)
    k1, k2 = f.w_1.kernel_size[0], f.w_2.kernel_size[0]
    y = torch.relu(conv1d(h, f.w_1, (k1 - 1) // 2, compute))
    y = F.dropout(conv1d(y, f.w_2, (k2 - 1) // 2, compute), p_drop, training)
    return _layer_norm(y + h, f.layer_norm).masked_fill(mask.unsqueeze(-1), 0)


# ---- the FFT block as one autograd node on the training kernels (train.hip) -------------------------
_SINK = [False]
_DEFER = [None]  # in a grad_sink: the fused nodes' split-partial gradient reductions, run after backward
_PACKED = [{}]  # conv module -> (forward image, input-gradient image) refreshed by this step's pack launch


class grad_sink:
    """Inside: FFTBlockFn writes its parameter gradients straight into the existing ``p.grad``
    tensors (accumulating: the trainer's flat buffer, zeroed at the start of the step) and hands
    autograd nothing for them — no per-parameter AccumulateGrad add. Only for the flat-gradient
    step (TrainStep(graph=True / flat_grads=True)); DDP needs its autograd hooks."""

    def __enter__(self):
        self.prev = _SINK[0]
        _SINK[0] = True
        _DEFER[0] = []

    def __exit__(self, *exc):
        _SINK[0] = self.prev
        q, _DEFER[0] = _DEFER[0], None
        if q:  # the deferred gradient finishes, one batched launch per 32 (fs2_reduce_batch_launch)
            ops.reduce_flush(q, q[0][1])


def fused_block_on(blk, compute):
    """FS2_TRAIN_FUSED=0 restores the per-op autograd form (Conv1dFn / AttentionFn / torch)."""
    import os
    if os.environ.get("FS2_TRAIN_FUSED", "1") == "0" or compute != L.FS2_BF16:
        return False
    f = blk.pos_ffn
    return (blk.slf_attn.w_qs.in_features == 256 and f.w_1.kernel_size[0] in (1, 3, 5, 9)
            and f.w_2.kernel_size[0] in (1, 3, 5, 9) and f.w_1.out_channels % 8 == 0)


def _block_params(blk):
    a, f = blk.slf_attn, blk.pos_ffn
    return [a.w_qs.weight, a.w_qs.bias, a.w_ks.weight, a.w_ks.bias, a.w_vs.weight, a.w_vs.bias, a.fc.weight, a.fc.bias,
            a.layer_norm.weight, a.layer_norm.bias, f.w_1.weight, f.w_1.bias, f.w_2.weight, f.w_2.bias,
            f.layer_norm.weight, f.layer_norm.bias]


def _packT(w):
    """Input-gradient weight of a conv [N, Cin, KS] (Linear [N, Cin]): the conv of dy with taps
    flipped and W transposed, packed [Cin][KS][N] bf16."""
    w3 = w if w.dim() == 3 else w.unsqueeze(-1)
    return torch.empty(w3.shape[1], w3.shape[2], w3.shape[0], dtype=torch.bfloat16, device=w.device).copy_(
        w3.detach().flip(-1).permute(1, 2, 0))


class _TrainPack:
    """Every FFT block's MFMA weight images (forward and input-gradient forms, Q|K|V fused, Q|K|V
    bias concatenated) in persistent buffers, refreshed by ONE fs2_pack_train launch per forward
    (captured with the step). Built outside graph capture; rebuilt if a parameter moved."""

    def __init__(self, blocks, dev, extra_convs=()):
        from . import _lib as LL
        self.key = _pack_key(blocks, extra_convs)
        bf = dict(dtype=torch.bfloat16, device=dev)
        descs, self.per_block = [], []

        def add(src, fwd=None, tr=None, N=0, C=1, KS=1, n_off=0, N_tot=0, f32=0):
            d = LL.PackDesc()
            d.src = src.data_ptr()
            d.fwd = fwd.data_ptr() if fwd is not None else None
            d.tr = tr.data_ptr() if tr is not None else None
            d.N, d.C, d.KS, d.n_off, d.N_tot, d.f32_copy = N, C, KS, n_off, N_tot or N, f32
            descs.append(d)

        def conv_images(w):
            """forward [N][KS][cin_pad(C)] + input-gradient [C][KS][cin_pad(N)] images of a conv,
            zero-initialised (the padding channels stay zero)."""
            N, C, KS = w.shape
            cp, npd = ops.cin_pad(C, L.FS2_BF16), ops.cin_pad(N, L.FS2_BF16)
            fw, tr = torch.zeros(N, KS, cp, **bf), torch.zeros(C, KS, npd, **bf)
            add(w, fw, tr, N, C, KS, 0, npd)
            descs[-1].C_tot = cp
            return fw, tr

        self.extra = {}
        for conv in extra_convs:
            self.extra[conv] = conv_images(conv.weight)
        for blk in blocks:
            a, f = blk.slf_attn, blk.pos_ffn
            k1, k2, F_ = f.w_1.kernel_size[0], f.w_2.kernel_size[0], f.w_1.out_channels
            D = a.w_qs.in_features
            P = dict(qkv=torch.empty(3 * D, 1, D, **bf), qkvT=torch.empty(D, 1, 3 * D, **bf),
                     bqkv=torch.empty(3 * D, dtype=torch.float32, device=dev),
                     fc=torch.empty(D, 1, D, **bf), fcT=torch.empty(D, 1, D, **bf),
                     w1=torch.empty(F_, k1, D, **bf), w1T=torch.empty(D, k1, F_, **bf),
                     w2=torch.empty(D, k2, F_, **bf), w2T=torch.empty(F_, k2, D, **bf))
            for j, lin in enumerate((a.w_qs, a.w_ks, a.w_vs)):
                add(lin.weight, P["qkv"], P["qkvT"], D, D, 1, j * D, 3 * D)
                add(lin.bias, P["bqkv"], None, D, 1, 1, j * D, 3 * D, f32=1)
            add(a.fc.weight, P["fc"], P["fcT"], D, D, 1, 0, D)
            add(f.w_1.weight, P["w1"], P["w1T"], F_, D, k1, 0, F_)
            add(f.w_2.weight, P["w2"], P["w2T"], D, F_, k2, 0, D)
            self.per_block.append(P)
        n = len(descs)
        arr = (LL.PackDesc * n)(*descs)
        blocks_out = ctypes.c_int(0)
        L.check(LL.load().fs2_pack_train_plan(arr, n, ctypes.byref(blocks_out)), "fs2_pack_train_plan")
        raw = bytes(memoryview(arr).cast("B"))
        self.dev_descs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
        self.n, self.grid = n, blocks_out.value

    def run(self, stream_of):
        from . import _lib as LL
        L.check(LL.load().fs2_pack_train(ctypes.c_void_p(self.dev_descs.data_ptr()), self.n, self.grid,
                                         ops._stream(stream_of)), "fs2_pack_train")


def _pack_key(blocks, extra_convs=()):
    return tuple(p.data_ptr() for b in blocks for p in _block_params(b)) + tuple(c.weight.data_ptr()
                                                                                 for c in extra_convs)


def _train_pack(model, blocks, dev, extra_convs=()):
    """The model's _TrainPack (None while capturing before one exists: per-block packing then)."""
    tp = getattr(model, "_fs2_train_pack", None)
    if tp is not None and tp.key == _pack_key(blocks, extra_convs):
        return tp
    if torch.cuda.is_current_stream_capturing():
        return None
    tp = model._fs2_train_pack = _TrainPack(blocks, dev, extra_convs)
    return tp


def _extra_convs(model, compute):
    """VariancePredictor and PostNet convs whose images join the step's pack launch."""
    convs = []
    va = model.variance_adaptor
    for vp in (va.duration_predictor, va.pitch_predictor, va.energy_predictor):
        if _vp_fused_ok(vp, compute):
            convs += [vp.conv_layer.conv1d_1.conv, vp.conv_layer.conv1d_2.conv]
    if _postnet_fused_ok(model.postnet, compute):
        convs += [seq[0].conv for seq in model.postnet.convolutions]
    return convs


class FFTBlockFn(torch.autograd.Function):
    """transformer/Layers.py:21-30 (MHA SubLayers.py:29-57, FFN :85-93) in train mode as one node:
    forward Q|K|V conv (bf16 out) -> fs2_attention -> fc conv -> fs2_res_ln_fwd (dropout +
    residual + LN + mask) -> w_1 conv (relu, bf16 out) -> w_2 conv -> fs2_res_ln_fwd; backward
    fs2_res_ln_bwd (+ the conv bias gradient) -> w_2 input gradient with the relu mask in its
    epilogue (FS2_EPI_RELU_GRAD) -> w_1 input gradient + residual gradient in one epilogue ->
    fs2_res_ln_bwd -> fc input gradient -> fs2_attention_bwd -> Q|K|V input gradient + residual;
    every weight gradient on fs2_conv_wgrad (no unfolded copies). Returns (y f32, y bf16): the
    bf16 copy is the next block's MFMA input (not differentiable)."""

    @staticmethod
    def forward(ctx, x, x_bf, lens, seed, meta, *params):
        blk, p_drop, salt, pk = meta
        (wq, bq, wk, bk, wv, bv, wfc, bfc, g1, be1, w1, b1, w2, b2, g2, be2) = params
        a, f = blk.slf_attn, blk.pos_ffn
        H, dk = a.n_head, a.d_k
        temp = float(np.power(dk, 0.5))
        k1, k2 = f.w_1.kernel_size[0], f.w_2.kernel_size[0]
        BF = L.FS2_BF16
        xb = x_bf if x_bf is not None else x.to(torch.bfloat16)
        if pk is None:  # per-block packing (no persistent pack yet)
            wqkv = torch.cat([wq, wk, wv], 0).detach()
            pk = dict(qkv=ops.pack_conv_weight(wqkv, BF), bqkv=torch.cat([bq, bk, bv]).detach(),
                      fc=ops.pack_conv_weight(wfc, BF), w1=ops.pack_conv_weight(w1, BF),
                      w2=ops.pack_conv_weight(w2, BF), qkvT=_packT(wqkv), fcT=_packT(wfc), w1T=_packT(w1),
                      w2T=_packT(w2))
        qkv = ops.conv1d(xb, pk["qkv"], pk["bqkv"], cin=256, ks=1, pad=0, compute=BF, epilogue=L.EPI_BIAS,
                         out_dtype=BF)
        B_, T_ = x.shape[0], x.shape[1]
        lse = torch.empty(B_ * T_, H, device=x.device, dtype=torch.float32)
        att = ops.attention(qkv, lens, H, dk, temp, lse=lse)
        a1 = ops.conv1d(att, pk["fc"], bfc.detach(), cin=256, ks=1, pad=0, compute=BF, epilogue=L.EPI_BIAS,
                        out_dtype=L.FS2_F32)
        h, hb, xh1, rs1 = ops.res_ln_fwd(a1, x.contiguous(), g1.detach(), be1.detach(), a.layer_norm.eps, lens,
                                         p_drop, seed, salt)
        u = ops.conv1d(hb, pk["w1"], b1.detach(), cin=256, ks=k1, pad=(k1 - 1) // 2, compute=BF,
                       epilogue=L.EPI_BIAS_RELU, out_dtype=BF)
        a2 = ops.conv1d(u, pk["w2"], b2.detach(), cin=w2.shape[1], ks=k2, pad=(k2 - 1) // 2, compute=BF,
                        epilogue=L.EPI_BIAS, out_dtype=L.FS2_F32)
        y, yb, xh2, rs2 = ops.res_ln_fwd(a2, h, g2.detach(), be2.detach(), f.layer_norm.eps, lens, p_drop, seed,
                                         salt + 1)
        ctx.save_for_backward(xb, qkv, att, hb, u, xh1, rs1, xh2, rs2, lens, lse, *params)
        ctx.packT = (pk["qkvT"], pk["fcT"], pk["w1T"], pk["w2T"])
        ctx.meta = (H, dk, temp, k1, k2, p_drop, salt, seed)
        ctx.mark_non_differentiable(yb)
        # the bf16 copy never gets a gradient: without this autograd zero-fills one of its size
        # per block per step (a FillFunc launch each)
        ctx.set_materialize_grads(False)
        return y, yb

    @staticmethod
    def backward(ctx, dy, _dyb):
        xb, qkv, att, hb, u, xh1, rs1, xh2, rs2, lens, lse, *params = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros(xb.shape, device=xb.device, dtype=torch.float32)
        (wq, bq, wk, bk, wv, bv, wfc, bfc, g1, be1, w1, b1, w2, b2, g2, be2) = params
        H, dk, temp, k1, k2, p_drop, salt, seed = ctx.meta
        wqkvT, wfcT, w1T, w2T = ctx.packT
        BF = L.FS2_BF16
        sink = _SINK[0] and all(p.grad is not None for p in params)
        acc = sink
        G = (lambda p: p.grad) if sink else (lambda p: None)
        pad1, pad2 = (k1 - 1) // 2, (k2 - 1) // 2
        F_ = w1.shape[0]
        # FFN: LN backward, w_2 gradients, relu-masked input gradient, w_1 gradients, + residual
        q = _DEFER[0] if sink else None
        dres2, da2, dg2, dbe2, db2 = ops.res_ln_bwd(dy, xh2, rs2, g2.detach(), lens, p_drop, seed, salt + 1,
                                                    dgamma=G(g2), dbeta=G(be2), dbias=G(b2), accumulate=acc, defer=q)
        dw2, _ = ops.conv_wgrad(da2, u, k2, pad2, dw=G(w2), accumulate=acc, defer=q)
        du = ops.conv1d(da2, w2T, None, cin=256, ks=k2, pad=k2 - 1 - pad2, compute=BF, epilogue=L.EPI_RELU_GRAD,
                        out_dtype=BF, residual=u)
        dw1, db1 = ops.conv_wgrad(du, hb, k1, pad1, dw=G(w1), db=G(b1), want_db=True, accumulate=acc, defer=q)
        dh = ops.conv1d(du, w1T, None, cin=F_, ks=k1, pad=k1 - 1 - pad1, compute=BF, epilogue=L.EPI_BIAS_RES,
                        out_dtype=L.FS2_F32, residual=dres2)
        # attention sub-layer
        dres1, da1, dg1, dbe1, dbfc = ops.res_ln_bwd(dh, xh1, rs1, g1.detach(), lens, p_drop, seed, salt,
                                                     dgamma=G(g1), dbeta=G(be1), dbias=G(bfc), accumulate=acc, defer=q)
        dwfc, _ = ops.conv_wgrad(da1, att, 1, 0, dw=G(wfc), accumulate=acc, defer=q)
        datt = ops.conv1d(da1, wfcT, None, cin=256, ks=1, pad=0, compute=BF, epilogue=L.EPI_BIAS,
                          out_dtype=L.FS2_F32)
        dqkv = ops.attention_bwd(qkv, att, datt, lens, H, dk, temp, lse=lse)
        if sink:
            ops.conv_wgrad(dqkv, xb, 1, 0, parts=([wq.grad, wk.grad, wv.grad], [bq.grad, bk.grad, bv.grad]),
                           accumulate=True, defer=q)
            gq = [None] * 6
        else:
            dws = [torch.empty_like(w) for w in (wq, wk, wv)]
            dbs = [torch.empty_like(b) for b in (bq, bk, bv)]
            ops.conv_wgrad(dqkv, xb, 1, 0, parts=(dws, dbs))
            gq = [dws[0], dbs[0], dws[1], dbs[1], dws[2], dbs[2]]
        dx = ops.conv1d(dqkv, wqkvT, None, cin=3 * H * dk, ks=1, pad=0, compute=BF,
                        epilogue=L.EPI_BIAS_RES, out_dtype=L.FS2_F32, residual=dres1)
        if sink:
            grads = gq + [None] * 10
        else:
            grads = gq + [dwfc.view_as(wfc), dbfc, dg1, dbe1, dw1.view_as(w1), db1, dw2.view_as(w2), db2, dg2, dbe2]
        return (dx, None, None, None, None, *grads)


class EmbeddingFn(torch.autograd.Function):
    """nn.Embedding with its weight gradient on fs2_embedding_bwd (deterministic, no atomics;
    padding_idx honoured); gradient sink as FFTBlockFn."""

    @staticmethod
    def forward(ctx, idx, weight, padding_idx):
        ctx.save_for_backward(idx, weight)
        ctx.padding_idx = padding_idx
        return F.embedding(idx, weight)

    @staticmethod
    def backward(ctx, dy):
        idx, weight = ctx.saved_tensors
        if _SINK[0] and weight.grad is not None:
            ops.embedding_bwd(idx, dy, weight.shape[0], ctx.padding_idx, out=weight.grad, accumulate=True)
            return None, None, None
        return None, ops.embedding_bwd(idx, dy, weight.shape[0], ctx.padding_idx), None


def _embed(emb, idx, fused):
    if not fused:
        return emb(idx)
    return EmbeddingFn.apply(idx, emb.weight, emb.padding_idx)


class CondFn(torch.autograd.Function):
    """The conditioning of fastspeech2.py:101-110 in training: x + speaker_emb(speakers) +
    emotion_linear(cat(emotion_emb, arousal_emb, valence_emb)) broadcast over the positions.
    Forward: fs2_cond_vectors (one launch) and the two adds in the reference's order; backward:
    fs2_cond_bwd (two launches, deterministic) instead of the autograd of four lookups, a cat, the
    Linear + ReLU and the broadcast adds (~20 launches); gradient sink as FFTBlockFn."""

    @staticmethod
    def forward(ctx, x, speakers, emotions, arousals, valences, spk_w, emo_w, aro_w, val_w, lin_w, lin_b):
        D = x.shape[-1]
        spk, emo = ops.cond_vectors(speakers, spk_w, emotions, arousals, valences, emo_w, aro_w, val_w, lin_w, lin_b,
                                    D)
        y = x + spk.unsqueeze(1) if spk is not None else x.clone()
        if emo is not None:
            y.add_(emo.unsqueeze(1))
        ctx.save_for_backward(speakers, emotions, arousals, valences, spk_w, emo_w, aro_w, val_w, lin_w, lin_b, emo)
        return y

    @staticmethod
    def backward(ctx, dy):
        speakers, emotions, arousals, valences, spk_w, emo_w, aro_w, val_w, lin_w, lin_b, emo = ctx.saved_tensors
        params = (spk_w, emo_w, aro_w, val_w, lin_w, lin_b)  # None where the model has no such table
        present = [p for p in params if p is not None]
        sink = _SINK[0] and all(p.grad is not None for p in present)
        if sink:
            grads = [None if p is None else p.grad for p in params]
        else:
            grads = [None if p is None else torch.zeros_like(p) for p in params]
        ops.cond_bwd(dy.float(), speakers, spk_w, emotions, arousals, valences, emo_w, aro_w, val_w, lin_w, emo,
                     *grads)
        if sink:
            grads = [None] * 6
        return (dy, None, None, None, None, *grads)


def cond_fused_on(model, x):
    """CondFn applies: f32 positions, fs2_cond_bwd's limits (B <= 64 and its LDS bound), at least one
    conditioning table; FS2_TRAIN_COND=0 keeps the per-op autograd form."""
    if os.environ.get("FS2_TRAIN_COND", "1") == "0" or x.dtype != torch.float32 or not x.is_cuda:
        return False
    if model.speaker_emb is None and model.emotion_emb is None:
        return False
    B, D = x.shape[0], x.shape[-1]
    emo = model.emotion_emb is not None
    return B <= 64 and (not emo or (B * D + 16 * D + 32 * B) * 4 + 24 * B <= 65536)


def _packT_any(w):
    """Input-gradient weight of a conv whose output width may need channel padding as the
    transposed conv's input (PostNet's 80 mel channels)."""
    N = w.shape[0]
    if N == ops.cin_pad(N, L.FS2_BF16):
        return _packT(w)
    return ops.pack_conv_weight(w.detach().flip(-1).transpose(0, 1), L.FS2_BF16)


class PostNetFn(torch.autograd.Function):
    """The PostNet (transformer/Layers.py:92-137) in train mode + the residual (fastspeech2.py:136)
    as one node: per layer fs2_conv1d (f32 out) -> fs2_bn_train_fwd (batch-statistic BatchNorm with
    running-stat update, tanh on layers 0..3, dropout 0.5, bf16 copy for the next conv; the last
    adds mel); backward per layer fs2_bn_train_bwd -> fs2_conv_wgrad (+ bias) -> input-gradient
    conv (the first one adds the residual's gradient in its epilogue)."""

    @staticmethod
    def forward(ctx, mel, meta, *params):
        postnet, p_drop, seed, salt = meta
        convs = postnet.convolutions
        n = len(convs)
        BF = L.FS2_BF16
        x_bf = mel.detach().to(torch.bfloat16)
        saved = []
        out = None
        for i, seq in enumerate(convs):
            bn = seq[1]
            w, b, g, be = params[4 * i:4 * i + 4]
            N, Cin, KS = w.shape
            pad = (KS - 1) // 2
            imgs = _PACKED[0].get(seq[0].conv)
            wf, wT = imgs if imgs is not None else (ops.pack_conv_weight(w, BF), _packT_any(w))
            z = ops.conv1d(x_bf, wf, b.detach(), cin=Cin, ks=KS, pad=pad, compute=BF, epilogue=L.EPI_BIAS,
                           out_dtype=L.FS2_F32)
            last = i == n - 1
            yb, yf, mean, rstd = ops.bn_train_fwd(z, g.detach(), be.detach(), bn.eps, bn.momentum, bn.running_mean,
                                                  bn.running_var, use_tanh=not last, p_drop=p_drop, seed=seed,
                                                  salt=salt + i, residual=mel.detach() if last else None,
                                                  want_bf16=not last, want_f32=last)
            saved.append((x_bf, z, mean, rstd, wT, pad, KS))
            x_bf, out = yb, yf
        # BatchNorm's step counters, all layers in one multi-tensor launch (one add kernel each before)
        nbt = [seq[1].num_batches_tracked for seq in convs if seq[1].num_batches_tracked is not None]
        if nbt:
            torch._foreach_add_(nbt, 1)
        ctx.saved = saved
        ctx.meta = (p_drop, seed, salt)
        ctx.save_for_backward(*params)
        return out

    @staticmethod
    def backward(ctx, dout):
        params = ctx.saved_tensors
        p_drop, seed, salt = ctx.meta
        n = len(ctx.saved)
        dout = dout.contiguous()
        sink = _SINK[0] and all(t.grad is not None for t in params)
        grads = [None] * len(params)
        dy = dout
        dmel = None
        for i in reversed(range(n)):
            x_bf, z, mean, rstd, wT, pad, KS = ctx.saved[i]
            w, b, g, be = params[4 * i:4 * i + 4]
            N = w.shape[0]
            last = i == n - 1
            dz, dg, dbe = ops.bn_train_bwd(dy, z, g.detach(), be.detach(), mean, rstd, use_tanh=not last,
                                           p_drop=p_drop, seed=seed, salt=salt + i,
                                           dgamma=g.grad if sink else None, dbeta=be.grad if sink else None,
                                           accumulate=sink)
            dw, db = ops.conv_wgrad(dz, x_bf, KS, pad, dw=w.grad if sink else None, db=b.grad if sink else None,
                                    want_db=True, accumulate=sink, defer=_DEFER[0] if sink else None)
            if not sink:
                grads[4 * i:4 * i + 4] = [dw, db, dg, dbe]
            if i > 0:
                dy = ops.conv1d(dz, wT, None, cin=N, ks=KS, pad=KS - 1 - pad, compute=L.FS2_BF16,
                                epilogue=L.EPI_BIAS, out_dtype=L.FS2_F32)
            else:
                dmel = ops.conv1d(dz, wT, None, cin=N, ks=KS, pad=KS - 1 - pad, compute=L.FS2_BF16,
                                  epilogue=L.EPI_BIAS_RES, out_dtype=L.FS2_F32, residual=dout)
        return (dmel, None, *grads)


def _postnet_fused_ok(postnet, compute):
    if os.environ.get("FS2_TRAIN_FUSED", "1") == "0" or compute != L.FS2_BF16:
        return False
    for seq in postnet.convolutions:
        conv, bn = seq[0].conv, seq[1]
        if conv.kernel_size[0] not in (1, 3, 5, 9) or conv.out_channels % 8 or conv.in_channels % 8 or \
                conv.out_channels > 1024 or bn.momentum is None or not bn.track_running_stats:
            return False
    return True


def _postnet_params(postnet):
    ps = []
    for seq in postnet.convolutions:
        conv, bn = seq[0].conv, seq[1]
        ps += [conv.weight, conv.bias, bn.weight, bn.bias]
    return ps


def fft_block_fused(blk, x, x_bf, lens, seed, salt, p_drop, packed=None):
    y, yb = FFTBlockFn.apply(x, x_bf, lens, seed, (blk, float(p_drop), int(salt), packed), *_block_params(blk))
    return y, yb


def _train_seed(model, dev):
    """The dropout seed of the fused blocks: one device int64 advanced once per forward (inside a
    captured step too, so every replay draws new masks)."""
    s = getattr(model, "_fs2_train_seed", None)
    if s is None or s.device != dev:
        s = torch.tensor([int(torch.randint(0, 2 ** 62, (1,)).item())], dtype=torch.int64, device=dev)
        model._fs2_train_seed = s
    return s


class VPLayerFn(torch.autograd.Function):
    """One VariancePredictor layer in train mode (model/modules.py:218-235): Conv (fs2_conv1d, f32
    out) -> fs2_relu_ln_fwd (relu + LayerNorm + dropout, bf16 copy for the next conv); backward
    fs2_relu_ln_bwd (+ the conv's bias gradient) -> input gradient conv -> fs2_conv_wgrad."""

    @staticmethod
    def forward(ctx, x, x_bf, meta, w, b, g, be):
        pad, p_drop, seed, salt, eps = meta[:5]
        N, Cin, KS = w.shape
        BF = L.FS2_BF16
        xb = x_bf if x_bf is not None else x.to(torch.bfloat16)
        wf, wT = meta[5] if len(meta) > 5 and meta[5] is not None else (ops.pack_conv_weight(w, BF), _packT_any(w))
        a = ops.conv1d(xb, wf, b.detach(), cin=Cin, ks=KS, pad=pad, compute=BF, epilogue=L.EPI_BIAS,
                       out_dtype=L.FS2_F32)
        y, yb, xh, rs = ops.relu_ln_fwd(a, g.detach(), be.detach(), eps, p_drop, seed, salt)
        ctx.save_for_backward(xb, a, xh, rs, w, b, g, be)
        ctx.meta = meta
        ctx.wT = wT
        ctx.mark_non_differentiable(yb)
        ctx.set_materialize_grads(False)  # (as FFTBlockFn: no zero-filled gradient for yb)
        return y, yb

    @staticmethod
    def backward(ctx, dy, _dyb):
        xb, a, xh, rs, w, b, g, be = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros(xh.shape, device=xh.device, dtype=torch.float32)
        pad, p_drop, seed, salt, eps = ctx.meta[:5]
        N, Cin, KS = w.shape
        sink = _SINK[0] and all(t.grad is not None for t in (w, b, g, be))
        G = (lambda t: t.grad) if sink else (lambda t: None)
        q = _DEFER[0] if sink else None
        da, dg, dbe, db = ops.relu_ln_bwd(dy, a, xh, rs, g.detach(), p_drop, seed, salt, dgamma=G(g), dbeta=G(be),
                                          dbias=G(b), accumulate=sink, defer=q)
        dw, _ = ops.conv_wgrad(da, xb, KS, pad, dw=G(w), accumulate=sink, defer=q)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = ops.conv1d(da, ctx.wT, None, cin=N, ks=KS, pad=KS - 1 - pad, compute=L.FS2_BF16,
                            epilogue=L.EPI_BIAS, out_dtype=L.FS2_F32)
        if sink:
            return dx, None, None, None, None, None, None
        return dx, None, None, dw, db, dg, dbe


class VPHeadLayerFn(torch.autograd.Function):
    """The VariancePredictor's second layer WITH its head (model/modules.py:225-250, train mode):
    Conv (fs2_conv1d, f32 out) -> fs2_relu_ln_head_fwd (relu + LayerNorm + dropout + Linear(256->1) +
    masked_fill in one launch: no y tensor, no hipBLASLt GEMV and elementwise launches); backward
    fs2_relu_ln_head_bwd (the LayerNorm and head gradients straight from the predictor output's
    gradient) -> input gradient conv -> fs2_conv_wgrad. FS2_VP_HEAD_FUSED=0: VPLayerFn + F.linear."""

    @staticmethod
    def forward(ctx, x, x_bf, mask, meta, w, b, g, be, hw, hb):
        pad, p_drop, seed, salt, eps = meta[:5]
        N, Cin, KS = w.shape
        BF = L.FS2_BF16
        xb = x_bf if x_bf is not None else x.to(torch.bfloat16)
        wf, wT = meta[5] if len(meta) > 5 and meta[5] is not None else (ops.pack_conv_weight(w, BF), _packT_any(w))
        a = ops.conv1d(xb, wf, b.detach(), cin=Cin, ks=KS, pad=pad, compute=BF, epilogue=L.EPI_BIAS,
                       out_dtype=L.FS2_F32)
        out, xh, rs = ops.relu_ln_head_fwd(a, g.detach(), be.detach(), eps, hw.detach().reshape(-1), hb.detach(), mask,
                                           p_drop, seed, salt)
        ctx.save_for_backward(xb, a, xh, rs, w, b, g, be, hw, hb, mask)
        ctx.meta = meta
        ctx.wT = wT
        return out

    @staticmethod
    def backward(ctx, dout):
        xb, a, xh, rs, w, b, g, be, hw, hb, mask = ctx.saved_tensors
        pad, p_drop, seed, salt, eps = ctx.meta[:5]
        N, Cin, KS = w.shape
        sink = _SINK[0] and all(t.grad is not None for t in (w, b, g, be, hw, hb))
        G = (lambda t: t.grad) if sink else (lambda t: None)
        q = _DEFER[0] if sink else None
        da, dg, dbe, db, dhw, dhb = ops.relu_ln_head_bwd(
            dout.float(), mask, hw.detach().reshape(-1), be.detach(), a, xh, rs, g.detach(), p_drop, seed, salt,
            dgamma=G(g), dbeta=G(be), dbias=G(b), dhw=None if G(hw) is None else G(hw).view(-1), dhb=G(hb),
            accumulate=sink, defer=q)
        dw, _ = ops.conv_wgrad(da, xb, KS, pad, dw=G(w), accumulate=sink, defer=q)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = ops.conv1d(da, ctx.wT, None, cin=N, ks=KS, pad=KS - 1 - pad, compute=L.FS2_BF16,
                            epilogue=L.EPI_BIAS, out_dtype=L.FS2_F32)
        if sink:
            return dx, None, None, None, None, None, None, None, None, None
        return dx, None, None, None, dw, db, dg, dbe, dhw.view_as(hw), dhb.view_as(hb)


def _vp_fused(vp, x, mask, training, seed, salt):
    cl = vp.conv_layer
    c1, c2 = cl.conv1d_1.conv, cl.conv1d_2.conv
    k = c1.kernel_size[0]
    p1 = cl.dropout_1.p if training else 0.0
    p2 = cl.dropout_2.p if training else 0.0
    pk = _PACKED[0]
    h, hb = VPLayerFn.apply(x.contiguous(), None, ((k - 1) // 2, p1, seed, salt, cl.layer_norm_1.eps, pk.get(c1)),
                            c1.weight, c1.bias, cl.layer_norm_1.weight, cl.layer_norm_1.bias)
    lin = vp.linear_layer
    if os.environ.get("FS2_VP_HEAD_FUSED", "1") != "0" and lin.in_features == 256 and lin.out_features == 1 \
            and lin.bias is not None and mask is not None and mask.shape == x.shape[:-1]:
        return VPHeadLayerFn.apply(h, hb, mask, (1, p2, seed, salt + 1, cl.layer_norm_2.eps, pk.get(c2)), c2.weight,
                                   c2.bias, cl.layer_norm_2.weight, cl.layer_norm_2.bias, lin.weight, lin.bias)
    h, _ = VPLayerFn.apply(h, hb, (1, p2, seed, salt + 1, cl.layer_norm_2.eps, pk.get(c2)), c2.weight, c2.bias,
                           cl.layer_norm_2.weight, cl.layer_norm_2.bias)
    out = F.linear(h, lin.weight, lin.bias).squeeze(-1)
    return out.masked_fill(mask, 0.0)


def _vp_fused_ok(vp, compute):
    cl = vp.conv_layer
    c1, c2 = cl.conv1d_1.conv, cl.conv1d_2.conv
    return (os.environ.get("FS2_TRAIN_FUSED", "1") != "0" and compute == L.FS2_BF16 and c1.out_channels == 256
            and c2.out_channels == 256 and c1.kernel_size[0] in (1, 3, 5, 9) and c2.kernel_size[0] in (1, 3, 5, 9)
            and c1.in_channels % 8 == 0)


def variance_predictor(vp, x, mask, training, compute, seed=None, salt=0):
    """model/modules.py:209-250 (conv1d_2 padding hard-coded to 1, :230)."""
    if seed is not None and _vp_fused_ok(vp, compute):
        return _vp_fused(vp, x, mask, training, seed, salt)
    cl = vp.conv_layer
    k = cl.conv1d_1.conv.kernel_size[0]
    h = torch.relu(conv1d(x, cl.conv1d_1.conv, (k - 1) // 2, compute))
    h = F.dropout(_layer_norm(h, cl.layer_norm_1), cl.dropout_1.p, training)
    h = torch.relu(conv1d(h, cl.conv1d_2.conv, 1, compute))
    h = F.dropout(_layer_norm(h, cl.layer_norm_2), cl.dropout_2.p, training)
    out = F.linear(h, vp.linear_layer.weight, vp.linear_layer.bias).squeeze(-1)
    return out.masked_fill(mask, 0.0)


class VarianceEmbedFn(torch.autograd.Function):
    """x + Embedding(bucketize(value, bins)) (model/modules.py:80-100, x + emb :117-126) as one
    fs2_variance_embed_ex launch; backward: dx = dy, the table's gradient on fs2_embedding_bwd over
    the saved bucket indices (deterministic; gradient sink as EmbeddingFn). value carries no
    gradient (bucketize is piecewise constant)."""

    @staticmethod
    def forward(ctx, x, value, bins, weight):
        out, idx = ops.variance_embed_ex(x.detach(), value, bins, weight.detach())
        ctx.save_for_backward(idx, weight)
        return out

    @staticmethod
    def backward(ctx, dy):
        idx, weight = ctx.saved_tensors
        gw = None
        if ctx.needs_input_grad[3]:
            if _SINK[0] and weight.grad is not None:
                ops.embedding_bwd(idx, dy, weight.shape[0], None, out=weight.grad, accumulate=True)
            else:
                gw = ops.embedding_bwd(idx, dy, weight.shape[0], None)
        return dy, None, None, gw


def _variance_embed(va, kind, x, target, mask, control, training, compute, seed=None, salt=0):
    """model/modules.py:80-100,117-126 (energy is scaled by p_control in the reference): the
    prediction, and x + the embedding of its bucket (fs2_variance_embed_ex, VarianceEmbedFn)."""
    pred = variance_predictor(getattr(va, f"{kind}_predictor"), x, mask, training, compute, seed, salt)
    bins = getattr(va, f"{kind}_bins")
    table = getattr(va, f"{kind}_embedding")
    if target is None:
        pred = pred * control
    value = target if target is not None else pred
    return pred, VarianceEmbedFn.apply(x.contiguous(), value.detach(), bins, table.weight)


class LengthRegulatorFn(torch.autograd.Function):
    """LengthRegulator gather (model/modules.py:161-194 + pad, utils/tools.py:360-378) over T
    output frames, optionally + the decoder's position encoding (transformer/Models.py:158-160)
    in the same pass (fs2_lr_expand); backward: fs2_lr_backward, a deterministic per-phoneme
    segmented sum over its frames (no scatter-add atomics)."""

    @staticmethod
    def forward(ctx, x, cum, mel_len, T, pe):
        out = ops.lr_expand(x.detach().float(), cum, mel_len, T, pe=pe, out_dtype=L.FS2_F32)
        ctx.save_for_backward(cum)
        ctx.n, ctx.dtype = x.shape[1], x.dtype
        return out

    @staticmethod
    def backward(ctx, dy):
        (cum,) = ctx.saved_tensors
        return ops.lr_backward(dy, cum, ctx.n).to(ctx.dtype), None, None, None, None


def _length_regulate(x, dur, max_len, crop=None, pe=None):
    """LengthRegulator (model/modules.py:161-194) on HIP: the duration scan, then the gather over
    T = max_len (or max(mel_len): one host read) frames, cropped to ``crop`` frames (the training
    decoder's max_seq_len, transformer/Models.py:154-162) and with ``pe`` [>= T, D] added when
    given. Returns (x [B, T', D] f32, mel_len, T) with T the uncropped length."""
    cum, mel_len, _ = ops.lr_durations(dur if dur.dtype in (torch.int64, torch.float32) else dur.to(torch.int64))
    T = int(max_len) if max_len else int(mel_len.max().item())
    Tc = T if crop is None else min(T, int(crop))
    return LengthRegulatorFn.apply(x.contiguous(), cum, mel_len, Tc, pe), mel_len, T


def _mask(lengths, width):
    return ops.length_mask(lengths, width)


def _device_ok(dev):
    return dev.type == "cuda"


def train_forward(model, speakers, emotions, arousals, valences, texts, src_lens, max_src_len, mels=None,
                  mel_lens=None, max_mel_len=None, p_targets=None, e_targets=None, d_targets=None, p_control=1.0,
                  e_control=1.0, d_control=1.0):
    dev = texts.device
    if not _device_ok(dev):
        raise RuntimeError("fs2amd: training runs on the HIP kernels only (ROCm device tensors; no CPU fallback)")
    compute = L.FS2_BF16 if model.precision == "bf16" else L.FS2_F32
    training = model.training and model.train_dropout
    tr = model.model_config["transformer"]
    enc, dec, va = model.encoder, model.decoder, model.variance_adaptor
    src_lens = src_lens.to(dev)
    B, Lx = texts.shape
    src_masks = _mask(src_lens, max_src_len)
    if mel_lens is not None:  # get_mask_from_lengths falls back to max(lengths) (utils/tools.py:153-155)
        mel_masks = _mask(mel_lens, max_mel_len if max_mel_len is not None else int(mel_lens.max().item()))
    else:
        mel_masks = None
    lens_src = src_lens.to(torch.int64).contiguous()

    # encoder (transformer/Models.py:73-100; training never recomputes the PE table)
    fused = all(fused_block_on(b, compute) for b in list(enc.layer_stack) + list(dec.layer_stack))
    _PACKED[0] = {}
    packs = [None] * (len(enc.layer_stack) + len(dec.layer_stack))
    if fused:
        seed = _train_seed(model, dev)
        if training:
            seed.add_(1)
        if os.environ.get("FS2_TRAIN_PACK", "1") != "0":
            tp = _train_pack(model, list(enc.layer_stack) + list(dec.layer_stack), dev, _extra_convs(model, compute))
            if tp is not None:
                tp.run(texts)
                packs = tp.per_block
                _PACKED[0] = tp.extra
    x = _embed(enc.src_word_emb, texts, fused) + enc.position_enc[:, :Lx, :]
    xb = None
    for i, blk in enumerate(enc.layer_stack):
        if fused:
            x, xb = fft_block_fused(blk, x, xb, lens_src, seed, 2 * i, tr["encoder_dropout"] if training else 0.0,
                                    packs[i])
        else:
            x = fft_block(blk, x, src_masks, lens_src, tr["encoder_dropout"], training, compute)
    if fused and cond_fused_on(model, x):
        emo_on = model.emotion_emb is not None
        spk_w = model.speaker_emb.weight if model.speaker_emb is not None else None
        x = CondFn.apply(x, speakers if spk_w is not None else None, emotions if emo_on else None,
                         arousals if emo_on else None, valences if emo_on else None, spk_w,
                         *((model.emotion_emb.weight, model.arousal_emb.weight, model.valence_emb.weight,
                            model.emotion_linear[0].weight, model.emotion_linear[0].bias) if emo_on else (None,) * 5))
    else:
        if model.speaker_emb is not None:
            x = x + _embed(model.speaker_emb, speakers, fused).unsqueeze(1)
        if model.emotion_emb is not None:
            emb = torch.cat([_embed(model.emotion_emb, emotions, fused), _embed(model.arousal_emb, arousals, fused),
                             _embed(model.valence_emb, valences, fused)], -1)
            x = x + model.emotion_linear(emb).unsqueeze(1)

    # variance adaptor (model/modules.py:102-158)
    vseed = seed if fused else None
    log_d = variance_predictor(va.duration_predictor, x, src_masks, training, compute, vseed, 1000)
    p_pred = e_pred = None
    if va.pitch_feature_level == "phoneme_level":
        p_pred, x = _variance_embed(va, "pitch", x, p_targets, src_masks, p_control, training, compute, vseed, 1002)
    if va.energy_feature_level == "phoneme_level":
        e_pred, x = _variance_embed(va, "energy", x, e_targets, src_masks, p_control, training, compute, vseed,
                                      1004)
    # phoneme-level variance (this config): the decoder crop and its position encoding join the
    # LengthRegulator's gather (one pass); frame-level variance needs the bare expanded x first
    phoneme_level = va.pitch_feature_level != "frame_level" and va.energy_feature_level != "frame_level"
    crop = dec.max_seq_len if phoneme_level else None
    pe = dec.position_enc[0].detach().contiguous() if phoneme_level else None
    if d_targets is not None:
        x, mel_len, T_lr = _length_regulate(x, d_targets, max_mel_len, crop, pe)
        d_rounded = d_targets
    else:
        d_rounded = torch.clamp(torch.round(torch.exp(log_d) - 1) * d_control, min=0)
        x, mel_len, T_lr = _length_regulate(x, d_rounded, None, crop, pe)
        mel_masks = _mask(mel_len, T_lr)
    if va.pitch_feature_level == "frame_level":
        p_pred, x = _variance_embed(va, "pitch", x, p_targets, mel_masks, p_control, training, compute, vseed,
                                      1002)
    if va.energy_feature_level == "frame_level":
        e_pred, x = _variance_embed(va, "energy", x, e_targets, mel_masks, p_control, training, compute, vseed,
                                      1004)

    # decoder (transformer/Models.py:139-171, training: crop to max_seq_len)
    T = min(x.shape[1], dec.max_seq_len)
    if not phoneme_level:
        x = x[:, :T] + dec.position_enc[:, :T, :]
    mel_masks = mel_masks[:, :T]
    dec_lens = torch.clamp((~mel_masks).sum(1), max=T)
    xb = None
    for i, blk in enumerate(dec.layer_stack):
        if fused:
            ne = len(enc.layer_stack)
            x, xb = fft_block_fused(blk, x.contiguous(), xb, dec_lens, seed, 2 * (ne + i),
                                    tr["decoder_dropout"] if training else 0.0, packs[ne + i])
        else:
            x = fft_block(blk, x, mel_masks, dec_lens, tr["decoder_dropout"], training, compute)

    # mel_linear + PostNet (+ residual) (fastspeech2.py:134-136, transformer/Layers.py:129-137)
    mel = linear(x, model.mel_linear, compute)
    p_post = 0.5 if training else 0.0
    if fused and model.training and _postnet_fused_ok(model.postnet, compute):
        postnet_mel = PostNetFn.apply(mel, (model.postnet, p_post, seed, 2000), *_postnet_params(model.postnet))
        return (mel, postnet_mel, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_len)
    y = mel
    n = len(model.postnet.convolutions)
    for i, seq in enumerate(model.postnet.convolutions):
        conv, bn = seq[0].conv, seq[1]
        z = conv1d(y, conv, (conv.kernel_size[0] - 1) // 2, compute)
        z = F.batch_norm(z.transpose(1, 2), bn.running_mean, bn.running_var, bn.weight, bn.bias, model.training,
                         bn.momentum, bn.eps).transpose(1, 2)
        if bn.num_batches_tracked is not None and model.training:
            bn.num_batches_tracked.add_(1)
        y = F.dropout(torch.tanh(z) if i < n - 1 else z, p_post, training)
    postnet_mel = y + mel
    return (mel, postnet_mel, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_len)
