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
    ``fs2_lr_expand``, the differentiable gather (and its scatter-add gradient) in torch;
  * LayerNorm, dropout, BatchNorm, embeddings, losses: torch on the device.
Parity: tests/test_gpu_train.py against the reference's own gradients (train_grads.npz).
"""
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


def variance_predictor(vp, x, mask, training, compute):
    """model/modules.py:209-250 (conv1d_2 padding hard-coded to 1, :230)."""
    cl = vp.conv_layer
    k = cl.conv1d_1.conv.kernel_size[0]
    h = torch.relu(conv1d(x, cl.conv1d_1.conv, (k - 1) // 2, compute))
    h = F.dropout(_layer_norm(h, cl.layer_norm_1), cl.dropout_1.p, training)
    h = torch.relu(conv1d(h, cl.conv1d_2.conv, 1, compute))
    h = F.dropout(_layer_norm(h, cl.layer_norm_2), cl.dropout_2.p, training)
    out = F.linear(h, vp.linear_layer.weight, vp.linear_layer.bias).squeeze(-1)
    return out.masked_fill(mask, 0.0)


def _variance_embed(va, kind, x, target, mask, control, training, compute):
    """model/modules.py:80-100,117-126 (energy is scaled by p_control in the reference)."""
    pred = variance_predictor(getattr(va, f"{kind}_predictor"), x, mask, training, compute)
    bins = getattr(va, f"{kind}_bins")
    table = getattr(va, f"{kind}_embedding")
    if target is not None:
        emb = table(torch.bucketize(target, bins))
    else:
        pred = pred * control
        emb = table(torch.bucketize(pred, bins))
    return pred, emb


def _length_regulate(x, dur, max_len):
    """LengthRegulator (model/modules.py:161-194): HIP scan + source-index map, torch gather."""
    cum, mel_len, _ = ops.lr_durations(dur if dur.dtype in (torch.int64, torch.float32) else dur.to(torch.int64))
    T = int(max_len) if max_len else int(mel_len.max().item())
    im = ops.lr_expand(x.detach(), cum, mel_len, T, map_only=True)
    B, Lx, D = x.shape
    xz = torch.cat([x, x.new_zeros(B, 1, D)], 1)
    idx = torch.where(im < 0, torch.full_like(im, Lx), im).long()
    return torch.gather(xz, 1, idx.unsqueeze(-1).expand(-1, -1, D)), mel_len


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
    x = enc.src_word_emb(texts) + enc.position_enc[:, :Lx, :]
    for blk in enc.layer_stack:
        x = fft_block(blk, x, src_masks, lens_src, tr["encoder_dropout"], training, compute)
    if model.speaker_emb is not None:
        x = x + model.speaker_emb(speakers).unsqueeze(1)
    if model.emotion_emb is not None:
        emb = torch.cat([model.emotion_emb(emotions), model.arousal_emb(arousals), model.valence_emb(valences)], -1)
        x = x + model.emotion_linear(emb).unsqueeze(1)

    # variance adaptor (model/modules.py:102-158)
    log_d = variance_predictor(va.duration_predictor, x, src_masks, training, compute)
    p_pred = e_pred = None
    if va.pitch_feature_level == "phoneme_level":
        p_pred, emb = _variance_embed(va, "pitch", x, p_targets, src_masks, p_control, training, compute)
        x = x + emb
    if va.energy_feature_level == "phoneme_level":
        e_pred, emb = _variance_embed(va, "energy", x, e_targets, src_masks, p_control, training, compute)
        x = x + emb
    if d_targets is not None:
        x, mel_len = _length_regulate(x, d_targets, max_mel_len)
        d_rounded = d_targets
    else:
        d_rounded = torch.clamp(torch.round(torch.exp(log_d) - 1) * d_control, min=0)
        x, mel_len = _length_regulate(x, d_rounded, None)
        mel_masks = _mask(mel_len, int(mel_len.max().item()))
    if va.pitch_feature_level == "frame_level":
        p_pred, emb = _variance_embed(va, "pitch", x, p_targets, mel_masks, p_control, training, compute)
        x = x + emb
    if va.energy_feature_level == "frame_level":
        e_pred, emb = _variance_embed(va, "energy", x, e_targets, mel_masks, p_control, training, compute)
        x = x + emb

    # decoder (transformer/Models.py:139-171, training: crop to max_seq_len)
    T = min(x.shape[1], dec.max_seq_len)
    x = x[:, :T] + dec.position_enc[:, :T, :]
    mel_masks = mel_masks[:, :T]
    dec_lens = torch.clamp((~mel_masks).sum(1), max=T)
    for blk in dec.layer_stack:
        x = fft_block(blk, x, mel_masks, dec_lens, tr["decoder_dropout"], training, compute)

    # mel_linear + PostNet (+ residual) (fastspeech2.py:134-136, transformer/Layers.py:129-137)
    mel = linear(x, model.mel_linear, compute)
    y = mel
    n = len(model.postnet.convolutions)
    p_post = 0.5 if training else 0.0
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
