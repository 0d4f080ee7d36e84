"""FastSpeech2.forward on the fs2hip kernels — the launch sequence of the hot path.

Mirrors model/fastspeech2.py:73-148 step by step (eval semantics, reference quirks kept):

  src_masks / mel_masks                       utils/tools.py:152-160 (returned tensors)
  embed + PE                    fs2_embed_pe   transformer/Models.py:82-91
  4 x FFT block (encoder)       5 launches     transformer/Layers.py:21-30
     Q|K|V GEMM (N=768)  -> attention -> fc + res + LN + mask -> conv k9 + ReLU -> conv k1 + res + LN + mask
     (the last block's epilogue also adds the speaker and emotion vectors, fastspeech2.py:101-110)
  VarianceAdaptor                              model/modules.py:102-158
     duration VP (f32), pitch VP -> bucketize/embed add, energy VP (uses p_control, :124-125)
     -> LengthRegulator scan (+ duration rounding :132-135) -> gather (+ decoder PE add)
  6 x FFT block (decoder)                      transformer/Models.py:139-171
  mel_linear, PostNet (BN folded) + residual   fastspeech2.py:134-136, transformer/Layers.py:129-137

Every arithmetic step is a HIP kernel launched on torch.cuda.current_stream(); torch only
allocates buffers and builds the two boolean mask tensors the 10-tuple returns. With
``max_mel_len`` given (teacher-forced / training-style batches) the path has no host sync;
without it, one device->host read of max(mel_len) sizes the decoder (the reference does
B*L_max .item() syncs in LengthRegulator.expand).
"""
import numpy as np
import torch

from . import _lib as L
from . import ops
from .model import sinusoid_table


def _mask(lengths, width):
    """get_mask_from_lengths (utils/tools.py:152-160): True = padding (one fs2_length_masks launch)."""
    if lengths.is_cuda:
        return ops.length_mask(lengths, width)
    ids = torch.arange(0, width, device=lengths.device).unsqueeze(0).expand(lengths.shape[0], -1)
    return ids >= lengths.unsqueeze(1).expand(-1, width)


def _pe(P, which, n):
    tab = P.enc_pe if which == "enc" else P.dec_pe
    if n <= tab.shape[0]:
        return tab
    # eval with a sequence longer than max_seq_len: the reference recomputes the table for the
    # whole length (Models.py:82-87,145-152); its first rows equal the stored ones.
    key = f"_pe_{which}_{n}"
    if not hasattr(P, key):
        setattr(P, key, sinusoid_table(n, tab.shape[1]).to(tab.device))
    return getattr(P, key)


# Optional measurement hook: when a list, the decoder's FFN conv-k9 launches are bracketed by
# HIP events on the launch stream (bench.py's live roofline timing of the dominant kernel).
TIMERS = None


def fft_block(P, lp, x, lens, addvec1=None, addvec2=None, timed=False, layout=None):
    """One FFT block (transformer/Layers.py:21-30) = 5 launches. With ``layout`` (ops.SeqLayout)
    x is packed [B*T, d_model]: only valid frames exist and no mask is applied (nothing to mask)."""
    c = P.compute
    dt = P.act_dtype
    H, dk = lp.n_head, lp.d_k
    d_model = H * dk
    if layout is not None:
        lens = None
    qkv = ops.conv1d(x, lp.wqkv, lp.bqkv, cin=d_model, ks=1, pad=0, compute=c, epilogue=L.EPI_BIAS, out_dtype=dt,
                     layout=layout)
    att = ops.attention(qkv, lens, H, dk, float(np.power(dk, 0.5)), layout=layout)
    h = ops.conv1d(att, lp.wfc, lp.bfc, cin=d_model, ks=1, pad=0, compute=c, epilogue=L.EPI_RES_LN, out_dtype=dt,
                   residual=x, ln=lp.ln1, lens=lens, layout=layout)
    if timed and TIMERS is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    f = ops.conv1d(h, lp.w1, lp.b1, cin=lp.c1, ks=lp.k1, pad=lp.p1, compute=c, epilogue=L.EPI_BIAS_RELU, out_dtype=dt,
                   layout=layout)
    if timed and TIMERS is not None:
        e1.record()
        TIMERS.append((e0, e1))
    return ops.conv1d(f, lp.w2, lp.b2, cin=lp.c2, ks=lp.k2, pad=lp.p2, compute=c, epilogue=L.EPI_RES_LN, out_dtype=dt,
                      residual=h, ln=lp.ln2, lens=lens, addvec1=addvec1, addvec2=addvec2, layout=layout)


def packed_decoder_ok(P):
    """The packed decoder equals the reference's padded one when every padded frame an FFT block
    reads through a conv tap is zero there: h (input of w_1) is masked after the attention
    LayerNorm, and f = relu(w_1 h + b) (input of w_2) is not, so w_2 must be kernel-1
    (model.yaml conv_kernel_size [9, 1]). Attention only sees keys < len either way.
    FS2_PACKED_DECODER=0 forces the padded path."""
    import os
    if os.environ.get("FS2_PACKED_DECODER", "1") == "0":
        return False
    return all(lp.k2 == 1 and lp.p2 == 0 for lp in P.dec_layers)


def variance_predictor(vp, x, lens):
    """VariancePredictor (model/modules.py:209-250): 2 launches -> f32 [B, T] (f32 or bf16 MFMA)."""
    h = ops.conv1d(x, vp.w1, vp.b1, cin=vp.c1, ks=vp.k1, pad=vp.p1, compute=vp.compute, epilogue=L.EPI_RELU_LN,
                   out_dtype=vp.compute, ln=vp.ln1)
    return ops.conv1d(h, vp.w2, vp.b2, cin=vp.c2, ks=vp.k2, pad=vp.p2, compute=vp.compute,
                      epilogue=L.EPI_RELU_LN_DOT, ln=vp.ln2, lens=lens, dot=(vp.lin_w, vp.lin_b))


def _variance(P, kind, x, lens, target, control):
    pred = variance_predictor(P.vp[kind], x, lens)
    tgt = None
    if target is not None:
        tgt = target.to(device=x.device, dtype=torch.float32).contiguous()
    ops.variance_embed(x, pred, tgt, control, P.bins[kind], P.var_table[kind])
    return pred


def _device_ok(dev):
    return dev.type == "cuda"


def run_forward(model, speakers, emotions, arousals, valences, texts, src_lens, max_src_len, mels, mel_lens,
                max_mel_len, p_targets, e_targets, d_targets, p_control, e_control, d_control):
    dev = texts.device
    if not _device_ok(dev):
        raise RuntimeError("fs2amd: FastSpeech2.forward runs on the HIP kernels only; move the model and the batch "
                           "to a ROCm device (no CPU fallback)")
    P = model.packed(dev)
    va = model.variance_adaptor
    ids = lambda t: None if t is None else torch.as_tensor(t).to(device=dev, dtype=torch.int64).contiguous()
    speakers, emotions, arousals, valences = ids(speakers), ids(emotions), ids(arousals), ids(valences)
    B = texts.shape[0]
    Lx = int(max_src_len)
    if texts.shape[1] != Lx:
        raise RuntimeError(f"texts has {texts.shape[1]} positions but max_src_len is {Lx}")
    src_lens = src_lens.to(dev)
    src_masks = _mask(src_lens, Lx)
    mel_masks = _mask(mel_lens, max_mel_len if max_mel_len is not None else int(mel_lens.max().item())) \
        if mel_lens is not None else None
    lens_src = src_lens.to(torch.int64).contiguous()

    # ---- encoder (+ speaker / emotion conditioning fused into the last block's epilogue) -------
    x = ops.embed_pe(ids(texts), P.enc_emb, _pe(P, "enc", Lx), P.act_dtype)
    spk_vec = emo_vec = None
    if P.spk_table is not None or P.emo_table is not None:
        spk_vec, emo_vec = ops.cond_vectors(
            speakers if P.spk_table is not None else None, P.spk_table,
            emotions if P.emo_table is not None else None, arousals, valences, P.emo_table,
            getattr(P, "aro_table", None), getattr(P, "val_table", None), getattr(P, "emo_w", None),
            getattr(P, "emo_b", None), P.d_model)
    n_enc = len(P.enc_layers)
    for i, lp in enumerate(P.enc_layers):
        last = i == n_enc - 1
        x = fft_block(P, lp, x, lens_src, spk_vec if last else None, emo_vec if last else None)
    if n_enc == 0 and (spk_vec is not None or emo_vec is not None):
        raise NotImplementedError("encoder_layer = 0")

    # ---- variance adaptor --------------------------------------------------------------------
    phoneme_p = va.pitch_feature_level == "phoneme_level"
    phoneme_e = va.energy_feature_level == "phoneme_level"
    log_d = variance_predictor(P.vp["duration"], x, lens_src)
    p_pred = e_pred = None
    if phoneme_p:
        p_pred = _variance(P, "pitch", x, lens_src, p_targets, p_control)
    if phoneme_e:
        e_pred = _variance(P, "energy", x, lens_src, e_targets, p_control)  # p_control: modules.py:124-125

    if d_targets is not None:
        dur = d_targets.to(dev)
        if dur.dtype not in (torch.int64, torch.float32):
            dur = dur.to(torch.int64)
        cum, mel_len, _ = ops.lr_durations(dur)
        d_rounded = d_targets
    else:
        cum, mel_len, d_rounded = ops.lr_durations(log_d, logpred=True, d_control=d_control)
    if max_mel_len:
        T_out = int(max_mel_len)
    else:
        T_out = int(mel_len.max().item()) if B else 0
    if d_targets is None:
        mel_masks = _mask(mel_len, int(mel_len.max().item()) if B else 0)
    dec_lens = mel_len if d_targets is None else mel_lens.to(dev).to(torch.int64)
    if mel_masks is None or mel_masks.shape[1] != T_out:
        raise RuntimeError(f"decoder mask width {None if mel_masks is None else mel_masks.shape[1]} != length-"
                           f"regulated length {T_out} (the reference fails here too: Models.py:157)")
    frame_level = not (phoneme_p and phoneme_e)
    if model.training:
        T_dec = min(T_out, P.max_seq_len)
    else:
        T_dec = T_out
    if not frame_level and T_dec == T_out and packed_decoder_ok(P):
        # packed decoder: only the dec_lens frames of each utterance are computed
        # (cfg2: 24.9k of 27.5k rows, cfg4: 135k of 249k); mel_linear scatters back to [B, T, n_mel]
        lay = ops.SeqLayout(dec_lens, T_dec)
        x = ops.lr_expand(x, cum, mel_len, T_out, pe=_pe(P, "dec", T_out), out_dtype=P.act_dtype, out_layout=lay)
        for lp in P.dec_layers:
            x = fft_block(P, lp, x, None, timed=True, layout=lay)
        mel = ops.conv1d(x, P.mel_w, P.mel_b, cin=P.d_model, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_BIAS,
                         out_dtype=L.FS2_F32, src_layout=lay)
        postnet_mel = _postnet(P, mel)
        return (mel, postnet_mel, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_len)
    # LR gather with the decoder's position encoding fused (frame-level variance needs the bare
    # expanded x first, so the PE add moves to a second pass in that configuration)
    if frame_level:
        x = ops.lr_expand(x, cum, mel_len, T_out, pe=None, out_dtype=P.act_dtype)
        if not phoneme_p:
            p_pred = _variance(P, "pitch", x, dec_lens, p_targets, p_control)
        if not phoneme_e:
            e_pred = _variance(P, "energy", x, dec_lens, e_targets, p_control)
        x = x[:, :T_dec].contiguous()
        x = _add_pe(x, _pe(P, "dec", T_dec))
    else:
        x = ops.lr_expand(x, cum, mel_len, T_out, pe=_pe(P, "dec", T_out), out_dtype=P.act_dtype)
        if T_dec != T_out:
            x = x[:, :T_dec].contiguous()
    if T_dec != T_out:
        mel_masks = mel_masks[:, :T_dec]
        dec_lens = torch.clamp(dec_lens, max=T_dec)

    # ---- decoder --------------------------------------------------------------------------------
    for lp in P.dec_layers:
        x = fft_block(P, lp, x, dec_lens, timed=True)

    # ---- mel_linear + PostNet (+ residual) -----------------------------------------------------
    mel = ops.conv1d(x, P.mel_w, P.mel_b, cin=P.d_model, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_BIAS,
                     out_dtype=L.FS2_F32)
    postnet_mel = _postnet(P, mel)
    return (mel, postnet_mel, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_len)


def _postnet(P, mel):
    """PostNet (BN folded, transformer/Layers.py:92-137) + residual (fastspeech2.py:136), padded
    [B, T, n_mel] like the reference: its padded frames (bias values) feed the k5 taps."""
    y = mel
    n_pn = len(P.postnet)
    for i, lp in enumerate(P.postnet):
        if i < n_pn - 1:
            y = ops.conv1d(y, lp.w, lp.b, cin=lp.cin, ks=lp.k, pad=lp.p, compute=P.compute,
                           epilogue=L.EPI_BIAS_TANH, out_dtype=P.act_dtype)
        else:
            y = ops.conv1d(y, lp.w, lp.b, cin=lp.cin, ks=lp.k, pad=lp.p, compute=P.compute, epilogue=L.EPI_BIAS_RES,
                           out_dtype=L.FS2_F32, residual=mel)
    return y


def _add_pe(x, pe):
    """x[b, t] += pe[t] via the LR gather with identity durations (every frame its own source)."""
    B, T, D = x.shape
    ones = torch.ones(B, T, dtype=torch.int64, device=x.device)
    cum, ml, _ = ops.lr_durations(ones)
    return ops.lr_expand(x, cum, ml, T, pe=pe, out_dtype=ops._dt(x))
