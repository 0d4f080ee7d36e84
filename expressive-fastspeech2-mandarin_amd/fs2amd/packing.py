"""Weight packing for the fs2hip kernels (host side, once per parameter version).

* Q|K|V projections concatenated into one [768, 1, Cin_pad] GEMM operand (one launch, one
  read of x instead of three: SubLayers.py:39-41).
* Conv1d weights [N, Cin, K] re-laid to [N, K, Cin_pad] (k-steps = (tap, channel block)).
* PostNet BatchNorm1d (eval: running stats) folded into its conv: w' = w * g/sqrt(rv+eps),
  b' = (b - rm) * g/sqrt(rv+eps) + beta (transformer/Layers.py:92-135).
* bf16 precision: FFT blocks, mel_linear, PostNet in bf16; VariancePredictors exact f32
  (vp_precision "fp32"), bf16 ("bf16") or split-precision bf16x3 ("bf16x3", the default: w = w_hi +
  w_lo, the hidden activation as two bf16 planes, three bf16 MFMA products per term), the latter
  also stacked in the column-split form (duration + pitch conv weights side by side).
* fp8 precision (cfg5): as bf16, plus the FFN Conv1d pair of every FFT block, and the Q|K|V
  projection of every block after the first of its stack, in e4m3fn with per-output-channel
  weight scales; the dequantisation vector col_scale = s_in * s_w[n] uses the layer's static
  input-activation scale from FastSpeech2.calibrate_fp8 (s = amax / 448).
Everything else (LayerNorm affine, biases, embedding tables, bins, PE tables) stays f32.
"""
from types import SimpleNamespace

import torch

from . import _lib as L
from .ops import FP8_MAX, pack_conv_weight, pack_conv_weight_fp8, pack_conv_weight_split, pack_ffn8_weights, \
    pack_ffn_weights, pack_frag_rows, pack_vp_fused, pack_wconv_tail, pack_wconv_weight


def _f32(t, device):
    return t.detach().to(device=device, dtype=torch.float32).contiguous()


def _fft_layer(layer, device, compute, key=None, fp8_scales=None):
    a, f = layer.slf_attn, layer.pos_ffn
    wqkv = torch.cat([a.w_qs.weight, a.w_ks.weight, a.w_vs.weight], 0).to(device)
    bqkv = torch.cat([a.w_qs.bias, a.w_ks.bias, a.w_vs.bias], 0)
    fp8 = None
    if fp8_scales is not None:
        sc = fp8_scales[key]
        s_h, s_f, s_x = (max(sc[k], 1e-6) / FP8_MAX for k in ("h", "f", "x"))
        w1, sw1 = pack_conv_weight_fp8(f.w_1.weight.to(device))
        w2, sw2 = pack_conv_weight_fp8(f.w_2.weight.to(device))
        fp8 = SimpleNamespace(s_h=s_h, s_f=s_f, s_x=s_x, w1=w1, w2=w2, cs1=(sw1 * s_h).contiguous(),
                              cs2=(sw2 * s_f).contiguous(), wqkv=None, cs_qkv=None, w12_8=None)
        if tuple(w1.shape) == (1024, 9, 256) and w2.shape[0] == 256 and w2.shape[-1] == 1024:
            fp8.w12_8 = pack_ffn8_weights(w1, w2)  # the fused e4m3 FFN (fs2_ffn8)
        if key[1] > 0:  # input produced by the previous block's LN epilogue, which writes the fp8 copy
            wq, swq = pack_conv_weight_fp8(wqkv)
            fp8.wqkv, fp8.cs_qkv = wq, (swq * s_x).contiguous()
    return SimpleNamespace(
        key=key, fp8=fp8,
        n_head=a.n_head, d_k=a.d_k,
        wqkv=pack_conv_weight(wqkv, compute), bqkv=_f32(bqkv, device),
        wfc=pack_conv_weight(a.fc.weight.to(device), compute), bfc=_f32(a.fc.bias, device),
        ln1=(_f32(a.layer_norm.weight, device), _f32(a.layer_norm.bias, device), a.layer_norm.eps),
        w1=pack_conv_weight(f.w_1.weight.to(device), compute), b1=_f32(f.w_1.bias, device),
        k1=f.w_1.kernel_size[0], p1=f.w_1.padding[0], c1=f.w_1.in_channels,
        w2=pack_conv_weight(f.w_2.weight.to(device), compute), b2=_f32(f.w_2.bias, device),
        k2=f.w_2.kernel_size[0], p2=f.w_2.padding[0], c2=f.w_2.in_channels,
        ln2=(_f32(f.layer_norm.weight, device), _f32(f.layer_norm.bias, device), f.layer_norm.eps),
        w12=_ffn_pair(f, device, compute),
        # Q|K|V in fragment order for the previous block's fused FFN epilogue (fs2_ffn wqkv)
        wqf=pack_frag_rows(wqkv) if compute == L.FS2_BF16 and wqkv.shape[0] % 256 == 0 and wqkv.shape[1] == 256
        else None,
        # the attention output projection in fragment order for the fused FFN's prologue (fs2_ffn pre_w)
        wfcf=pack_frag_rows(a.fc.weight.to(device)) if compute == L.FS2_BF16 and tuple(a.fc.weight.shape) == (256, 256)
        else None,
    )


def qkv_pe_rows(pe, a, compute):
    """pe W^T + b of a block's concatenated Q|K|V projection, f64-accumulated, f32 [rows, 768]; W
    rounded to bf16 first in bf16 compute (the weights the fs2_conv1d projection multiplies)."""
    w = torch.cat([a.w_qs.weight, a.w_ks.weight, a.w_vs.weight], 0).detach().to(pe.device)
    b = torch.cat([a.w_qs.bias, a.w_ks.bias, a.w_vs.bias], 0).detach().to(pe.device)
    if compute == L.FS2_BF16:
        w = w.to(torch.bfloat16)
    return (pe.double() @ w.double().t() + b.double()).float().contiguous()


def _qkv_pe_table(pe, layers, device, compute):
    """The decoder's first Q|K|V projection of the position encoding (runtime.decode_packed: the
    LengthRegulator launch then projects the frames by linearity, fs2_lr_fused_proj) and the
    attention module it came from (runtime._qkv_pe: longer tables on demand)."""
    if len(layers) == 0 or compute != L.FS2_BF16:
        return None
    a = layers[0].slf_attn
    return SimpleNamespace(table=qkv_pe_rows(pe, a, compute), attn=a, compute=compute)


def _ffn_pair(f, device, compute):
    """w_1 | w_2 in the fs2_ffn layout (bf16 FFNs of the shapes the fused kernel covers), else None."""
    ks, F, D = f.w_1.kernel_size[0], f.w_1.out_channels, f.w_1.in_channels
    if compute != L.FS2_BF16 or D != 256 or F not in (512, 1024) or ks not in (3, 9) or f.w_2.kernel_size[0] != 1:
        return None
    return pack_ffn_weights(f.w_1.weight.to(device), f.w_2.weight.to(device))


def _vp(vp, device, compute, split=False):
    cl = vp.conv_layer
    c1, c2 = cl.conv1d_1.conv, cl.conv1d_2.conv
    if split:  # bf16x3: [x_hi | x_hi] x [w_hi | w_lo], then [h_hi | h_hi | h_lo] x [w_hi | w_lo | w_hi]
        return SimpleNamespace(
            compute=L.FS2_BF16, split=True,
            w1=pack_conv_weight_split(c1.weight.to(device), ("hi", "lo")), b1=_f32(c1.bias, device),
            k1=c1.kernel_size[0], p1=c1.padding[0], c1=c1.in_channels,
            ln1=(_f32(cl.layer_norm_1.weight, device), _f32(cl.layer_norm_1.bias, device), cl.layer_norm_1.eps),
            w2=pack_conv_weight_split(c2.weight.to(device), ("hi", "lo", "hi")), b2=_f32(c2.bias, device),
            k2=c2.kernel_size[0], p2=c2.padding[0], c2=c2.in_channels,
            ln2=(_f32(cl.layer_norm_2.weight, device), _f32(cl.layer_norm_2.bias, device), cl.layer_norm_2.eps),
            lin_w=_f32(vp.linear_layer.weight.view(-1), device), lin_b=float(vp.linear_layer.bias.detach().cpu()[0]),
        )
    return SimpleNamespace(
        compute=compute, split=False,
        w1=pack_conv_weight(c1.weight.to(device), compute), b1=_f32(c1.bias, device), k1=c1.kernel_size[0],
        p1=c1.padding[0], c1=c1.in_channels,
        ln1=(_f32(cl.layer_norm_1.weight, device), _f32(cl.layer_norm_1.bias, device), cl.layer_norm_1.eps),
        w2=pack_conv_weight(c2.weight.to(device), compute), b2=_f32(c2.bias, device), k2=c2.kernel_size[0],
        p2=c2.padding[0], c2=c2.in_channels,
        ln2=(_f32(cl.layer_norm_2.weight, device), _f32(cl.layer_norm_2.bias, device), cl.layer_norm_2.eps),
        lin_w=_f32(vp.linear_layer.weight.view(-1), device), lin_b=float(vp.linear_layer.bias.detach().cpu()[0]),
    )


def _vp_columns(vps, device):
    """Column-split bf16x3 form of G VariancePredictors that read the same input (runtime.
    variance_predictors): conv1 / conv2 weights of the G predictors stacked along N (one launch
    each, workgroups own column slices), LayerNorm / Linear parameters stacked per group for
    fs2_vp_norm / fs2_vp_head. conv1 reads [x_hi | x_hi] (x is bf16: x_lo = 0) against
    [w_hi | w_lo]; conv2 reads each group's [h_hi | h_hi | h_lo] against [w_hi | w_lo | w_hi]."""
    cls = [vp.conv_layer for vp in vps]
    c1s = [cl.conv1d_1.conv for cl in cls]
    c2s = [cl.conv1d_2.conv for cl in cls]
    geo = {(c.kernel_size[0], c.padding[0], c.in_channels, c.out_channels) for c in c1s + c2s}
    eps = {cl.layer_norm_1.eps for cl in cls} | {cl.layer_norm_2.eps for cl in cls}
    if len(geo) != 1 or len(eps) != 1:
        return None
    k, p, cin, cout = geo.pop()
    if cin != 256 or cout != 256:
        return None
    cat = lambda ts: torch.cat([_f32(t, device).reshape(-1) for t in ts]).contiguous()
    return SimpleNamespace(
        G=len(vps), c=cin, k=k, p=p, eps=eps.pop(),
        w1=torch.cat([pack_conv_weight_split(c.weight.to(device), ("hi", "lo")) for c in c1s], 0).contiguous(),
        b1=cat([c.bias for c in c1s]),
        g1=cat([cl.layer_norm_1.weight for cl in cls]), be1=cat([cl.layer_norm_1.bias for cl in cls]),
        w2=torch.cat([pack_conv_weight_split(c.weight.to(device), ("hi", "lo", "hi")) for c in c2s], 0).contiguous(),
        b2=cat([c.bias for c in c2s]),
        g2=cat([cl.layer_norm_2.weight for cl in cls]), be2=cat([cl.layer_norm_2.bias for cl in cls]),
        lin_w=cat([vp.linear_layer.weight for vp in vps]), lin_b=cat([vp.linear_layer.bias for vp in vps]),
    )


def _vp_fused(vps, device):
    """fs2_vp_fused form of G VariancePredictors that read the same input (bf16x3): the conv
    weights as hi / lo parts in fragment order, the seven 256-vectors per predictor."""
    cls = [vp.conv_layer for vp in vps]
    convs = [(cl.conv1d_1.conv, cl.conv1d_2.conv) for cl in cls]
    ok = all(c.in_channels == 256 and c.out_channels == 256 and c.kernel_size[0] == 3 and c.padding[0] == 1
             for pair in convs for c in pair)
    eps = {cl.layer_norm_1.eps for cl in cls} | {cl.layer_norm_2.eps for cl in cls}
    if not ok or len(eps) != 1:
        return None
    vec = torch.stack([torch.stack([_f32(t, device).reshape(-1) for t in (
        cl.conv1d_1.conv.bias, cl.layer_norm_1.weight, cl.layer_norm_1.bias, cl.conv1d_2.conv.bias,
        cl.layer_norm_2.weight, cl.layer_norm_2.bias, vp.linear_layer.weight)]) for cl, vp in zip(cls, vps)])
    return SimpleNamespace(
        G=len(vps), eps=eps.pop(), vec=vec.contiguous(),
        w=pack_vp_fused([(c1.weight.to(device), c2.weight.to(device)) for c1, c2 in convs]),
        lin_b=torch.cat([_f32(vp.linear_layer.bias, device).reshape(-1) for vp in vps]).contiguous())


def _postnet(pn, device, compute):
    layers = []
    for seq in pn.convolutions:
        conv, bn = seq[0].conv, seq[1]
        s = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
        b = (conv.bias.detach().float() - bn.running_mean.detach().float()) * s + bn.bias.detach().float()
        wfr = wtail = None
        if compute == L.FS2_BF16 and conv.in_channels in (512, 80) and conv.out_channels == 512 \
                and conv.kernel_size[0] == 5:
            # the weight-streamed kernel's fragment order (fs2_wconv)
            wfr = pack_wconv_weight(conv.weight.to(device), scale=s.to(device))
        if compute == L.FS2_BF16 and conv.in_channels == 512 and conv.out_channels == 80 \
                and conv.kernel_size[0] == 5 and conv.padding[0] == 2:
            # the last conv + residual on fs2_wconv's N = 80 form
            wtail = pack_wconv_tail(conv.weight.to(device), scale=s.to(device))
        layers.append(SimpleNamespace(w=pack_conv_weight(conv.weight.to(device), compute, scale=s.to(device)),
                                      b=_f32(b, device), k=conv.kernel_size[0], p=conv.padding[0],
                                      cin=conv.in_channels, cout=conv.out_channels, wfr=wfr, wtail=wtail))
    return layers


def pack_model(model, device, precision, vp_precision="fp32", fp8_scales=None):
    device = torch.device(device)
    big = L.FS2_BF16 if precision in ("bf16", "fp8") else L.FS2_F32
    low = precision in ("bf16", "fp8")
    vpc = L.FS2_BF16 if (low and vp_precision == "bf16") else L.FS2_F32
    vsplit = low and vp_precision == "bf16x3"
    if precision == "fp8" and fp8_scales is None:
        raise RuntimeError("fs2amd: fp8 precision needs activation scales: call model.calibrate_fp8(**batch) first")
    sc = fp8_scales if precision == "fp8" else None
    va = model.variance_adaptor
    P = SimpleNamespace(precision=precision, compute=big, act_dtype=big, device=device)
    P.enc_emb = _f32(model.encoder.src_word_emb.weight, device)
    P.enc_pe = _f32(model.encoder.position_enc[0], device)
    P.dec_pe = _f32(model.decoder.position_enc[0], device)
    P.enc_layers = [_fft_layer(l, device, big, ("enc", i), sc) for i, l in enumerate(model.encoder.layer_stack)]
    P.dec_layers = [_fft_layer(l, device, big, ("dec", i), sc) for i, l in enumerate(model.decoder.layer_stack)]
    P.dec_qkv_pe = _qkv_pe_table(P.dec_pe, model.decoder.layer_stack, device, big)
    P.vp = {k: _vp(getattr(va, f"{k}_predictor"), device, vpc, vsplit) for k in ("duration", "pitch", "energy")}
    # bf16x3 VariancePredictors in their column-split form (duration + pitch side by side, energy)
    P.vpcols = None
    P.vpfused = None
    if vsplit:
        dp = _vp_columns([va.duration_predictor, va.pitch_predictor], device)
        en = _vp_columns([va.energy_predictor], device)
        if dp is not None and en is not None:
            P.vpcols = SimpleNamespace(dp=dp, energy=en)
        # ... and as whole fused predictors (fs2_vp_fused: one launch per set)
        fdp = _vp_fused([va.duration_predictor, va.pitch_predictor], device)
        fen = _vp_fused([va.energy_predictor], device)
        P.vpfused = SimpleNamespace(dp=fdp, energy=fen) if fdp is not None and fen is not None else None
    P.bins = {k: _f32(getattr(va, f"{k}_bins"), device) for k in ("pitch", "energy")}
    P.var_table = {k: _f32(getattr(va, f"{k}_embedding").weight, device) for k in ("pitch", "energy")}
    P.mel_w = pack_conv_weight(model.mel_linear.weight.to(device), big)
    P.mel_b = _f32(model.mel_linear.bias, device)
    P.n_mel = model.mel_linear.out_features
    P.postnet = _postnet(model.postnet, device, big)
    P.spk_table = _f32(model.speaker_emb.weight, device) if model.speaker_emb is not None else None
    if model.emotion_emb is not None:
        P.emo_table = _f32(model.emotion_emb.weight, device)
        P.aro_table = _f32(model.arousal_emb.weight, device)
        P.val_table = _f32(model.valence_emb.weight, device)
        P.emo_w = _f32(model.emotion_linear[0].weight, device)
        P.emo_b = _f32(model.emotion_linear[0].bias, device)
    else:
        P.emo_table = None
    P.d_model = model.encoder.d_model
    P.max_seq_len = model.encoder.max_seq_len
    return P
