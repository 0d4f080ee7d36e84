"""HiFi-GAN V1 generator (mel -> waveform) on the fs2hip conv kernels.

Drop-in for ``hifigan.Generator`` (hifigan/models.py:112-173; same constructor ``Generator(h)``,
same weight-normed parameter names, ``forward(x[B, 80, T]) -> [B, 1, T*prod(upsample_rates)]``,
``remove_weight_norm()``) and for ``utils/model.py:42-92`` ``get_vocoder`` / ``vocoder_infer``
(HiFi-GAN branch; the MelGAN branch is a remote ``torch.hub`` fetch and is not provided).

Every conv runs in ``fs2_conv1d`` (implicit GEMM on MFMA) with the activations channels-last
``[B, T_stage, C]`` in HBM and the generator's elementwise work fused into epilogues:

* ``conv_pre``: Conv1d(80 -> 512, k7) + the first upsampler's ``leaky_relu(0.1)`` (EPI_BIAS_LRELU).
* ``ups[i]``: ConvTranspose1d(k, stride u, padding (k-u)/2) rewritten as ONE dense conv: output
  sample t*u + r (phase r) only sees inputs t + q_r - j, so the transposed conv is a 3-tap Conv1d
  whose N = u * Cout outputs per input frame are the u phases side by side — and [T, u*Cout]
  row-major IS [T*u, Cout], so the interleave costs nothing. Its epilogue writes the raw output
  (the ResBlocks' residual) and ``leaky_relu(0.1)`` of it (their convs1 input) in one pass.
* ``ResBlock`` (k, dilations 1/3/5): convs1 dilated conv + leaky_relu (EPI_BIAS_LRELU, dilation in
  the halo), convs2 conv + residual (EPI_RES_SUM) whose second output is the next pair's
  ``leaky_relu(x)``; the last pair of resblock j also adds the running multi-receptive-field sum
  ``xs`` (residual2, in place) and, for the last kernel, divides by ``num_kernels`` and emits
  ``leaky_relu(xs / 3)`` for the next upsampler (slope 0.1) or for ``conv_post`` (slope 0.01,
  ``F.leaky_relu``'s default, hifigan/models.py:159).
* ``conv_post``: Conv1d(32 -> 1, k7) + tanh (EPI_BIAS_TANH; N padded to 4).

Weight norm (``w = g * v / ||v||`` per output row, dim 0) is folded on the host when the weights
are packed, as the reference's ``remove_weight_norm()`` does before inference.
"""
import json
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L

LRELU_SLOPE = 0.1  # hifigan/models.py:7

V1_CONFIG = {  # hifigan/config.json (the generator's keys)
    "resblock": "1", "upsample_rates": [8, 8, 2, 2], "upsample_kernel_sizes": [16, 16, 4, 4],
    "upsample_initial_channel": 512, "resblock_kernel_sizes": [3, 7, 11],
    "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]], "num_mels": 80, "hop_size": 256,
    "sampling_rate": 22050,
}


class AttrDict(dict):
    """hifigan/__init__.py AttrDict: a dict whose keys are attributes."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


def get_padding(kernel_size, dilation=1):
    return int((kernel_size * dilation - dilation) / 2)


def _wn(module):
    # the reference's (deprecated) torch.nn.utils.weight_norm: parameters weight_g / weight_v
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return nn.utils.weight_norm(module)


class ResBlock(nn.Module):
    """Parameter holder of hifigan/models.py:20-114 (ResBlock1)."""

    def __init__(self, h, channels, kernel_size=3, dilation=(1, 3, 5)):
        super().__init__()
        self.h, self.kernel_size, self.dilation = h, kernel_size, tuple(dilation)
        self.convs1 = nn.ModuleList([_wn(nn.Conv1d(channels, channels, kernel_size, 1, dilation=d,
                                                   padding=get_padding(kernel_size, d))) for d in dilation])
        self.convs2 = nn.ModuleList([_wn(nn.Conv1d(channels, channels, kernel_size, 1, dilation=1,
                                                   padding=get_padding(kernel_size, 1))) for _ in dilation])

    def remove_weight_norm(self):
        for c in list(self.convs1) + list(self.convs2):
            if hasattr(c, "weight_g"):
                nn.utils.remove_weight_norm(c)


def _weight(conv):
    """Effective weight of a (possibly weight-normed) conv: g * v / ||v||, norm over dims != 0."""
    if hasattr(conv, "weight_g"):
        return torch._weight_norm(conv.weight_v.detach(), conv.weight_g.detach(), 0)
    return conv.weight.detach()


def phase_conv_weights(w, u, padding):
    """ConvTranspose1d weight [Cin, Cout, K] (stride u, padding p) -> an equivalent Conv1d over the
    input frames with N = u*Cout outputs (phase-major: column r*Cout + c is output sample t*u + r,
    channel c): returns (weight [u*Cout, Cin, KS], conv padding). Output sample t*u + r sums
    x[t + q - j] * w[:, c, j*u + s] over j, with q, s = divmod(r + p, u)."""
    cin, cout, K = w.shape
    taps = []
    for r in range(u):
        q, s = divmod(r + padding, u)
        for j in range(K // u + 1):
            k = j * u + s
            if k < K:
                taps.append((r, q - j, k))
    offs = [t[1] for t in taps]
    lo, hi = min(offs), max(offs)
    out = torch.zeros(u * cout, cin, hi - lo + 1, dtype=w.dtype, device=w.device)
    for r, off, k in taps:
        out[r * cout:(r + 1) * cout, :, off - lo] = w[:, :, k].t()
    return out, -lo


class Generator(nn.Module):
    """hifigan/models.py:112-173 (V1 generator) with the forward on fs2_conv1d."""

    def __init__(self, h):
        super().__init__()
        h = h if isinstance(h, AttrDict) else AttrDict(h)
        self.h = h
        self.num_kernels = len(h.resblock_kernel_sizes)
        self.num_upsamples = len(h.upsample_rates)
        self.conv_pre = _wn(nn.Conv1d(80, h.upsample_initial_channel, 7, 1, padding=3))
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(h.upsample_rates, h.upsample_kernel_sizes)):
            self.ups.append(_wn(nn.ConvTranspose1d(h.upsample_initial_channel // (2 ** i),
                                                   h.upsample_initial_channel // (2 ** (i + 1)), k, u,
                                                   padding=(k - u) // 2)))
        self.resblocks = nn.ModuleList()
        for i in range(len(self.ups)):
            ch = h.upsample_initial_channel // (2 ** (i + 1))
            for k, d in zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes):
                self.resblocks.append(ResBlock(h, ch, k, d))
        self.conv_post = _wn(nn.Conv1d(ch, 1, 7, 1, padding=3))
        self._precision = "fp32"
        self._packs = {}
        self.register_load_state_dict_post_hook(lambda mod, keys: mod._packs.clear())

    # ---- precision / packing -------------------------------------------------------------------
    def set_precision(self, dtype):
        if dtype not in ("fp32", "bf16"):
            raise ValueError("vocoder precision must be 'fp32' or 'bf16'")
        self._precision = dtype
        return self

    @property
    def hop(self):
        return int(np.prod(self.h.upsample_rates))

    def remove_weight_norm(self):
        for m in [self.conv_pre, self.conv_post, *self.ups]:
            if hasattr(m, "weight_g"):
                nn.utils.remove_weight_norm(m)
        for rb in self.resblocks:
            rb.remove_weight_norm()
        self._packs.clear()

    def packed(self, device):
        from . import ops

        fp = sum(p._version for p in self.parameters())
        key = (self._precision, str(device))
        ent = self._packs.get(key)
        if ent is not None and ent[0] == fp:
            return ent[1]
        c = L.FS2_BF16 if self._precision == "bf16" else L.FS2_F32
        dev = torch.device(device)

        def conv(m):
            w = _weight(m).float().to(dev)
            return {"w": ops.pack_conv_weight(w, c), "b": m.bias.detach().float().to(dev).contiguous(),
                    "cin": w.shape[1], "ks": w.shape[2], "dil": m.dilation[0], "pad": m.padding[0]}

        P = {"compute": c, "pre": conv(self.conv_pre), "ups": [], "rb": []}
        for m, u in zip(self.ups, self.h.upsample_rates):
            w, pad = phase_conv_weights(_weight(m).float().to(dev), u, m.padding[0])
            b = m.bias.detach().float().to(dev).repeat(u).contiguous()
            P["ups"].append({"w": ops.pack_conv_weight(w, c), "b": b, "cin": w.shape[1], "ks": w.shape[2], "pad": pad,
                             "u": u, "cout": w.shape[0] // u})
        for rb in self.resblocks:
            P["rb"].append([(conv(c1), conv(c2)) for c1, c2 in zip(rb.convs1, rb.convs2)])
        # the narrow stages' multi-receptive-field blocks as one fused launch each (fs2_hifigan_mrf;
        # the 32-channel stage, and the 64-channel one with FS2_VOC_PAIR64=0)
        P["mrf"] = {}
        # the 128- and 64-channel stages: one fused launch per ResBlock1 dilation pair
        # (fs2_hifigan_pair; 64 channels: 5.6 vs 7.3 ms for the stage as one MRF launch)
        P["pair"] = {}
        if c == L.FS2_BF16 and list(self.h.resblock_kernel_sizes) == [3, 7, 11] and \
                all(list(d) == [1, 3, 5] for d in self.h.resblock_dilation_sizes) and str(self.h.resblock) == "1":
            nk = self.num_kernels
            for i in range(self.num_upsamples):
                ch = self.h.upsample_initial_channel // (2 ** (i + 1))
                if ch in (128, 64):
                    P["pair"][i] = [[(ops.pack_wconv_tail(_weight(c1).float().to(dev)), c1.bias.detach().float().to(dev),
                                      ops.pack_wconv_tail(_weight(c2).float().to(dev)), c2.bias.detach().float().to(dev),
                                      c1.kernel_size[0], c1.dilation[0])
                                     for c1, c2 in zip(rb.convs1, rb.convs2)]
                                    for rb in self.resblocks[i * nk:(i + 1) * nk]]
                if ch not in (32, 64):
                    continue
                ws, bs = [], []
                for j in range(nk):
                    rb = self.resblocks[i * nk + j]
                    for c1, c2 in zip(rb.convs1, rb.convs2):
                        for m in (c1, c2):
                            ws.append(ops.pack_wconv_tail(_weight(m).float().to(dev)))
                            bs.append(m.bias.detach().float().to(dev))
                P["mrf"][i] = (torch.cat(ws).contiguous(), torch.cat(bs).contiguous())
        wp = _weight(self.conv_post).float().to(dev)
        w4 = torch.zeros(4, wp.shape[1], wp.shape[2], device=dev)
        w4[:1] = wp
        b4 = torch.zeros(4, device=dev)
        b4[:1] = self.conv_post.bias.detach().float()
        P["post"] = {"w": ops.pack_conv_weight(w4, c), "b": b4, "cin": wp.shape[1], "ks": wp.shape[2], "pad": 3}
        if c == L.FS2_BF16 and wp.shape[1] == 32 and wp.shape[2] == 7:
            # the streaming one-channel kernel (fs2_hifigan_post): bf16 weights tap-major [7, 32]
            P["post1"] = (wp[0].t().contiguous().to(torch.bfloat16), float(self.conv_post.bias.detach()[0]))
        self._packs[key] = (fp, P)
        return P

    def _pair_stage(self, chains, xu, out_slope):
        """A 128- or 64-channel stage's multi-receptive-field block as 9 fs2_hifigan_pair launches
        (256-sample tiles at C = 128, 512-sample tiles at C = 64):
        chain j's pairs 0 and 1 ping-pong between two buffers, its last pair adds into the running
        sum xs (in place), and the last chain's emits leaky_relu(xs / num_kernels, out_slope)."""
        from . import ops

        nk = len(chains)
        xa, xb, xs, nxt = (torch.empty_like(xu) for _ in range(4))
        for j, pairs in enumerate(chains):
            xp = xu
            for pi, (w1, b1, w2, b2, k, d) in enumerate(pairs):
                if pi < len(pairs) - 1:
                    xn = xa if xp is not xa else xb
                    ops.hifigan_pair(xp, w1, b1, w2, b2, k, d, out=xn)
                    xp = xn
                elif j < nk - 1:
                    ops.hifigan_pair(xp, w1, b1, w2, b2, k, d, xs=xs if j > 0 else None, out=xs)
                else:
                    ops.hifigan_pair(xp, w1, b1, w2, b2, k, d, xs=xs, out_scale=1.0 / nk, out_slope=out_slope,
                                     out_act=True, out=nxt)
        return nxt

    # ---- forward ---------------------------------------------------------------------------------
    def forward(self, x):
        """x: mel [B, n_mels, T] (the reference's layout) -> waveform [B, 1, T * hop] (f32)."""
        return self.forward_btc(x.transpose(1, 2)).unsqueeze(1)

    def forward_btc(self, mel):
        """mel [B, T, n_mels] (FastSpeech2's postnet output layout, no transpose) -> [B, T * hop] f32."""
        from . import ops

        if not mel.is_cuda:
            raise RuntimeError("fs2amd: the HiFi-GAN generator runs on the HIP kernels only (no CPU fallback)")
        P = self.packed(mel.device)
        c = P["compute"]
        dt = ops.torch_dtype(c)
        B, T, _ = mel.shape
        x = mel.to(dt).contiguous()

        def run(inp, p, epi, out, T_rows, **kw):
            return ops.conv1d(inp.view(B, T_rows, -1), p["w"], p["b"], cin=p["cin"], ks=p["ks"], pad=p["pad"],
                              compute=c, epilogue=epi, out=out.view(B, T_rows, -1), **kw)

        h = torch.empty(B, T, P["pre"]["w"].shape[0], device=mel.device, dtype=dt)
        run(x, P["pre"], L.EPI_BIAS_LRELU, h, T, act_slope=LRELU_SLOPE)
        nk = self.num_kernels
        for i, up in enumerate(P["ups"]):
            T2 = T * up["u"]
            C = up["cout"]
            xu = torch.empty(B, T2, C, device=mel.device, dtype=dt)      # ups output (residual of pair 0)
            last_stage = i == len(P["ups"]) - 1
            if i in P["pair"] and os.environ.get("FS2_VOC_PAIR", "1") != "0" and \
                    (C == 128 or os.environ.get("FS2_VOC_PAIR64", "1") != "0"):
                # one launch per dilation pair (leaky_relu of the pair input applied on chip)
                run(h, up, L.EPI_BIAS, xu, T)
                T = T2
                h = self._pair_stage(P["pair"][i], xu, 0.01 if last_stage else LRELU_SLOPE)
                continue
            a0 = torch.empty_like(xu)                                    # leaky_relu(xu): convs1 input of pair 0
            run(h, up, L.EPI_BIAS, xu, T, out2=a0.view(B, T, -1), out2_act=True, out2_slope=LRELU_SLOPE)
            T = T2
            if i in P["mrf"] and os.environ.get("FS2_VOC_MRF", "1") != "0":
                # the stage's 18 ResBlock convs, their average and the next leaky_relu in one launch
                wm, bm = P["mrf"][i]
                h = ops.hifigan_mrf(xu, a0, wm, bm, 0.01 if last_stage else LRELU_SLOPE)
                continue
            xs = torch.empty_like(xu)                                    # multi-receptive-field sum
            nxt = torch.empty_like(xu)                                   # leaky_relu(xs / nk): next stage's input
            xa, xb, aa, tt = (torch.empty_like(xu) for _ in range(4))
            for j in range(nk):
                pairs = P["rb"][i * nk + j]
                xp, ap = xu, a0
                for pi, (c1, c2) in enumerate(pairs):
                    run(ap, c1, L.EPI_BIAS_LRELU, tt, T, dilation=c1["dil"], act_slope=LRELU_SLOPE)
                    if pi < len(pairs) - 1:
                        xn = xa if xp is not xa else xb
                        run(tt, c2, L.EPI_RES_SUM, xn, T, residual=xp.view(B, T, -1), out2=aa.view(B, T, -1),
                            out2_act=True, out2_slope=LRELU_SLOPE)
                        xp, ap = xn, aa
                    else:  # last pair: fold into the running sum xs (in place), /nk at the last kernel
                        kw = dict(residual=xp.view(B, T, -1), residual2=xs.view(B, T, -1) if j > 0 else None)
                        if j == nk - 1:
                            kw.update(out_div=float(nk), out2=nxt.view(B, T, -1), out2_act=True,
                                      out2_slope=0.01 if last_stage else LRELU_SLOPE)
                        run(tt, c2, L.EPI_RES_SUM, xs, T, **kw)
            h = nxt
        if "post1" in P and h.dtype == torch.bfloat16 and T % 2 == 0 and os.environ.get("FS2_VOC_POST", "1") != "0":
            # conv_post + tanh as a streaming one-channel kernel (FS2_VOC_POST=0: the MFMA conv, A/B)
            return ops.hifigan_post(h.view(B, T, -1), *P["post1"])
        wav = torch.empty(B, T, 4, device=mel.device, dtype=torch.float32)
        run(h, P["post"], L.EPI_BIAS_TANH, wav, T, out_dtype=L.FS2_F32)
        return wav[..., 0]


def flops_per_frame(h=V1_CONFIG):
    """Algorithmic multiply-add FLOPs (x2) per mel frame of the generator (conv_pre, the
    transposed convs counted at their true K/u taps per output sample, the 3 x 6 ResBlock convs
    per stage, conv_post); V1: ~614 MFLOP per frame."""
    c = h["upsample_initial_channel"]
    f = 2 * h["num_mels"] * 7 * c
    spf = 1
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        cin, cout = c // 2 ** i, c // 2 ** (i + 1)
        spf *= u
        f += spf * 2 * cin * cout * (k // u)
        f += spf * sum(2 * cout * cout * rk * 2 * len(rd) for rk, rd in
                       zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"]))
    f += spf * 2 * (c // 2 ** len(h["upsample_rates"])) * 7
    return f


def get_vocoder(config, device, ckpt_dir="hifigan"):
    """utils/model.py:42-71, HiFi-GAN branch: Generator from <ckpt_dir>/config.json (V1 if absent),
    weights from <ckpt_dir>/generator_{LJSpeech,universal}.pth.tar["generator"] loaded with
    weights_only=True (the reference's files are Git-LFS-missing here: then a FileNotFoundError,
    as the reference raises), weight norm removed, eval, on ``device``."""
    name = config["vocoder"]["model"]
    speaker = config["vocoder"]["speaker"]
    if name != "HiFi-GAN":
        raise NotImplementedError(f"vocoder {name!r}: only HiFi-GAN is provided (MelGAN is a remote torch.hub fetch)")
    cfg_path = os.path.join(ckpt_dir, "config.json")
    h = V1_CONFIG
    if os.path.exists(cfg_path):
        with open(cfg_path) as f:
            h = json.load(f)
    vocoder = Generator(AttrDict(h))
    fname = {"LJSpeech": "generator_LJSpeech.pth.tar", "universal": "generator_universal.pth.tar"}[speaker]
    ckpt = torch.load(os.path.join(ckpt_dir, fname), map_location="cpu", weights_only=True)
    vocoder.load_state_dict(ckpt["generator"])
    vocoder.eval()
    vocoder.remove_weight_norm()
    return vocoder.to(device)


def vocoder_infer(mels, vocoder, model_config, preprocess_config, lengths=None):
    """utils/model.py:74-92 (HiFi-GAN branch): mels [B, n_mels, T] -> list of int16 waveforms,
    each cut to lengths[i] samples when given. The float -> int16 scaling runs on the device,
    so only 2 bytes per sample cross PCIe."""
    name = model_config["vocoder"]["model"]
    if name != "HiFi-GAN":
        raise NotImplementedError(f"vocoder {name!r}")
    with torch.no_grad():
        wavs = vocoder(mels).squeeze(1)
        wavs = (wavs * preprocess_config["preprocessing"]["audio"]["max_wav_value"]).to(torch.int16)
    wavs = [w for w in wavs.cpu().numpy()]
    if lengths is not None:
        for i in range(len(mels)):
            wavs[i] = wavs[i][: lengths[i]]
    return wavs
