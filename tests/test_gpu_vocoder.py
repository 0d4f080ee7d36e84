"""HiFi-GAN generator on the HIP conv kernels against the reference generator's outputs
(tests/golden/vocoder.npz) and the dilated / wide-tap conv tiles against F.conv1d.

Tolerances (stated here): fp32 mode (exact-f32 MFMA, only summation order differs) |wav - ref|
<= 2e-3 absolute (|wav| <= 0.77); bf16 mode (bf16 operands, f32 accumulation, bf16 activations
between the 67 convs) max |err| <= 0.08 and SNR >= 25 dB against the reference waveform.
Conv kernels: f32 2e-5, bf16 2.5e-2 relative to the output scale."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _common import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


@pytest.fixture(scope="module")
def gen():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from fs2amd.synth_weights import fill_vocoder
    from fs2amd.vocoder import V1_CONFIG, Generator

    g = Generator(V1_CONFIG)
    fill_vocoder(g, V1_CONFIG, seed=0)
    return g.to(DEV).eval()


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "vocoder.npz"))


def _snr_db(ref, got):
    return 10 * np.log10((ref ** 2).sum() / max(((ref - got) ** 2).sum(), 1e-30))


@pytest.mark.parametrize("case", ["cfg1", "mini2"])
def test_vocoder_fp32_matches_reference(gen, golden, case):
    mel = torch.from_numpy(golden[f"{case}__mel"]).to(DEV)
    with torch.no_grad():
        y = gen.set_precision("fp32")(mel)
    torch.cuda.synchronize()
    ref = golden[f"{case}__wav"]
    got = y.cpu().numpy()
    assert got.shape == ref.shape
    err = np.abs(got - ref).max()
    print(f"vocoder fp32 {case}: max|err| {err:.2e}, SNR {_snr_db(ref, got):.1f} dB")
    assert err <= 2e-3, err


@pytest.mark.parametrize("case", ["cfg1", "mini2"])
def test_vocoder_bf16_within_tolerance(gen, golden, case):
    mel = torch.from_numpy(golden[f"{case}__mel"]).to(DEV)
    with torch.no_grad():
        y = gen.set_precision("bf16")(mel)
    torch.cuda.synchronize()
    ref = golden[f"{case}__wav"]
    got = y.cpu().numpy()
    err, snr = np.abs(got - ref).max(), _snr_db(ref, got)
    print(f"vocoder bf16 {case}: max|err| {err:.2e}, SNR {snr:.1f} dB")
    assert err <= 0.08 and snr >= 25.0, (err, snr)
    gen.set_precision("fp32")


def test_vocoder_infer_int16(gen, golden):
    """utils/model.py:74-92: int16 waveforms, each cut to its length in samples."""
    from fs2amd.vocoder import vocoder_infer
    from fs2amd import config as C

    mel = torch.from_numpy(golden["mini2__mel"]).to(DEV)
    lengths = [200 * 256, 150 * 256]
    wavs = vocoder_infer(mel, gen.set_precision("fp32"), C.ESD_MODEL_CONFIG, C.ESD_PREPROCESS_CONFIG, lengths)
    ref = (golden["mini2__wav"][:, 0] * 32768.0).astype("int16")
    for w, r, n in zip(wavs, ref, lengths):
        assert w.dtype == np.int16 and w.shape == (n,)
        assert np.abs(w.astype(np.int32) - r[:n].astype(np.int32)).max() <= 80  # 2e-3 * 32768 + 1


@pytest.mark.parametrize("cin,n,k,d,compute", [(128, 128, 11, 5, 0), (64, 64, 7, 3, 0), (32, 32, 11, 5, 0),
                                               (32, 32, 3, 1, 1), (64, 64, 11, 5, 1), (256, 256, 7, 3, 1),
                                               (32, 4, 7, 1, 0)])
def test_dilated_conv_matches_torch(cin, n, k, d, compute):
    """The wide-tap tiles (dilation in the LDS halo, N = 4..256) vs F.conv1d, per-sequence zero
    padding, with the leaky-ReLU epilogue and the out2 activation."""
    from fs2amd import _lib as L, ops

    g = torch.Generator().manual_seed(k * 100 + d)
    B, T = 3, 301
    pad = (k * d - d) // 2
    x = torch.randn(B, T, cin, generator=g)
    w = torch.randn(n, cin, k, generator=g) / (cin * k) ** 0.5
    b = torch.randn(n, generator=g) * 0.1
    dt = torch.float32 if compute == 0 else torch.bfloat16
    xd = x.to(DEV, dt)
    out = torch.empty(B, T, n, device=DEV, dtype=dt)
    o2 = torch.empty(B, T, n, device=DEV, dtype=torch.float32)
    ops.conv1d(xd, ops.pack_conv_weight(w.to(DEV), compute), b.to(DEV), cin=cin, ks=k, pad=pad, compute=compute,
               epilogue=L.EPI_BIAS_LRELU, out=out, dilation=d, act_slope=0.1, out2=o2, out2_act=True, out2_slope=0.3)
    torch.cuda.synchronize()
    xr = x if compute == 0 else x.to(torch.bfloat16).float()
    wr = w if compute == 0 else w.to(torch.bfloat16).float()
    ref = F.leaky_relu(F.conv1d(xr.transpose(1, 2), wr, b, padding=pad, dilation=d).transpose(1, 2), 0.1)
    tol = 2e-5 if compute == 0 else 2.5e-2
    scale = float(ref.abs().max())
    assert float((out.float().cpu() - ref).abs().max()) <= tol * scale
    assert float((o2.cpu() - F.leaky_relu(out.float().cpu(), 0.3)).abs().max()) <= 1e-6 * scale + (0 if compute == 0 else 1e-2 * scale)


def test_res_sum_epilogue(gen):
    """EPI_RES_SUM: y = (conv + bias + residual + residual2) / div, residual2 aliasing out."""
    from fs2amd import _lib as L, ops

    g = torch.Generator().manual_seed(3)
    B, T, C, k = 2, 97, 64, 7
    x, r, acc = (torch.randn(B, T, C, generator=g) for _ in range(3))
    w = torch.randn(C, C, k, generator=g) / (C * k) ** 0.5
    b = torch.randn(C, generator=g) * 0.1
    out = acc.to(DEV).contiguous()
    ops.conv1d(x.to(DEV), ops.pack_conv_weight(w.to(DEV), 0), b.to(DEV), cin=C, ks=k, pad=3, compute=0,
               epilogue=L.EPI_RES_SUM, out=out, residual=r.to(DEV), residual2=out, out_div=3.0)
    ref = (F.conv1d(x.transpose(1, 2), w, b, padding=3).transpose(1, 2) + r + acc) / 3.0
    assert float((out.cpu() - ref).abs().max()) <= 2e-5 * float(ref.abs().max())


@pytest.mark.parametrize("C,T", [(32, 1100), (64, 600), (32, 256), (64, 77)])
def test_hifigan_mrf_fused_stage(gen, C, T):
    """fs2_hifigan_mrf (a stage's 3 ResBlock1 chains of 6 convs each, their average and the next
    leaky_relu in one launch; 256-sample tiles with a 64-sample halo, intermediates on chip)
    against a float64 statement of hifigan/models.py:20-45,152-158 on the same bf16 input and
    bf16-rounded weights, with the kernel's bf16 rounding points (each conv output and the running
    x stored as bf16; xs summed in f32): max |err| <= 3e-2 of the output scale, mean <= 2e-3. Tile
    edges and utterance edges (T not a multiple of 256, T < 256) included."""
    from fs2amd import ops

    g = torch.Generator().manual_seed(C + T)
    B = 3
    ws = [torch.randn(C, C, k, generator=g) / (C * k) ** 0.5 for k in (3, 7, 11) for _ in range(6)]
    bs = [0.05 * torch.randn(C, generator=g) for _ in range(18)]
    x = (0.5 * torch.randn(B, T, C, generator=g)).to(torch.bfloat16)
    xa = F.leaky_relu(x.float(), 0.1).to(torch.bfloat16)
    wp = torch.cat([ops.pack_wconv_tail(w.to(DEV)) for w in ws]).contiguous()
    bp = torch.cat(bs).to(DEV).contiguous()
    out = ops.hifigan_mrf(x.to(DEV), xa.to(DEV), wp, bp, 0.01)
    torch.cuda.synchronize()

    def conv(z, w, b, d):
        k = w.shape[-1]
        wq = w.to(torch.bfloat16).double()
        return F.conv1d(z.transpose(1, 2), wq, b.double(), dilation=d, padding=(k * d - d) // 2).transpose(1, 2)

    bf = lambda t: t.to(torch.bfloat16).double()
    xs = 0
    for j, k in enumerate((3, 7, 11)):
        cur = x.double()
        act = xa.double()
        for pi, d in enumerate((1, 3, 5)):
            t = bf(F.leaky_relu(conv(act, ws[6 * j + 2 * pi], bs[6 * j + 2 * pi], d), 0.1))
            v = conv(t, ws[6 * j + 2 * pi + 1], bs[6 * j + 2 * pi + 1], 1) + cur
            if pi < 2:
                cur, act = bf(v), bf(F.leaky_relu(v, 0.1))
            else:
                xs = xs + v
    ref = F.leaky_relu(xs / 3, 0.01)
    err = (out.double().cpu() - ref).abs()
    scale = float(ref.abs().max())
    assert float(err.max()) <= 3e-2 * scale and float(err.mean()) <= 2e-3 * scale, (float(err.max()), float(err.mean()), scale)


@pytest.mark.parametrize("C,T,k,d,mode", [(128, 1000, 11, 5, "plain"), (128, 300, 7, 3, "xs"), (128, 77, 3, 1, "last"),
                                          (128, 513, 11, 1, "last"), (128, 256, 3, 5, "plain"), (128, 40, 7, 5, "xs"),
                                          (64, 1500, 11, 5, "xs"), (64, 600, 7, 3, "last"), (64, 512, 3, 1, "plain"),
                                          (64, 90, 11, 5, "plain")])
def test_hifigan_pair_matches_f64(C, T, k, d, mode):
    """fs2_hifigan_pair (one ResBlock1 dilation pair at C = 128 / 64: lrelu, dilated conv, lrelu,
    conv, residual, optionally + the running sum and the stage's closing leaky_relu, one launch;
    256- / 512-sample tiles, the dilated conv's halo on chip) against a float64 statement of hifigan/models.py:34-45 on
    the same bf16 input and bf16-rounded weights, with the kernel's bf16 rounding points (lrelu(x)
    and the first conv's output stored as bf16): max |err| <= 2e-2 of the output scale, mean <=
    2e-3. Tile and utterance edges included (T not a multiple of 256, T < 256, dilation halo
    larger than the sequence)."""
    from fs2amd import ops

    g = torch.Generator().manual_seed(T + 10 * k + d + C)
    B = 3
    w1, w2 = (torch.randn(C, C, k, generator=g) / (C * k) ** 0.5 for _ in range(2))
    b1, b2 = (0.05 * torch.randn(C, generator=g) for _ in range(2))
    x = (0.5 * torch.randn(B, T, C, generator=g)).to(torch.bfloat16)
    xs = (0.5 * torch.randn(B, T, C, generator=g)).to(torch.bfloat16)
    kw = {}
    if mode != "plain":
        kw["xs"] = xs.to(DEV)
    if mode == "last":
        kw.update(out_scale=1.0 / 3, out_slope=0.01, out_act=True)
    out = ops.hifigan_pair(x.to(DEV), ops.pack_wconv_tail(w1.to(DEV)), b1.to(DEV), ops.pack_wconv_tail(w2.to(DEV)),
                           b2.to(DEV), k, d, **kw)
    torch.cuda.synchronize()

    def conv(z, w, b, dd):
        return F.conv1d(z.transpose(1, 2), w.to(torch.bfloat16).double(), b.double(), dilation=dd,
                        padding=(k * dd - dd) // 2).transpose(1, 2)

    bf = lambda t: t.to(torch.bfloat16).double()
    a = bf(F.leaky_relu(x.double(), 0.1))
    t = bf(F.leaky_relu(conv(a, w1, b1, d), 0.1))
    y = conv(t, w2, b2, 1) + x.double()
    if mode != "plain":
        y = y + xs.double()
    ref = F.leaky_relu(y / 3, 0.01) if mode == "last" else y
    err = (out.double().cpu() - ref).abs()
    scale = float(ref.abs().max())
    assert float(err.max()) <= 2e-2 * scale and float(err.mean()) <= 2e-3 * scale, (float(err.max()), float(err.mean()), scale)


def test_hifigan_pair64_stage_matches_mrf(gen):
    """The 64-channel stage on fs2_hifigan_pair (9 pair launches, the default) against the same
    stage as one fs2_hifigan_mrf launch (FS2_VOC_PAIR64=0): same waveform within bf16 noise."""
    g = torch.Generator().manual_seed(6)
    mel = (torch.randn(2, 80, 41, generator=g) - 4.0).to(DEV)
    gen.set_precision("bf16")
    try:
        assert 2 in gen.packed(torch.device(DEV))["pair"]  # the 64-channel stage
        with torch.no_grad():
            y1 = gen(mel).float().cpu()
            os.environ["FS2_VOC_PAIR64"] = "0"
            y0 = gen(mel).float().cpu()
    finally:
        os.environ.pop("FS2_VOC_PAIR64", None)
        gen.set_precision("fp32")
    snr = _snr_db(y0.numpy(), y1.numpy())
    assert snr >= 30.0, snr


def test_hifigan_pair_stage_matches_per_conv_path(gen):
    """The 128-channel stage on fs2_hifigan_pair (9 launches) against the same stage on the
    per-conv fs2_conv1d path (FS2_VOC_PAIR=0, 18 launches): same waveform within bf16 noise."""
    from fs2amd import _lib as L

    g = torch.Generator().manual_seed(5)
    mel = (torch.randn(2, 80, 57, generator=g) - 4.0).to(DEV)
    gen.set_precision("bf16")
    try:
        assert 1 in gen.packed(torch.device(DEV))["pair"]  # the 128-channel stage
        with torch.no_grad():
            y1 = gen(mel).float().cpu()
            os.environ["FS2_VOC_PAIR"] = "0"
            y0 = gen(mel).float().cpu()
    finally:
        os.environ.pop("FS2_VOC_PAIR", None)
        gen.set_precision("fp32")
    snr = _snr_db(y0.numpy(), y1.numpy())
    assert snr >= 30.0, snr


@pytest.mark.parametrize("B,T", [(3, 1024), (2, 600), (1, 514), (4, 6), (2, 130050)])
def test_hifigan_post_matches_f64(B, T):
    """fs2_hifigan_post (conv_post 32 -> 1, k = 7, pad 3, + tanh; hifigan/models.py:145,159-162) as
    the streaming one-channel kernel against a float64 statement on the same bf16 input and the
    bf16-rounded weights (the kernel's operand precision: v_dot2c_f32_bf16, f32 accumulation of 224
    products): max |err| <= 2e-5. Tile edges (T not a multiple of 512, T < 512, the 3-sample halo
    at both utterance ends) and the cfg2-sized per-utterance length (130,050 samples) included."""
    from fs2amd import ops

    g = torch.Generator().manual_seed(T + B)
    w = torch.randn(1, 32, 7, generator=g) / (32 * 7) ** 0.5
    bias = float(0.1 * torch.randn(1, generator=g))
    x = (0.7 * torch.randn(B, T, 32, generator=g)).to(torch.bfloat16)
    wt = w[0].t().contiguous().to(torch.bfloat16)
    out = ops.hifigan_post(x.to(DEV), wt.to(DEV), bias)
    torch.cuda.synchronize()
    ref = torch.tanh(F.conv1d(x.double().transpose(1, 2), wt.double().t()[None], torch.tensor([bias], dtype=torch.float64),
                              padding=3))[:, 0]
    err = (out.cpu().double() - ref).abs()
    assert out.shape == (B, T) and float(err.max()) <= 2e-5, float(err.max())


def test_vocoder_post_kernel_equals_mfma_path(gen, golden):
    """The bf16 generator with conv_post on fs2_hifigan_post equals the same generator with the
    MFMA conv_post (FS2_VOC_POST=0) within the two summation orders' f32 rounding (the stages
    before conv_post are the same launches, so their outputs are bit-identical)."""
    mel = torch.from_numpy(golden["mini2__mel"]).to(DEV)  # [B, n_mels, T]
    gen.set_precision("bf16")
    x = mel.transpose(1, 2).contiguous()
    with torch.no_grad():
        a = gen.forward_btc(x).clone()
        os.environ["FS2_VOC_POST"] = "0"
        try:
            b = gen.forward_btc(x).clone()
        finally:
            del os.environ["FS2_VOC_POST"]
    torch.cuda.synchronize()
    gen.set_precision("fp32")
    assert a.shape == b.shape and float((a - b).abs().max()) <= 1e-4, float((a - b).abs().max())
