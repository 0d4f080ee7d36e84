"""Per-kernel parity on the GPU, through the C ABI (fs2amd.ops -> libfs2hip.so).

Each HIP kernel is compared with a plain PyTorch fp32 CPU statement of the same op
(the reference's own ops: F.conv1d / F.layer_norm / bmm-softmax-bmm / bucketize) or,
for the LengthRegulator, with the oracle (bit-exact: it is index and copy work).
Tolerances (stated per test): f32 compute 2e-5 relative to the output scale (MFMA f32
is an exact f32 FMA chain; only the summation order differs), bf16 compute 2e-2.
"""
import ctypes
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from fs2amd import ops as o
    return o


def _L():
    from fs2amd import _lib
    return _lib


def _tol(compute):
    return 2e-5 if compute == 0 else 2.5e-2


def _ref_conv(x, w, b, pad):
    return F.conv1d(x.transpose(1, 2), w, b, padding=pad).transpose(1, 2)


def _rel_err(got, ref):
    return float((got.float().cpu() - ref).abs().max() / (ref.abs().max() + 1e-6))


@pytest.mark.parametrize("compute", [0, 1])
@pytest.mark.parametrize("B,T,Cin,N,KS", [(2, 37, 256, 768, 1), (3, 50, 256, 1024, 9), (2, 29, 1024, 256, 1),
                                          (1, 130, 80, 512, 5), (2, 70, 512, 80, 5), (4, 9, 256, 256, 3),
                                          # large shapes (bf16: the phased 256x256 kernel when FS2_CONV_PHASED=1)
                                          (24, 513, 256, 1024, 9), (48, 510, 512, 512, 5)])
def test_conv1d_bias_relu_tanh(ops, compute, B, T, Cin, N, KS):
    L = _L()
    g = torch.Generator().manual_seed(B * 1000 + T + N)
    x = torch.randn(B, T, Cin, generator=g)
    w = torch.randn(N, Cin, KS, generator=g) / np.sqrt(Cin * KS)
    b = torch.randn(N, generator=g) * 0.1
    pad = (KS - 1) // 2
    dt = torch.float32 if compute == 0 else torch.bfloat16
    xd = x.to(DEV, dt)
    xr = xd.float().cpu()
    wp = ops.pack_conv_weight(w.to(DEV), compute)
    wr = wp.float().cpu()[:, :, :Cin].permute(0, 2, 1)
    ref = _ref_conv(xr, wr, b, pad)
    for epi, fn in ((L.EPI_BIAS, lambda v: v), (L.EPI_BIAS_RELU, torch.relu), (L.EPI_BIAS_TANH, torch.tanh)):
        out = ops.conv1d(xd, wp, b.to(DEV), cin=Cin, ks=KS, pad=pad, compute=compute, epilogue=epi,
                         out_dtype=L.FS2_F32)
        torch.cuda.synchronize()
        assert _rel_err(out, fn(ref)) < _tol(compute), (epi, _rel_err(out, fn(ref)))


@pytest.mark.parametrize("compute", [0, 1])
def test_conv1d_f32_input_bf16_compute_and_residual(ops, compute):
    """PostNet first/last layer shapes: f32 mel in, f32 residual out."""
    L = _L()
    g = torch.Generator().manual_seed(3)
    B, T = 3, 77
    mel = torch.randn(B, T, 80, generator=g)
    w = torch.randn(80, 512, 5, generator=g) / np.sqrt(512 * 5)
    b = torch.randn(80, generator=g) * 0.1
    h = torch.randn(B, T, 512, generator=g)
    dt = torch.float32 if compute == 0 else torch.bfloat16
    wp = ops.pack_conv_weight(w.to(DEV), compute)
    wr = wp.float().cpu()[:, :, :512].permute(0, 2, 1)
    hd = h.to(DEV, dt)
    out = ops.conv1d(hd, wp, b.to(DEV), cin=512, ks=5, pad=2, compute=compute, epilogue=L.EPI_BIAS_RES,
                     out_dtype=L.FS2_F32, residual=mel.to(DEV))
    ref = _ref_conv(hd.float().cpu(), wr, b, 2) + mel
    torch.cuda.synchronize()
    assert _rel_err(out, ref) < _tol(compute)
    # f32 input into the bf16-compute loader (conv0 of the PostNet reads the f32 mel)
    w0 = torch.randn(512, 80, 5, generator=g) / np.sqrt(400)
    wp0 = ops.pack_conv_weight(w0.to(DEV), compute)
    out0 = ops.conv1d(mel.to(DEV), wp0, None, cin=80, ks=5, pad=2, compute=compute, epilogue=L.EPI_BIAS,
                      out_dtype=L.FS2_F32)
    xin = mel.to(dt).float()
    ref0 = _ref_conv(xin, wp0.float().cpu()[:, :, :80].permute(0, 2, 1), None, 2)
    torch.cuda.synchronize()
    assert _rel_err(out0, ref0) < _tol(compute)


@pytest.mark.parametrize("B,T", [(3, 77), (64, 430)])
def test_conv1d_bf16_out2_copy(ops, B, T):
    """Elementwise epilogue with out2: f32 output + its bf16 copy (mel_linear -> PostNet). The copy
    is bit-equal to bf16(out), and PostNet's first conv on the copy equals the conv on the f32 mel
    (the bf16 GEMM rounds f32 inputs the same way)."""
    L = _L()
    g = torch.Generator().manual_seed(B + T)
    x = torch.randn(B, T, 256, generator=g).to(DEV, torch.bfloat16)
    w = torch.randn(80, 256, 1, generator=g) / 16
    b = torch.randn(80, generator=g) * 0.1
    wp = ops.pack_conv_weight(w.to(DEV), L.FS2_BF16)
    cp = torch.empty(B, T, 80, device=DEV, dtype=torch.bfloat16)
    mel = ops.conv1d(x, wp, b.to(DEV), cin=256, ks=1, pad=0, compute=L.FS2_BF16, epilogue=L.EPI_BIAS,
                     out_dtype=L.FS2_F32, out2=cp)
    torch.cuda.synchronize()
    assert torch.equal(cp, mel.to(torch.bfloat16))
    w0 = torch.randn(512, 80, 5, generator=g) / np.sqrt(400)
    wp0 = ops.pack_conv_weight(w0.to(DEV), L.FS2_BF16)
    b0 = (torch.randn(512, generator=g) * 0.1).to(DEV)
    with ops.splitk_enabled(False):
        ya = ops.conv1d(mel, wp0, b0, cin=80, ks=5, pad=2, compute=L.FS2_BF16, epilogue=L.EPI_BIAS_TANH,
                        out_dtype=L.FS2_BF16)
        yb = ops.conv1d(cp, wp0, b0, cin=80, ks=5, pad=2, compute=L.FS2_BF16, epilogue=L.EPI_BIAS_TANH,
                        out_dtype=L.FS2_BF16)
    torch.cuda.synchronize()
    assert (ya.float() - yb.float()).abs().max().item() <= 1e-2, (ya.float() - yb.float()).abs().max().item()


@pytest.mark.parametrize("compute", [0, 1])
@pytest.mark.parametrize("B,T,Cin", [(5, 41, 256), (64, 401, 1024)])  # the 2nd routes to the 8-wave 128x256 tile
def test_conv1d_res_ln_mask_addvec(ops, compute, B, T, Cin):
    L = _L()
    g = torch.Generator().manual_seed(5)
    C = 256
    x = torch.randn(B, T, Cin, generator=g)
    res = torch.randn(B, T, C, generator=g)
    w = torch.randn(C, Cin, 1, generator=g) / np.sqrt(Cin)
    b = torch.randn(C, generator=g) * 0.1
    gam, bet = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    lens = torch.tensor([41, 1, 0, 17, 40]) if B == 5 else torch.randint(0, T + 1, (B,), generator=g)
    av1, av2 = torch.randn(B, C, generator=g), torch.randn(B, C, generator=g)
    dt = torch.float32 if compute == 0 else torch.bfloat16
    wp = ops.pack_conv_weight(w.to(DEV), compute)
    xd, rd = x.to(DEV, dt), res.to(DEV, dt)
    out = ops.conv1d(xd, wp, b.to(DEV), cin=Cin, ks=1, pad=0, compute=compute, epilogue=L.EPI_RES_LN,
                     out_dtype=L.FS2_F32, residual=rd, ln=(gam.to(DEV), bet.to(DEV), 1e-5), lens=lens.to(DEV),
                     addvec1=av1.to(DEV), addvec2=av2.to(DEV))
    pre = _ref_conv(xd.float().cpu(), wp.float().cpu()[:, :, :Cin].permute(0, 2, 1), b, 0) + rd.float().cpu()
    y = F.layer_norm(pre, (C,), gam, bet)
    mask = torch.arange(T)[None, :] >= lens[:, None]
    y = y.masked_fill(mask.unsqueeze(-1), 0) + av1[:, None, :] + av2[:, None, :]
    torch.cuda.synchronize()
    assert _rel_err(out, y) < _tol(compute) * 4


def test_conv1d_variance_predictor_f32(ops):
    """conv k3 + ReLU + LN, then conv k3 + ReLU + LN + Linear(256->1) + mask, exact-f32 MFMA."""
    L = _L()
    g = torch.Generator().manual_seed(9)
    B, T, C = 3, 23, 256
    x = torch.randn(B, T, C, generator=g)
    w1 = torch.randn(C, C, 3, generator=g) / np.sqrt(3 * C)
    w2 = torch.randn(C, C, 3, generator=g) / np.sqrt(3 * C)
    b1, b2 = torch.randn(C, generator=g) * 0.1, torch.randn(C, generator=g) * 0.1
    g1, be1 = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    g2, be2 = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    lw, lb = torch.randn(C, generator=g) / 16, 0.3
    lens = torch.tensor([23, 5, 11])
    for xin in (x.to(DEV), x.to(DEV, torch.bfloat16)):
        h = ops.conv1d(xin, ops.pack_conv_weight(w1.to(DEV), 0), b1.to(DEV), cin=C, ks=3, pad=1, compute=0,
                       epilogue=L.EPI_RELU_LN, out_dtype=0, ln=(g1.to(DEV), be1.to(DEV), 1e-5))
        o = ops.conv1d(h, ops.pack_conv_weight(w2.to(DEV), 0), b2.to(DEV), cin=C, ks=3, pad=1, compute=0,
                       epilogue=L.EPI_RELU_LN_DOT, ln=(g2.to(DEV), be2.to(DEV), 1e-5), lens=lens.to(DEV),
                       dot=(lw.to(DEV), lb))
        xr = xin.float().cpu()
        hr = F.layer_norm(torch.relu(_ref_conv(xr, w1, b1, 1)), (C,), g1, be1)
        orf = F.layer_norm(torch.relu(_ref_conv(hr, w2, b2, 1)), (C,), g2, be2) @ lw + lb
        orf = orf.masked_fill(torch.arange(T)[None] >= lens[:, None], 0.0)
        torch.cuda.synchronize()
        assert o.shape == (B, T)
        assert float((o.cpu() - orf).abs().max()) < 2e-4


def _ref_attention(qkv, lens, H, dk):
    B, T, _ = qkv.shape
    q, k, v = qkv[..., :H * dk], qkv[..., H * dk:2 * H * dk], qkv[..., 2 * H * dk:]
    split = lambda t: t.view(B, T, H, dk).permute(2, 0, 1, 3).reshape(H * B, T, dk)
    q, k, v = split(q), split(k), split(v)
    mask = (torch.arange(T)[None, :] >= lens[:, None]).unsqueeze(1).expand(-1, T, -1).repeat(H, 1, 1)
    a = torch.bmm(q, k.transpose(1, 2)) / np.power(dk, 0.5)
    a = torch.softmax(a.masked_fill(mask, -np.inf), dim=2)
    o = torch.bmm(a, v).view(H, B, T, dk).permute(1, 2, 0, 3).reshape(B, T, H * dk)
    return o


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T", [(3, 70), (2, 431), (1, 5)])
def test_attention(ops, dtype, B, T):
    g = torch.Generator().manual_seed(T)
    H, dk = 2, 128
    qkv = torch.randn(B, T, 3 * H * dk, generator=g)
    lens = torch.randint(1, T + 1, (B,), generator=g)
    lens[0] = T
    qd = qkv.to(DEV, dtype)
    out = ops.attention(qd, lens.to(DEV), H, dk, float(np.power(dk, 0.5)))
    ref = _ref_attention(qd.float().cpu(), lens, H, dk)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert _rel_err(out, ref) < tol


def test_length_regulate_bit_exact_vs_oracle_cases(ops, golden_dir):
    from oracle import fs2_oracle as O

    z = np.load(os.path.join(golden_dir, "lr_cases.npz"))
    names = sorted({k.split("__")[0] for k in z.files})
    for n in names:
        x = torch.from_numpy(z[f"{n}__x"])
        d = torch.from_numpy(z[f"{n}__d"])
        ml = int(z[f"{n}__max_len"])
        max_len = None if ml < 0 else ml
        # D=5 in the reference fixture; the kernel needs D % 8 == 0 -> pad channels, compare the first 5
        xp = F.pad(x, (0, 3))
        out, mel_len = ops.length_regulate(xp.to(DEV), d.to(DEV), max_len)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out[..., :5].cpu().numpy(), z[f"{n}__out"], err_msg=n)
        np.testing.assert_array_equal(mel_len.cpu().numpy(), z[f"{n}__mel_len"], err_msg=n)
        ref_out, ref_len = O.length_regulate(x, d, max_len)
        np.testing.assert_array_equal(out[..., :5].cpu().numpy(), ref_out.numpy(), err_msg=n)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_length_regulate_cfg4_index_map_and_values(ops, golden_dir, dtype):
    """LR stress shape (B=256, L up to 160, T_max ~1000): index map bit-exact vs the reference capture,
    values bit-exact (pure copy) vs the oracle's C restatement, PE fusion exact in f32."""
    z = np.load(os.path.join(golden_dir, "cfg4_lr_index.npz"))
    d = torch.from_numpy(z["d"].astype(np.int64))
    T = int(z["max_mel_len"])
    B, Lx = d.shape
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, Lx, 256, generator=g).to(dtype)
    cum, mel_len, _ = ops.lr_durations(d.to(DEV))
    out, im = ops.lr_expand(x.to(DEV), cum, mel_len, T, index_map=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(im.cpu().numpy(), z["index_map"].astype(np.int32))
    np.testing.assert_array_equal(mel_len.cpu().numpy(), z["mel_len"])
    imt = torch.from_numpy(z["index_map"].astype(np.int64))
    ref = torch.where((imt >= 0)[..., None], x[torch.arange(B)[:, None], imt.clamp(min=0)], torch.zeros((), dtype=dtype))
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("crop", [0, 37])
def test_length_regulate_one_launch_cfg4(ops, golden_dir, dtype, crop):
    """fs2_length_regulate's one launch (lr_pad_kernel: per-workgroup scan, phoneme ranges painted
    into the frame map, 128 frames per workgroup at this size) at the LR stress shape: index map,
    mel_len and the padded values bit-exact against the reference capture, also with max_len
    cropping the output below max(mel_len) (mel_len stays the uncropped total, modules.py:180)."""
    z = np.load(os.path.join(golden_dir, "cfg4_lr_index.npz"))
    d = torch.from_numpy(z["d"].astype(np.int64))
    T = int(z["max_mel_len"]) - crop
    B, Lx = d.shape
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B, Lx, 256, generator=g).to(dtype)
    out, mel_len, im = ops.length_regulate(x.to(DEV), d.to(DEV), T, return_index_map=True)
    torch.cuda.synchronize()
    imt = torch.from_numpy(z["index_map"].astype(np.int64))[:, :T]
    np.testing.assert_array_equal(im.cpu().numpy(), imt.numpy().astype(np.int32))
    np.testing.assert_array_equal(mel_len.cpu().numpy(), z["mel_len"])
    ref = torch.where((imt >= 0)[..., None], x[torch.arange(B)[:, None], imt.clamp(min=0)], torch.zeros((), dtype=dtype))
    assert torch.equal(out.cpu(), ref)


def test_length_regulate_logpred_rounding(ops):
    """duration = clamp(round(exp(logd) - 1) * d_control, min=0) with half-to-even rounding."""
    from oracle import fs2_oracle as O

    g = torch.Generator().manual_seed(4)
    logd = torch.randn(6, 33, generator=g) * 1.2 + 1.0
    logd[0, :4] = torch.log(torch.tensor([1.5, 2.5, 3.5, 0.5]) + 1)  # exact-ish ties
    for dc in (0.8, 1.0, 1.3):
        cum, mel_len, dr = ops.lr_durations(logd.to(DEV), logpred=True, d_control=dc)
        ref = torch.clamp(torch.round(torch.exp(logd) - 1) * dc, min=0)
        torch.cuda.synchronize()
        assert torch.equal(dr.cpu(), ref), dc
        im, ml = O.length_regulate_index_map(ref, None)
        np.testing.assert_array_equal(mel_len.cpu().numpy(), ml.numpy())


def test_variance_embed(ops):
    g = torch.Generator().manual_seed(2)
    M, D = 300, 256
    bins = torch.linspace(-2.0, 8.0, 255)
    table = torch.randn(256, D, generator=g)
    x = torch.randn(M, D, generator=g)
    pred = torch.randn(M, generator=g) * 4
    pred[:5] = torch.tensor([-5.0, 8.0, 9.0, bins[10].item(), bins[200].item()])
    for target in (None, torch.randn(M, generator=g) * 3):
        xd, pd = x.clone().to(DEV), pred.clone().to(DEV)
        ops.variance_embed(xd, pd, None if target is None else target.to(DEV), 1.2, bins.to(DEV), table.to(DEV))
        v = pred * 1.2 if target is None else target
        ref = x + F.embedding(torch.bucketize(v, bins), table)
        torch.cuda.synchronize()
        assert torch.equal(xd.cpu(), ref)
        if target is None:
            assert torch.equal(pd.cpu(), pred * 1.2)


def test_embed_pe_and_cond(ops):
    g = torch.Generator().manual_seed(8)
    table = torch.randn(139, 256, generator=g)
    pe = torch.randn(2001, 256, generator=g)
    tok = torch.randint(0, 139, (4, 19), generator=g)
    out = ops.embed_pe(tok.to(DEV), table.to(DEV), pe.to(DEV), 0)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), F.embedding(tok, table) + pe[:19][None])
    spk_t = torch.randn(10, 256, generator=g)
    emo_t, aro_t, val_t = torch.randn(5, 128, generator=g), torch.randn(4, 64, generator=g), torch.randn(5, 64, generator=g)
    lw, lb = torch.randn(256, 256, generator=g) / 16, torch.randn(256, generator=g) * 0.1
    s, e, a, v = (torch.tensor([3, 9, 0]), torch.tensor([4, 0, 2]), torch.tensor([1, 3, 0]), torch.tensor([0, 4, 2]))
    so, eo = ops.cond_vectors(s.to(DEV), spk_t.to(DEV), e.to(DEV), a.to(DEV), v.to(DEV), emo_t.to(DEV),
                              aro_t.to(DEV), val_t.to(DEV), lw.to(DEV), lb.to(DEV), 256)
    torch.cuda.synchronize()
    assert torch.equal(so.cpu(), spk_t[s])
    ref = torch.relu(F.linear(torch.cat([emo_t[e], aro_t[a], val_t[v]], -1), lw, lb))
    assert float((eo.cpu() - ref).abs().max()) < 1e-5


def test_embed_pe_out_of_vocab_is_loud(ops):
    """The reference's nn.Embedding raises on an id outside the table; here the row is NaN and
    the next check raises IndexError (never a silent clamp to a valid row)."""
    g = torch.Generator().manual_seed(9)
    table, pe = torch.randn(139, 256, generator=g), torch.randn(2001, 256, generator=g)
    tok = torch.randint(0, 139, (2, 7), generator=g)
    tok[1, 3], tok[0, 0] = 139, -1
    out = ops.embed_pe(tok.to(DEV), table.to(DEV), pe.to(DEV), 0).cpu()
    assert torch.isnan(out[1, 3]).all() and torch.isnan(out[0, 0]).all()
    ok = torch.ones(2, 7, dtype=torch.bool)
    ok[1, 3] = ok[0, 0] = False
    assert torch.equal(out[ok], (F.embedding(tok.clamp(0, 138), table) + pe[:7][None])[ok])
    with pytest.raises(IndexError):
        ops.raise_if_bad_ids(torch.device(DEV))
    ops.raise_if_bad_ids(torch.device(DEV))  # the count was consumed


def test_single_hip_runtime_loaded(ops):
    """Our library must share torch's HIP runtime (one libamdhip64 in the process)."""
    maps = open("/proc/self/maps").read()
    hip = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert len(hip) == 1, hip
    assert any("libfs2hip.so" in line for line in maps.splitlines())


def test_length_masks(ops):
    lens = torch.tensor([0, 3, 7, 9, 2])
    m = ops.length_mask(lens.to(DEV), 7)
    torch.cuda.synchronize()
    assert torch.equal(m.cpu(), torch.arange(7)[None, :] >= lens[:, None])


def test_phased_conv_kernel_parity():
    """The phased 256x256 conv kernel (FS2_CONV_PHASED=1) against a float64 conv of the same
    bf16 operands (f32 accumulation: 1e-3 of max), padded and packed rows, a channel tail
    (Cin=80), and a race screen: 20 repeated launches must be bit-identical. Child process
    (the switch is read once per process)."""
    import subprocess
    import sys

    code = r"""
import sys, torch, numpy as np, torch.nn.functional as F
sys.path.insert(0, 'expressive-fastspeech2-mandarin_amd')
from fs2amd import ops, _lib as L
g = torch.Generator().manual_seed(1)
for (B, T, Cin, N, KS, packed) in [(24, 513, 256, 1024, 9, False), (48, 510, 512, 512, 5, False),
                                   (40, 333, 80, 512, 5, False), (30, 431, 256, 1024, 9, True)]:
    lens = torch.randint(0, T + 1, (B,), generator=g)
    lens[0] = T
    lens[1] = 0
    valid = (torch.arange(T)[None, :] < lens[:, None])[..., None]
    x = torch.randn(B, T, Cin, generator=g)
    if packed:
        x = x * valid
    x = x.to(torch.bfloat16)
    w = (torch.randn(N, Cin, KS, generator=g) / np.sqrt(Cin * KS))
    b = (torch.randn(N, generator=g) * 0.1)
    wp = ops.pack_conv_weight(w.cuda(), L.FS2_BF16)
    kw = dict(cin=Cin, ks=KS, pad=(KS - 1) // 2, compute=L.FS2_BF16, epilogue=L.EPI_BIAS_RELU, out_dtype=L.FS2_F32)
    ref = torch.relu(F.conv1d(x.double().transpose(1, 2), wp.double().cpu()[:, :, :Cin].permute(0, 2, 1),
                              b.double(), padding=(KS - 1) // 2).transpose(1, 2))
    if packed:
        lay = ops.SeqLayout(lens.cuda(), T)
        rm = lay.rowmap.long().cpu()
        xp = torch.zeros(B * T, Cin, dtype=torch.bfloat16)
        ok = rm >= 0
        xp[rm[ok]] = x.reshape(-1, Cin)[ok]
        run = lambda: ops.conv1d(xp.cuda(), wp, b.cuda(), layout=lay, **kw)
        R = int(lay.cu[-1])
        pick = lambda o: o[:R].cpu().double()
        ref = ref.reshape(-1, N)[valid.reshape(-1)]
    else:
        xc = x.cuda()
        run = lambda: ops.conv1d(xc, wp, b.cuda(), **kw)
        pick = lambda o: o.cpu().double()
    first = run()
    err = float((pick(first) - ref).abs().max() / ref.abs().max())
    assert err < 1e-3, (B, T, Cin, N, KS, packed, err)
    for _ in range(20):
        assert torch.equal(run(), first), ("nondeterministic", B, T, Cin, N, KS, packed)
print('ok')
"""
    env = dict(os.environ, FS2_CONV_PHASED="1")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=repo, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_split_precision_variance_predictor_matches_f32():
    """VariancePredictor in bf16x3 split precision (bf16 MFMA, channel-block map, two-plane LN
    output) vs exact-f32 MFMA on the same bf16 input: |d| <= 2e-4 + 2e-4 |y| (the split keeps
    ~16 mantissa bits of weights and hidden activations)."""
    from fs2amd.runtime import variance_predictor
    from fs2amd.model import FastSpeech2
    from fs2amd.synth_weights import fill_module
    from _common import configs

    pc, mc, _ = configs()
    m = FastSpeech2(pc, mc)
    fill_module(m, seed=0)
    m = m.to("cuda").eval()
    P32 = m.set_precision("bf16", "fp32").packed("cuda")
    P3 = m.set_precision("bf16", "bf16x3").packed("cuda")
    g = torch.Generator().manual_seed(4)
    B, L = 16, 57
    x = torch.randn(B, L, 256, generator=g).to("cuda", torch.bfloat16)
    lens = torch.randint(1, L + 1, (B,), generator=g).to("cuda")
    for k in ("duration", "pitch", "energy"):
        a = variance_predictor(P32.vp[k], x, lens)
        b = variance_predictor(P3.vp[k], x, lens)
        torch.cuda.synchronize()
        err = (a - b).abs()
        assert bool((err <= 2e-4 + 2e-4 * a.abs()).all()), (k, float(err.max()))


@pytest.mark.parametrize("B,L", [(16, 57), (64, 64), (3, 5)])
def test_vp_columns_match_f32_and_embed(B, L):
    """Column-split bf16x3 VariancePredictors (runtime.variance_predictors: conv1 over duration +
    pitch's stacked columns, fs2_vp_norm, grouped conv2, fs2_vp_head) vs each predictor on
    exact-f32 MFMA: |d| <= 2e-4 + 2e-4 |y| as the split test above. The head's embedding add:
    x += table[bucketize(v)] with v = pred * control (pred scaled in place) or the target (pred
    kept), exact against torch on the kernel's own predictions (modules.py:80-100,117-126)."""
    from fs2amd.runtime import variance_predictor, variance_predictors
    from fs2amd.model import FastSpeech2
    from fs2amd.synth_weights import fill_module
    from _common import configs

    pc, mc, _ = configs()
    m = FastSpeech2(pc, mc)
    fill_module(m, seed=0)
    m = m.to("cuda").eval()
    P32 = m.set_precision("bf16", "fp32").packed("cuda")
    P3 = m.set_precision("bf16", "bf16x3").packed("cuda")
    assert P3.vpcols is not None
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, L, 256, generator=g).to("cuda", torch.bfloat16)
    lens = torch.randint(1, L + 1, (B,), generator=g).to("cuda")
    dp = variance_predictors(P3.vpcols.dp, x, lens)
    en = variance_predictors(P3.vpcols.energy, x, lens)
    assert dp.shape == (2, B, L) and en.shape == (1, B, L)
    for got, k in ((dp[0], "duration"), (dp[1], "pitch"), (en[0], "energy")):
        ref = variance_predictor(P32.vp[k], x, lens)
        err = (ref - got).abs()
        assert bool((err <= 2e-4 + 2e-4 * ref.abs()).all()), (k, float(err.max()))
        pad = torch.arange(L, device="cuda")[None, :] >= lens[:, None]
        assert bool((got[pad] == 0).all())
    bins, table = P3.bins["pitch"], P3.var_table["pitch"]

    def embedded(v):
        idx = torch.bucketize(v, bins)
        return (x.float() + table[idx]).to(torch.bfloat16)

    x2 = x.clone()
    p2 = variance_predictors(P3.vpcols.dp, x2, lens, embed=(1, x2, None, 1.3, bins, table))
    assert torch.equal(p2[0], dp[0]) and torch.equal(p2[1], dp[1] * 1.3)
    assert torch.equal(x2, embedded(p2[1]))
    tgt = torch.randn(B, L, generator=g).to("cuda")
    x3 = x.clone()
    p3 = variance_predictors(P3.vpcols.dp, x3, lens, embed=(1, x3, tgt, 1.0, bins, table))
    assert torch.equal(p3[1], dp[1]) and torch.equal(x3, embedded(tgt))


@pytest.mark.parametrize("B,L", [(64, 64), (3, 45), (5, 17), (2, 1), (7, 160), (1, 33)])
def test_vp_fused_matches_f32_and_columns(B, L):
    """fs2_vp_fused (one launch per predictor set: conv1 + LN1 + conv2 + LN2 + Linear + mask, bf16x3,
    32-row tiles with the conv halo recomputed; ragged utterance / tile boundaries: L = 45, 17, 1,
    160, 33) vs each predictor on exact-f32 MFMA within |d| <= 2e-4 + 2e-4 |y| (the column-split
    form's bound), padded positions exactly 0. The embedding group's x_out = x + table[bucketize(v)]
    is exact against torch on the kernel's own predictions: v = pred * control (pred scaled) or the
    target (pred kept); x itself is not modified."""
    from fs2amd import ops
    from fs2amd.runtime import variance_predictor, variance_predictors
    from fs2amd.model import FastSpeech2
    from fs2amd.synth_weights import fill_module
    from _common import configs

    pc, mc, _ = configs()
    m = FastSpeech2(pc, mc)
    fill_module(m, seed=0)
    m = m.to("cuda").eval()
    P32 = m.set_precision("bf16", "fp32").packed("cuda")
    P3 = m.set_precision("bf16", "bf16x3").packed("cuda")
    assert P3.vpfused is not None
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, L, 256, generator=g).to("cuda", torch.bfloat16)
    lens = torch.randint(1, L + 1, (B,), generator=g).to("cuda")
    x0 = x.clone()
    dp, none = ops.vp_fused(x, P3.vpfused.dp, lens)
    en, _ = ops.vp_fused(x, P3.vpfused.energy, lens)
    assert none is None and dp.shape == (2, B, L) and en.shape == (1, B, L)
    pad = torch.arange(L, device="cuda")[None, :] >= lens[:, None]
    cols = variance_predictors(P3.vpcols.dp, x, lens)
    for got, k in ((dp[0], "duration"), (dp[1], "pitch"), (en[0], "energy")):
        ref = variance_predictor(P32.vp[k], x, lens)
        err = (ref - got).abs()
        assert bool((err <= 2e-4 + 2e-4 * ref.abs()).all()), (k, float(err.max()))
        assert bool((got[pad] == 0).all())
    assert float((cols - dp).abs().max()) <= 4e-4 * max(1.0, float(cols.abs().max()))
    bins, table = P3.bins["pitch"], P3.var_table["pitch"]

    def embedded(v):
        return (x.float() + table[torch.bucketize(v, bins)]).to(torch.bfloat16)

    p2, x2 = ops.vp_fused(x, P3.vpfused.dp, lens, embed=(1, None, 1.3, bins, table))
    assert torch.equal(p2[0], dp[0]) and torch.equal(p2[1], dp[1] * 1.3)
    assert torch.equal(x2, embedded(p2[1])) and torch.equal(x, x0)
    tgt = torch.randn(B, L, generator=g).to("cuda")
    p3, x3 = ops.vp_fused(x, P3.vpfused.dp, lens, embed=(1, tgt, 1.0, bins, table))
    assert torch.equal(p3[1], dp[1]) and torch.equal(x3, embedded(tgt))
    e4, x4 = ops.vp_fused(x, P3.vpfused.energy, lens, embed=(0, None, 0.8, P3.bins["energy"], P3.var_table["energy"]))
    assert torch.equal(e4[0], en[0] * 0.8)
    assert torch.equal(x4, (x.float() + P3.var_table["energy"][torch.bucketize(e4[0], P3.bins["energy"])]).to(
        torch.bfloat16))


@pytest.mark.parametrize("compute", [0, 1])
@pytest.mark.parametrize("B,T,packed,shape", [
    (1, 8576, False, None),    # 67 x 8 tiles: one full round + a 24-tile tail (256 CUs)
    (3, 50, False, None),      # all-tail launch (16 tiles)
    (1, 10400, False, None),   # 3 segments per tail tile: they start mid channel block
    (64, 430, True, None),     # cfg2 decoder shape on packed rows (bf16: phased kernel + 128x128 rows left)
    (1, 40000, False, None),   # bf16 phased: 2 whole rounds
    (1, 16796, False, None),   # bf16 phased: 1 round + an 8-tile tail
    (1, 40000, False, (512, 512, 5))])  # PostNet conv shape (40 k-tiles)
def test_conv_splitk_tail(ops, compute, B, T, packed, shape):
    """Split-K tail (ops.splitk_enabled): tail tiles cut along K across idle workgroups, summed
    in segment order by the last arriver (128x128 kernel). Against the unsplit launches (ops.splitk_enabled(False)): f32 2e-5 /
    bf16 2.5e-2 of the output scale; and bit-identical across repeated launches (fixed
    summation order, counters reset themselves)."""
    L = _L()
    g = torch.Generator().manual_seed(T)
    Cin, N, KS = shape if shape is not None else (256, 1024, 9)
    dt = torch.float32 if compute == 0 else torch.bfloat16
    x = torch.randn(B, T, Cin, generator=g).to(DEV, dt)
    w = ops.pack_conv_weight((torch.randn(N, Cin, KS, generator=g) / np.sqrt(Cin * KS)).to(DEV), compute)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    kw = dict(cin=Cin, ks=KS, pad=(KS - 1) // 2, compute=compute, epilogue=L.EPI_BIAS_RELU, out_dtype=L.FS2_F32)
    if packed:
        lens = torch.randint(200, T + 1, (B,), generator=g).to(DEV)
        kw["layout"] = ops.SeqLayout(lens, T)
        x = x.reshape(B * T, Cin)
    with ops.splitk_enabled(False):
        ref = ops.conv1d(x, w, b, **kw)
    outs = [ops.conv1d(x, w, b, **kw) for _ in range(3)]
    torch.cuda.synchronize()
    rows = int(kw["layout"].cu[-1]) if packed else B * T
    r = ref.reshape(-1, N)[:rows].float()
    for o in outs:
        o = o.reshape(-1, N)[:rows].float()
        err = float((o - r).abs().max() / (r.abs().max() + 1e-6))
        assert err < _tol(compute), err
        assert torch.equal(o, outs[0].reshape(-1, N)[:rows].float())


@pytest.mark.parametrize("K,N,relu,packed", [(256, 768, False, False), (256, 768, False, True), (128, 256, True, False),
                                             (64, 384, False, True), (192, 1280, True, False)])
def test_weight_resident_projection(ops, K, N, relu, packed):
    """Short-K bf16 projections (Q|K|V shape) take the weight-resident kernel (gemm_wres.hip):
    vs torch fp32 on the same bf16 operands, |d| <= 1e-2 * max|y| (bf16 output rounding); packed
    rows: only the valid rows are written."""
    L = _L()
    g = torch.Generator().manual_seed(21)
    B, T = 7, 433  # 3,031 rows: not a multiple of the 64-row tile
    x = torch.randn(B, T, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / np.sqrt(K))
    b = torch.randn(N, generator=g) * 0.1
    wp = ops.pack_conv_weight(w.to(DEV), 1)
    epi = L.EPI_BIAS_RELU if relu else L.EPI_BIAS
    ref = x.float().cpu() @ wp.float().cpu()[:, 0, :].T + b
    if relu:
        ref = ref.clamp_min(0)
    if packed:
        lens = torch.randint(0, T + 1, (B,), generator=g).to(DEV)
        lay = ops.SeqLayout(lens, T)
        xp = torch.zeros(B * T, K, device=DEV, dtype=torch.bfloat16)
        rm = lay.rowmap.long()
        ok = rm >= 0
        xp[rm[ok]] = x.view(B * T, K)[ok]
        out = torch.full((B * T, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        ops.conv1d(xp, wp, b.to(DEV), cin=K, ks=1, pad=0, compute=1, epilogue=epi, out=out, layout=lay)
        got = lay.unpack(out).float().cpu()
        mask = (torch.arange(T)[None, :] < lens.cpu()[:, None]).unsqueeze(-1)
        ref = ref * mask
        rows = int(lay.cu[-1])
        assert bool(torch.isnan(out[rows:].float()).all())  # nothing written past the active rows
    else:
        got = ops.conv1d(x, wp, b.to(DEV), cin=K, ks=1, pad=0, compute=1, epilogue=epi,
                         out_dtype=L.FS2_BF16).float().cpu()
    torch.cuda.synchronize()
    err = (got - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err


def test_attention_key_split(ops, monkeypatch):
    """fs2_attention_ex's key-split form over its work list (free-running synthesis: packed rows
    with a known row count, T > 256): sequences of up to 959 keys in 256-key ranges merged by the
    last range, against the float reference (2e-2 of the output scale, bf16 operands); sequences
    of <= 256 keys bit-identical to the unsplit kernel; the result bit-identical for two T buckets
    of the same batch (the split depends on each sequence's length only) and over repeated calls."""
    g = torch.Generator().manual_seed(11)
    H, dk = 2, 128
    lens = torch.tensor([959, 12, 256, 257, 300, 520, 64, 700, 1, 180, 511, 768], dtype=torch.int64)
    B, T = lens.numel(), 960
    C = 3 * H * dk
    qkv = torch.randn(B, T, C, generator=g).to(torch.bfloat16)

    def run(Tb, split):
        monkeypatch.setenv("FS2_ATTN_SPLIT", "1" if split else "0")
        lay = ops.SeqLayout(lens.to(DEV), Tb)
        lay.rows_hint = int(lens.sum())
        rm = lay.rowmap.long().cpu()
        ok = rm >= 0
        src = torch.zeros(B, Tb, C, dtype=torch.bfloat16)
        src[:, :min(T, Tb)] = qkv[:, :min(T, Tb)]
        xp = torch.zeros(lay.capacity, C, dtype=torch.bfloat16)
        xp[rm[ok]] = src.reshape(-1, C)[ok]
        out = ops.attention(xp.to(DEV), None, H, dk, float(np.power(dk, 0.5)), layout=lay)
        torch.cuda.synchronize()
        cu = lay.cu.long().cpu()
        return [out[int(cu[b]):int(cu[b + 1])].float().cpu() for b in range(B)]

    split = run(T, True)
    plain = run(T, False)
    ref = _ref_attention(qkv.float(), lens, H, dk)
    for b in range(B):
        n = int(lens[b])
        r = ref[b, :n]
        err = float((split[b] - r).abs().max() / r.abs().max())
        assert err < 2e-2, (b, n, err)
        if n <= 256:
            assert torch.equal(split[b], plain[b]), (b, n)
    again = run(T, True)
    other = run(1024, True)
    for b in range(B):
        assert torch.equal(again[b], split[b]), ("nondeterministic", b)
        assert torch.equal(other[b], split[b]), ("T-dependent", b)
