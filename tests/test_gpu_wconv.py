"""fs2_wconv — the PostNet's 512 -> 512 and 80 -> 512, k=5 Conv1d + folded BatchNorm + tanh on the
weight-streamed kernel (transformer/Layers.py:92-137).

* against a float64 PyTorch statement of the same op on the same bf16 operands (per-sequence zero
  taps, f32 result rounded to bf16 once): bf16 output tolerance;
* against the fs2_conv1d launch it replaces (same bf16 operands; only the f32 summation order
  differs): at most one bf16 ulp apart;
* ragged T (not multiples of the 112-row tile), B*T below one tile, a lone row; rows past B*T are
  never written.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from fs2amd import ops, _lib as L

    return ops, L


def _case(ops, L, B, T, seed, cin=512):
    g = torch.Generator(device=DEV).manual_seed(seed)
    w = torch.randn(512, cin, 5, device=DEV, generator=g) / (cin * 5) ** 0.5
    s = 1 + 0.1 * torch.randn(512, device=DEV, generator=g)  # a folded BatchNorm scale
    b = 0.1 * torch.randn(512, device=DEV, generator=g)
    x = torch.randn(B, T, cin, device=DEV, generator=g).to(torch.bfloat16)
    return x, w, s, b


@pytest.mark.parametrize("cin", [512, 80])  # 80: the PostNet's first conv, K = (tap, channel) flattened
@pytest.mark.parametrize("B,T,seed", [(64, 430, 1), (3, 37, 2), (1, 1, 3), (5, 113, 4)])
def test_wconv_matches_float64_and_conv1d(gpu, B, T, seed, cin):
    ops, L = gpu
    x, w, s, b = _case(ops, L, B, T, seed, cin)
    wq = (w * s[:, None, None]).to(torch.bfloat16)  # the operands both kernels see
    got = ops.wconv(x, ops.pack_wconv_weight(w, scale=s), b, ks=5, pad=2)
    ref = torch.tanh(torch.nn.functional.conv1d(x.double().transpose(1, 2), wq.double(), b.double(),
                                                padding=2).transpose(1, 2))
    err = (got.double() - ref).abs()
    assert float(err.max()) <= 8e-3 and float(err.mean()) <= 1e-3, (float(err.max()), float(err.mean()))
    two = ops.conv1d(x, ops.pack_conv_weight(w, L.FS2_BF16, scale=s), b, cin=cin, ks=5, pad=2, compute=L.FS2_BF16,
                     epilogue=L.EPI_BIAS_TANH, out_dtype=L.FS2_BF16)
    d = (got.float() - two.float()).abs()
    ulp = two.float().abs().clamp(min=2 ** -10) * 2 ** -7
    assert bool((d <= ulp).all()), float((d - ulp).max())


def test_wconv_writes_only_its_rows(gpu):
    ops, L = gpu
    x, w, s, b = _case(ops, L, 2, 50, 9)
    big = torch.full((2 * 50 + 7, 512), 3.0, device=DEV, dtype=torch.bfloat16)
    out = big[:100].view(2, 50, 512)
    ops.wconv(x, ops.pack_wconv_weight(w, scale=s), b, ks=5, pad=2, out=out)
    torch.cuda.synchronize()
    assert bool((big[100:] == 3.0).all())


def test_wconv_rejects(gpu):
    ops, L = gpu
    x, w, s, b = _case(ops, L, 2, 8, 1)
    wp = ops.pack_wconv_weight(w, scale=s)
    with pytest.raises(RuntimeError):
        ops.wconv(x, wp, b, ks=5, pad=2, out=x)  # out aliasing x
    with pytest.raises(TypeError):
        ops.wconv(x.float(), wp, b, ks=5, pad=2)
    with pytest.raises(AssertionError):
        ops.wconv(x, wp[:-1], b, ks=5, pad=2)


@pytest.mark.parametrize("B,T,seed", [(64, 430, 11), (3, 37, 12), (1, 1, 13), (5, 113, 14), (2, 3, 15)])
def test_pn_head_equals_two_wconv_launches(gpu, B, T, seed):
    """The PostNet's layers 0 and 1 in one launch (fs2_wconv with w2: 80 -> 512 -> 512, the first
    conv's output kept on chip with its 2-row halo recomputed) equal the two fs2_wconv launches
    BIT-EXACTLY: the same bf16 intermediate (same per-row arithmetic and k order for conv 1; conv 2
    is wconv's main loop on the same operands); ragged T, a lone row, T < the halo."""
    ops, L = gpu
    x, w1, s1, b1 = _case(ops, L, B, T, seed, 80)
    _, w2, s2, b2 = _case(ops, L, B, T, seed + 100, 512)
    p1, p2 = ops.pack_wconv_weight(w1, scale=s1), ops.pack_wconv_weight(w2, scale=s2)
    two = ops.wconv(ops.wconv(x, p1, b1, ks=5, pad=2), p2, b2, ks=5, pad=2)
    one = ops.wconv(x, p1, b1, ks=5, pad=2, second=(p2, b2))
    torch.cuda.synchronize()
    assert torch.equal(one, two), float((one.float() - two.float()).abs().max())


@pytest.mark.parametrize("B,T,seed", [(64, 430, 21), (3, 37, 22), (1, 1, 23), (5, 113, 24), (2, 3, 25)])
def test_pn_tail_matches_float64_and_conv1d(gpu, B, T, seed):
    """The PostNet's last conv + residual on fs2_wconv's N = 80 form (every wave all 80 columns,
    k-step weights through an LDS ring): against float64 on the same bf16 operands (f32 output:
    2e-4 relative to the output scale) and against the fs2_conv1d launch it replaces (same operands,
    only the f32 summation order differs: 2e-5)."""
    ops, L = gpu
    g = torch.Generator(device=DEV).manual_seed(seed)
    w = torch.randn(80, 512, 5, device=DEV, generator=g) / (512 * 5) ** 0.5
    sc = 1 + 0.1 * torch.randn(80, device=DEV, generator=g)
    b = 0.1 * torch.randn(80, device=DEV, generator=g)
    x = torch.randn(B, T, 512, device=DEV, generator=g).to(torch.bfloat16)
    res = torch.randn(B, T, 80, device=DEV, generator=g)
    wq = (w * sc[:, None, None]).to(torch.bfloat16)
    got = ops.wconv_tail(x, ops.pack_wconv_tail(w, scale=sc), b, res)
    ref = torch.nn.functional.conv1d(x.double().transpose(1, 2), wq.double(), b.double(), padding=2).transpose(1, 2) \
        + res.double()
    scale = float(ref.abs().max())
    assert float((got.double() - ref).abs().max()) <= 2e-4 * scale
    two = ops.conv1d(x, ops.pack_conv_weight(w, L.FS2_BF16, scale=sc), b, cin=512, ks=5, pad=2, compute=L.FS2_BF16,
                     epilogue=L.EPI_BIAS_RES, out_dtype=L.FS2_F32, residual=res)
    assert float((got - two).abs().max()) <= 2e-5 * scale


@pytest.mark.parametrize("prec", ["bf16"])
def test_postnet_valid_region_equals_padded(gpu, prec):
    """The PostNet's valid-region form (free-running batches padded to one long utterance: packed
    rows over each utterance's frames + 20, the rest from the constant row / tail block) equals the
    padded PostNet BIT-EXACTLY on every frame: both forms run the same kernels (fs2_wconv's padded
    and packed-row modes), padded frames hold mel_linear's bias as in the forward. Boundaries at
    len + 10 and T - 10 are checked by the all-frame equality; lengths 0, 1, T - 25, T - 45, T."""
    ops, L = gpu
    from fs2amd import runtime as R
    from fs2amd.model import FastSpeech2
    from fs2amd.synth_weights import fill_module
    from _common import configs

    pc, mc, _ = configs()
    m = FastSpeech2(pc, mc)
    fill_module(m, seed=3)
    m = m.to(DEV).eval().set_precision(prec)
    P = m.packed(DEV)
    T = 300
    lens = torch.tensor([0, 1, T - 25, T - 45, T, 37, 120, 2], device=DEV)
    B = lens.numel()
    g = torch.Generator(device=DEV).manual_seed(5)
    mel = torch.randn(B, T, 80, device=DEV, generator=g)
    pad = torch.arange(T, device=DEV)[None, :] >= lens[:, None]
    mel = torch.where(pad[..., None], P.mel_b.float().view(1, 1, 80), mel).contiguous()
    mel_bf = mel.to(torch.bfloat16) if prec == "bf16" else None
    with torch.no_grad():
        full = R._postnet(P, mel, mel_bf)
        valid = R._postnet(P, mel, mel_bf, lens, int(lens.sum()))
    torch.cuda.synchronize()
    assert torch.equal(valid, full), float((valid - full).abs().max())


@pytest.mark.parametrize("B,T,seed,packed", [(64, 430, 31, False), (3, 37, 32, False), (1, 1, 33, False),
                                             (5, 113, 34, False), (2, 3, 35, False), (9, 250, 36, True),
                                             (4, 61, 37, True)])
def test_pn_tail_fused_equals_two_launches(gpu, B, T, seed, packed):
    """The PostNet's layers 3 and 4 in one launch (fs2_wconv with a Cin = 512 w2: the 512 -> 512
    tanh output kept on chip, the 512 -> 80 conv + residual on each workgroup's 108 middle rows)
    equal fs2_wconv + the N = 80 tail launch BIT-EXACTLY: the same bf16 intermediate rows (per-row
    arithmetic independent of the 108-row tiling) and pn_tail's k-step order; ragged T, a lone row,
    T below the halo, padded rows and packed rows (lengths 0 / 1 / T included)."""
    ops, L = gpu
    x, w, s, b = _case(ops, L, B, T, seed, 512)
    g = torch.Generator(device=DEV).manual_seed(seed + 500)
    wt = torch.randn(80, 512, 5, device=DEV, generator=g) / (512 * 5) ** 0.5
    sc = 1 + 0.1 * torch.randn(80, device=DEV, generator=g)
    bt = 0.1 * torch.randn(80, device=DEV, generator=g)
    res = torch.randn(B, T, 80, device=DEV, generator=g)
    p, pt = ops.pack_wconv_weight(w, scale=s), ops.pack_wconv_tail(wt, scale=sc)
    lay = None
    if packed:
        lens = torch.randint(0, T + 1, (B,), generator=torch.Generator().manual_seed(seed)).to(DEV)
        lens[0], lens[-1] = T, 0
        if B > 2:
            lens[1] = 1
        lay = ops.SeqLayout(lens, T)
        rm = lay.rowmap.long()
        ok = rm >= 0
        xp = x.new_zeros(lay.capacity, 512)
        xp[rm[ok]] = x.reshape(-1, 512)[ok]
        rp = res.new_zeros(lay.capacity, 80)
        rp[rm[ok]] = res.reshape(-1, 80)[ok]
        x, res = xp, rp
    two = ops.wconv_tail(ops.wconv(x, p, b, ks=5, pad=2, layout=lay), pt, bt, res, layout=lay)
    one = ops.wconv(x, p, b, ks=5, pad=2, layout=lay, tail=(pt, bt, res))
    torch.cuda.synchronize()
    if lay is not None:
        R = int(lay.cu[-1])
        one, two = one[:R], two[:R]
    assert torch.equal(one, two), float((one - two).abs().max())
