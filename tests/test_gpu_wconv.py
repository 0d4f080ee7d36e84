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
