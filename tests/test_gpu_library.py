"""fs2amd.library on the GPU: the torch.library ops against the direct fs2amd.ops
launches (bit-identical: same kernels), torch.library.opcheck (schema, fake, autograd
registration), attention's registered backward against fs2_attention_bwd, and a function of the
ops compiled with ``torch.compile(fullgraph=True)`` (the fake implementations trace it; the
aot_eager backend, no code generation) equal to eager."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import fs2amd.library  # noqa: F401
    from fs2amd import ops, _lib as L

    return ops, L


def _attn_inputs(B=3, T=70, seed=0, dtype=torch.bfloat16):
    g = torch.Generator(device=DEV).manual_seed(seed)
    qkv = torch.randn(B, T, 768, device=DEV, generator=g).to(dtype)
    lens = torch.tensor([T] + [max(1, T - 13 * i) for i in range(1, B)], device=DEV)
    return qkv, lens


def test_attention_op_equals_direct_launch(gpu):
    ops, _ = gpu
    qkv, lens = _attn_inputs()
    a = torch.ops.fs2.attention(qkv, lens, 2, 128, 128 ** 0.5)
    b = ops.attention(qkv, lens, 2, 128, 128 ** 0.5)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_attention_op_autograd(gpu):
    ops, _ = gpu
    qkv, lens = _attn_inputs(seed=1)
    q = qkv.clone().requires_grad_(True)
    out = torch.ops.fs2.attention(q, lens, 2, 128, 128 ** 0.5)
    g = torch.randn(out.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(2)).to(out.dtype)
    out.backward(g)
    ref = ops.attention_bwd(qkv, out.detach(), g.float(), lens, 2, 128, 128 ** 0.5)
    torch.cuda.synchronize()
    assert torch.equal(q.grad, ref.to(qkv.dtype))


def test_opcheck(gpu):
    qkv, lens = _attn_inputs(B=2, T=40, seed=3)
    tests = ("test_schema", "test_faketensor", "test_autograd_registration")
    torch.library.opcheck(torch.ops.fs2.attention.default, (qkv, lens, 2, 128, 128 ** 0.5), test_utils=tests)
    x = torch.randn(2, 5, 256, device=DEV)
    dur = torch.tensor([[1, 2, 0, 3, 1], [2, 2, 2, 0, 0]], device=DEV)
    torch.library.opcheck(torch.ops.fs2.length_regulate.default, (x, dur, 12), test_utils=tests)


def test_length_regulate_op(gpu):
    ops, _ = gpu
    x = torch.randn(2, 5, 256, device=DEV)
    dur = torch.tensor([[1, 2, 0, 3, 1], [2, 2, 2, 0, 0]], device=DEV)
    y, ml = torch.ops.fs2.length_regulate(x, dur, 0)
    y2, ml2 = ops.length_regulate(x, dur)
    assert torch.equal(y, y2) and torch.equal(ml, ml2) and y.shape[1] == 7


def test_ffn_op_equals_direct_launch(gpu):
    ops, L = gpu
    g = torch.Generator(device=DEV).manual_seed(4)
    w1 = torch.randn(1024, 256, 9, device=DEV, generator=g) / 48.0
    w2 = torch.randn(256, 1024, 1, device=DEV, generator=g) / 32.0
    b1, b2 = 0.1 * torch.randn(1024, device=DEV, generator=g), 0.1 * torch.randn(256, device=DEV, generator=g)
    gam, bet = 1 + 0.1 * torch.randn(256, device=DEV, generator=g), 0.1 * torch.randn(256, device=DEV, generator=g)
    w12 = ops.pack_ffn_weights(w1, w2)
    x = torch.randn(4, 50, 256, device=DEV, generator=g).to(torch.bfloat16)
    lens = torch.tensor([50, 31, 7, 1], device=DEV)
    a = torch.ops.fs2.ffn(x, w12, b1, b2, gam, bet, 1e-5, lens, 9, 4)
    b = ops.ffn(x, w12, b1, b2, ks=9, pad=4, ln=(gam, bet, 1e-5), lens=lens)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_conv1d_op_equals_direct_launch(gpu):
    ops, L = gpu
    g = torch.Generator(device=DEV).manual_seed(5)
    w = torch.randn(256, 256, 3, device=DEV, generator=g) / 28.0
    b = 0.1 * torch.randn(256, device=DEV, generator=g)
    wp = ops.pack_conv_weight(w, L.FS2_BF16)
    x = torch.randn(3, 41, 256, device=DEV, generator=g).to(torch.bfloat16)
    a = torch.ops.fs2.conv1d(x, wp, b, 256, 3, 1, L.FS2_BF16, L.EPI_BIAS_RELU, L.FS2_BF16)
    r = ops.conv1d(x, wp, b, cin=256, ks=3, pad=1, compute=L.FS2_BF16, epilogue=L.EPI_BIAS_RELU,
                   out_dtype=L.FS2_BF16)
    ref = torch.relu(torch.nn.functional.conv1d(x.float().transpose(1, 2), w.to(torch.bfloat16).float(), b,
                                                padding=1)).transpose(1, 2)
    torch.cuda.synchronize()
    assert torch.equal(a, r) and a.shape == (3, 41, 256)
    assert (a.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    with pytest.raises(ValueError):
        torch.ops.fs2.conv1d(x, wp, b, 256, 3, 1, L.FS2_BF16, L.EPI_RES_LN, L.FS2_BF16)


def test_compile_fullgraph(gpu):
    """LengthRegulator -> attention over the expanded frames, traced whole (no graph break at the
    ctypes launches) and equal to the eager ops."""
    x = torch.randn(2, 6, 768, device=DEV).to(torch.bfloat16)
    dur = torch.tensor([[3, 1, 4, 1, 5, 9], [2, 6, 5, 3, 5, 0]], device=DEV)

    def fn(x, dur):
        y, ml = torch.ops.fs2.length_regulate(x, dur, 24)
        return torch.ops.fs2.attention(y, ml, 2, 128, 128 ** 0.5)

    torch._dynamo.reset()
    cfn = torch.compile(fn, backend="aot_eager", fullgraph=True)
    a = cfn(x, dur)
    b = fn(x, dur)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
