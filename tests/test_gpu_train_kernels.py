"""Training-step kernels (train.hip + the conv's FS2_EPI_RELU_GRAD epilogue) against float64
PyTorch statements of the same ops, through the C ABI.

* fs2_res_ln_fwd / fs2_res_ln_bwd: masked_fill(LayerNorm(dropout(a) + res)) and its autograd
  gradient (transformer/SubLayers.py:54-57,90-93, Layers.py:27-30). f32 throughout: outputs within
  2e-5 of the output scale; da (stored bf16) within 1e-2 relative. With dropout the keep mask is
  read back from the kernel itself (a = 1, res = 0: xhat > 0 exactly on kept elements) and the
  reference is evaluated with that mask; the keep fraction must be 1 - p within 1 %.
* fs2_colsum: float64 column sums, 1e-5 relative.
* fs2_conv_wgrad: dW[n, c, k] = sum dy[t, n] x[t + k - pad, c] per sequence, from the bf16-rounded
  operands in float64 (the kernel's MFMA products are exact, f32 accumulation): 2e-4 of the
  gradient scale. Sequence edges, T not a multiple of the 32-row chunk, N / C = 80 partial tiles,
  f32 and bf16 dy, bias gradient, accumulation and Q|K|V row parts.
"""
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


def _mask(lens, T):
    return torch.arange(T)[None, :] >= lens[:, None]


def _keep_mask(ops, B, T, p, seed, salt):
    ones = torch.ones(B, T, 256, device=DEV)
    g, b = torch.ones(256, device=DEV), torch.zeros(256, device=DEV)
    _, _, xh, _ = ops.res_ln_fwd(ones, torch.zeros_like(ones), g, b, 1e-5, None, p, seed, salt, want_bf16=False)
    return (xh > 0).cpu()


@pytest.mark.parametrize("p,res_bf16", [(0.0, False), (0.2, False), (0.1, True)])
def test_res_ln_fwd_bwd(ops, p, res_bf16):
    torch.manual_seed(1)
    B, T, D = 5, 37, 256
    lens = torch.tensor([37, 20, 1, 0, 33])
    a = torch.randn(B, T, D)
    res = torch.randn(B, T, D)
    if res_bf16:
        res = res.to(torch.bfloat16).float()
    gam, bet = 1 + 0.1 * torch.randn(D), 0.1 * torch.randn(D)
    seed = torch.tensor([1234567], dtype=torch.int64, device=DEV)
    salt = 7
    y, yb, xh, rs = ops.res_ln_fwd(a.to(DEV), (res.to(torch.bfloat16) if res_bf16 else res).to(DEV), gam.to(DEV),
                                   bet.to(DEV), 1e-5, lens.to(DEV), p, seed, salt)
    keep = _keep_mask(ops, B, T, p, seed, salt) if p > 0 else torch.ones(B, T, D, dtype=torch.bool)
    if p > 0:
        assert abs(float(keep.float().mean()) - (1 - p)) < 0.01
    ad, rd = a.double().requires_grad_(), res.double().requires_grad_()
    v = ad * keep / (1 - p) + rd
    ref = F.layer_norm(v, (D,), gam.double(), bet.double(), 1e-5).masked_fill(_mask(lens, T)[..., None], 0)
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    assert float((y.cpu().double() - ref).abs().max()) <= 2e-5 * scale
    assert float((yb.cpu().double() - ref).abs().max()) <= 1e-2 * scale
    dy = torch.randn(B, T, D)
    gd, bd = gam.double().requires_grad_(), bet.double().requires_grad_()
    ref2 = F.layer_norm(v, (D,), gd, bd, 1e-5).masked_fill(_mask(lens, T)[..., None], 0)
    ref2.backward(dy.double())
    # a's producer is a conv with a bias: its gradient is sum over rows of da
    dres, da, dg, dbe, dbias = ops.res_ln_bwd(dy.to(DEV), xh, rs, gam.to(DEV), lens.to(DEV), p, seed, salt)
    torch.cuda.synchronize()
    sc = float(rd.grad.abs().max())
    assert float((dres.cpu().double() - rd.grad).abs().max()) <= 2e-5 * sc
    assert float((da.cpu().double() - ad.grad).abs().max()) <= 1e-2 * float(ad.grad.abs().max())
    assert torch.allclose(dg.cpu().double(), gd.grad, rtol=1e-4, atol=1e-4 * float(gd.grad.abs().max()))
    assert torch.allclose(dbe.cpu().double(), bd.grad, rtol=1e-4, atol=1e-4 * float(bd.grad.abs().max()))
    dsum = ad.grad.sum((0, 1))
    assert torch.allclose(dbias.cpu().double(), dsum, rtol=1e-3, atol=1e-4 * float(dsum.abs().max()))
    # accumulate: a second call adds
    ops.res_ln_bwd(dy.to(DEV), xh, rs, gam.to(DEV), lens.to(DEV), p, seed, salt, dgamma=dg, dbeta=dbe, dbias=dbias,
                   accumulate=True)
    torch.cuda.synchronize()
    assert torch.allclose(dg.cpu().double(), 2 * gd.grad, rtol=1e-4, atol=2e-4 * float(gd.grad.abs().max()))


def test_res_ln_seed_advances_mask(ops):
    seed = torch.tensor([5], dtype=torch.int64, device=DEV)
    k1 = _keep_mask(ops, 2, 16, 0.3, seed, 3)
    k1b = _keep_mask(ops, 2, 16, 0.3, seed, 3)
    seed.add_(1)
    k2 = _keep_mask(ops, 2, 16, 0.3, seed, 3)
    k3 = _keep_mask(ops, 2, 16, 0.3, seed, 4)
    assert torch.equal(k1, k1b)
    assert not torch.equal(k1, k2) and not torch.equal(k2, k3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_colsum(ops, dtype):
    torch.manual_seed(2)
    x = torch.randn(3, 1111, 768).to(dtype)
    out = ops.colsum(x.to(DEV))
    torch.cuda.synchronize()
    ref = x.double().sum((0, 1))
    assert torch.allclose(out.cpu().double(), ref, rtol=1e-5, atol=1e-4)
    out2 = ops.colsum(x.to(DEV), out=out.clone(), accumulate=True)
    assert torch.allclose(out2.cpu().double(), 2 * ref, rtol=1e-5, atol=2e-4)


def _ref_wgrad(dy, x, ks, pad):
    # dW[n, c, k] = sum_{b,t} dy[b,t,n] x[b,t+k-pad,c]   (x zero outside [0, T))
    B, T, N = dy.shape
    C = x.shape[-1]
    xp = F.pad(x.double(), (0, 0, pad, ks - 1 - pad))
    xu = xp.unfold(1, ks, 1)  # [B, T, C, ks]
    return torch.einsum("btn,btck->nck", dy.double(), xu)


@pytest.mark.parametrize("N,C,ks,pad,T,dy_f32", [
    (1024, 256, 9, 4, 93, False),   # FFN w_1
    (256, 1024, 1, 0, 70, False),   # FFN w_2
    (768, 256, 1, 0, 64, True),     # Q|K|V (dqkv f32 from the attention backward)
    (256, 256, 3, 1, 45, False),    # VariancePredictor conv
    (512, 80, 5, 2, 40, False),     # PostNet first conv
    (80, 512, 5, 2, 33, True),      # PostNet last conv
    (80, 256, 1, 0, 17, False),     # mel_linear
])
def test_conv_wgrad(ops, N, C, ks, pad, T, dy_f32):
    torch.manual_seed(N + C + ks)
    B = 3
    dy = torch.randn(B, T, N)
    dy = dy if dy_f32 else dy.to(torch.bfloat16)
    x = torch.randn(B, T, C).to(torch.bfloat16)
    dw, db = ops.conv_wgrad(dy.to(DEV), x.to(DEV), ks, pad, want_db=True)
    torch.cuda.synchronize()
    dyr = dy.to(torch.bfloat16) if dy_f32 else dy   # the kernel's MFMA operands are bf16
    ref = _ref_wgrad(dyr, x, ks, pad)
    sc = float(ref.abs().max())
    err = float((dw.cpu().double() - ref).abs().max())
    assert err <= 2e-4 * sc, (err, sc)
    dbr = dy.double().sum((0, 1))
    assert torch.allclose(db.cpu().double(), dbr, rtol=1e-4, atol=1e-4 * float(dbr.abs().max()))
    dw2, db2 = ops.conv_wgrad(dy.to(DEV), x.to(DEV), ks, pad, dw=dw.clone(), db=db.clone(), accumulate=True)
    torch.cuda.synchronize()
    assert float((dw2.cpu().double() - 2 * ref).abs().max()) <= 4e-4 * sc


def test_conv_wgrad_qkv_parts(ops):
    torch.manual_seed(3)
    B, T, N, C = 2, 50, 768, 256
    dy = torch.randn(B, T, N)
    x = torch.randn(B, T, C).to(torch.bfloat16)
    dws = [torch.full((256, 256), 1.0, device=DEV) for _ in range(3)]
    dbs = [torch.full((256,), 1.0, device=DEV) for _ in range(3)]
    ops.conv_wgrad(dy.to(DEV), x.to(DEV), 1, 0, parts=(dws, dbs), accumulate=True)
    torch.cuda.synchronize()
    ref = _ref_wgrad(dy.to(torch.bfloat16), x, 1, 0)[..., 0] + 1.0
    dbr = dy.double().sum((0, 1)) + 1.0
    for i in range(3):
        assert float((dws[i].cpu().double() - ref[256 * i:256 * (i + 1)]).abs().max()) <= 2e-4 * float(ref.abs().max())
        assert torch.allclose(dbs[i].cpu().double(), dbr[256 * i:256 * (i + 1)], rtol=1e-4, atol=1e-3)


def test_conv_relu_grad_epilogue(ops):
    """FS2_EPI_RELU_GRAD: the input gradient of w_2 (its transposed conv) masked by relu(u) > 0."""
    from fs2amd import _lib as L
    torch.manual_seed(4)
    B, T, Cin, N = 2, 61, 256, 1024
    d = torch.randn(B, T, Cin).to(torch.bfloat16)
    w = torch.randn(N, Cin) / 16
    u = torch.relu(torch.randn(B, T, N)).to(torch.bfloat16)
    wp = ops.pack_conv_weight(w.to(DEV), L.FS2_BF16)
    out = ops.conv1d(d.to(DEV), wp, None, cin=Cin, ks=1, pad=0, compute=L.FS2_BF16, epilogue=L.EPI_RELU_GRAD,
                     out_dtype=L.FS2_BF16, residual=u.to(DEV))
    torch.cuda.synchronize()
    ref = (d.double() @ w.to(torch.bfloat16).double().t()) * (u.double() > 0)
    assert float((out.cpu().double() - ref).abs().max()) <= 1e-2 * float(ref.abs().max())
    assert bool(((out.cpu() == 0) | (u > 0)).all())


def test_pack_train_images(ops):
    """fs2_pack_train (one launch for every block's weight images) equals the per-weight torch
    packing (pack_conv_weight / the flipped-transposed input-gradient form) bit for bit."""
    from fs2amd import _lib as L
    from fs2amd.model import _FFTBlock
    from fs2amd.training import _TrainPack, _packT

    torch.manual_seed(5)
    blocks = [_FFTBlock(256, 2, 1024, (9, 1)).to(DEV), _FFTBlock(256, 2, 1024, (9, 3)).to(DEV)]
    extra = [torch.nn.Conv1d(80, 512, 5).to(DEV), torch.nn.Conv1d(512, 80, 5).to(DEV),
             torch.nn.Conv1d(256, 256, 3).to(DEV)]
    tp = _TrainPack(blocks, torch.device(DEV), extra)
    tp.run(torch.zeros(1, device=DEV))
    torch.cuda.synchronize()
    from fs2amd.training import _packT_any
    for conv in extra:  # VariancePredictor / PostNet convs, channel-padded images (80 channels)
        fw, tr = tp.extra[conv]
        ef, et = ops.pack_conv_weight(conv.weight, L.FS2_BF16), _packT_any(conv.weight)
        assert fw.shape == ef.shape and tr.shape == et.shape
        assert torch.equal(fw, ef) and torch.equal(tr, et)
    for blk, P in zip(blocks, tp.per_block):
        a, f = blk.slf_attn, blk.pos_ffn
        wqkv = torch.cat([a.w_qs.weight, a.w_ks.weight, a.w_vs.weight], 0).detach()
        exp = dict(qkv=ops.pack_conv_weight(wqkv, L.FS2_BF16), fc=ops.pack_conv_weight(a.fc.weight, L.FS2_BF16),
                   w1=ops.pack_conv_weight(f.w_1.weight, L.FS2_BF16), w2=ops.pack_conv_weight(f.w_2.weight, L.FS2_BF16),
                   qkvT=_packT(wqkv), fcT=_packT(a.fc.weight), w1T=_packT(f.w_1.weight), w2T=_packT(f.w_2.weight),
                   bqkv=torch.cat([a.w_qs.bias, a.w_ks.bias, a.w_vs.bias]).detach())
        for k, v in exp.items():
            assert P[k].shape == v.shape, k
            assert torch.equal(P[k], v), k


@pytest.mark.parametrize("p", [0.0, 0.5])
def test_relu_ln_fwd_bwd(ops, p):
    """fs2_relu_ln_fwd / _bwd: y = dropout(LayerNorm(relu(a))) (a VariancePredictor layer,
    model/modules.py:218-235) and its gradient against float64 autograd with the kernel's keep
    mask; same tolerances as the residual form."""
    torch.manual_seed(6)
    R, D = 333, 256
    a = torch.randn(R, D)
    gam, bet = 1 + 0.1 * torch.randn(D), 0.1 * torch.randn(D)
    seed = torch.tensor([99], dtype=torch.int64, device=DEV)
    salt = 11
    y, yb, xh, rs = ops.relu_ln_fwd(a.to(DEV), gam.to(DEV), bet.to(DEV), 1e-5, p, seed, salt)
    if p > 0:  # keep bits: the same hash as fs2_res_ln_fwd's (row * 256 + column, seed, salt)
        keep = _keep_mask(ops, 1, R, p, seed, salt).view(R, D)
    else:
        keep = torch.ones(R, D, dtype=torch.bool)
    ad = a.double().requires_grad_()
    gd, bd = gam.double().requires_grad_(), bet.double().requires_grad_()
    ref = F.layer_norm(torch.relu(ad), (D,), gd, bd, 1e-5) * keep / (1 - p)
    torch.cuda.synchronize()
    sc = float(ref.abs().max())
    assert float((y.cpu().double() - ref).abs().max()) <= 2e-5 * sc
    assert float((yb.cpu().double() - ref).abs().max()) <= 1e-2 * sc
    dy = torch.randn(R, D)
    ref.backward(dy.double())
    da, dg, dbe, db = ops.relu_ln_bwd(dy.to(DEV), a.to(DEV), xh, rs, gam.to(DEV), p, seed, salt)
    torch.cuda.synchronize()
    assert float((da.cpu().double() - ad.grad).abs().max()) <= 1e-2 * float(ad.grad.abs().max())
    assert torch.allclose(dg.cpu().double(), gd.grad, rtol=1e-4, atol=1e-4 * float(gd.grad.abs().max()))
    assert torch.allclose(dbe.cpu().double(), bd.grad, rtol=1e-4, atol=1e-4 * float(bd.grad.abs().max()))
    dsum = ad.grad.sum(0)
    assert torch.allclose(db.cpu().double(), dsum, rtol=1e-3, atol=1e-3 * float(dsum.abs().max()))


@pytest.mark.parametrize("p", [0.0, 0.5])
@pytest.mark.parametrize("defer", [False, True])
def test_relu_ln_head_fwd_bwd(ops, p, defer):
    """fs2_relu_ln_head_fwd / _bwd: the VariancePredictor's second layer and head,
    out = masked_fill(dropout(LayerNorm(relu(a))) . w + b, mask, 0) (model/modules.py:225-250), and
    the gradients of a, gamma, beta, the conv bias, w and b from the output's gradient, against
    float64 autograd with the kernel's keep mask; the head's gradients finished in place or deferred
    (fs2_reduce_batch_launch kind 2), accumulating into existing gradients in the deferred case."""
    torch.manual_seed(7)
    B, Lx, D = 9, 37, 256
    R = B * Lx
    a = torch.randn(R, D)
    gam, bet = 1 + 0.1 * torch.randn(D), 0.1 * torch.randn(D)
    hw, hb = torch.randn(D) / 16, 0.3 * torch.randn(1)
    mask = torch.rand(B, Lx) < 0.2
    seed = torch.tensor([77], dtype=torch.int64, device=DEV)
    salt = 5
    out, xh, rs = ops.relu_ln_head_fwd(a.to(DEV).view(B, Lx, D), gam.to(DEV), bet.to(DEV), 1e-5, hw.to(DEV), hb.to(DEV),
                                       mask.to(DEV), p, seed, salt)
    keep = _keep_mask(ops, 1, R, p, seed, salt).view(R, D) if p > 0 else torch.ones(R, D, dtype=torch.bool)
    ad = a.double().requires_grad_()
    gd, bd = gam.double().requires_grad_(), bet.double().requires_grad_()
    wd, hbd = hw.double().requires_grad_(), hb.double().requires_grad_()
    y = F.layer_norm(torch.relu(ad), (D,), gd, bd, 1e-5) * keep / (1 - p)
    ref = (y @ wd + hbd).view(B, Lx).masked_fill(mask, 0.0)
    torch.cuda.synchronize()
    assert out.shape == (B, Lx)
    assert float((out.cpu().double() - ref).abs().max()) <= 2e-5 * float(ref.abs().max())
    dout = torch.randn(B, Lx)
    ref.backward(dout.double())
    q = [] if defer else None
    base = [torch.randn(n, device=DEV) if defer else None for n in (D, D, D, D, 1)]
    prev = [None if t is None else t.clone() for t in base]
    da, dg, dbe, db, dhw, dhb = ops.relu_ln_head_bwd(dout.to(DEV), mask.to(DEV), hw.to(DEV), bet.to(DEV),
                                                     a.to(DEV).view(B, Lx, D), xh, rs, gam.to(DEV), p, seed, salt,
                                                     dgamma=base[0], dbeta=base[1], dbias=base[2], dhw=base[3],
                                                     dhb=base[4], accumulate=defer, defer=q)
    if defer:
        ops.reduce_flush(q, da)
    torch.cuda.synchronize()
    off = [torch.zeros(1, dtype=torch.float64) if t is None else t.cpu().double() for t in prev]
    assert float((da.cpu().double().view(R, D) - ad.grad).abs().max()) <= 1e-2 * float(ad.grad.abs().max())
    for got, want, o in ((dg, gd.grad, off[0]), (dbe, bd.grad, off[1]), (db, ad.grad.sum(0), off[2]),
                         (dhw, wd.grad, off[3]), (dhb, hbd.grad, off[4])):
        want = want + o
        assert torch.allclose(got.cpu().double(), want, rtol=1e-3, atol=1e-3 * float(want.abs().max())), \
            float((got.cpu().double() - want).abs().max())


@pytest.mark.parametrize("V,D,n,pad", [(300, 256, 1024, 0), (256, 256, 7000, None), (5, 64, 16, None)])
def test_embedding_bwd(ops, V, D, n, pad):
    """fs2_embedding_bwd against a float64 index_add (the nn.Embedding weight gradient), padding
    row zero; deterministic: two calls bit-identical."""
    torch.manual_seed(V + n)
    tok = torch.randint(0, V, (n,))
    tok[: n // 8] = 3  # a hot row
    dy = torch.randn(n, D)
    ref = torch.zeros(V, D, dtype=torch.float64).index_add_(0, tok, dy.double())
    if pad is not None:
        ref[pad] = 0
    o1 = ops.embedding_bwd(tok.to(DEV), dy.to(DEV), V, pad)
    o2 = ops.embedding_bwd(tok.to(DEV), dy.to(DEV), V, pad)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert float((o1.cpu().double() - ref).abs().max()) <= 1e-5 * float(ref.abs().max())


@pytest.mark.parametrize("B,L,T_cut", [(4, 23, None), (3, 64, 150), (2, 300, None)])
def test_lr_backward_segmented_sum(ops, B, L, T_cut):
    """fs2_lr_backward (the LengthRegulator gather's gradient, model/modules.py:161-194 under
    autograd) against float64 autograd of the reference's expand / cat / pad: zero and long
    durations, padded phonemes, a crop below max(mel_len) (T_cut: frames past it carry no
    gradient); 1e-6 of the gradient scale, and bit-identical across calls (no atomics)."""
    torch.manual_seed(B * L)
    lens = torch.randint(1, L + 1, (B,))
    lens[0] = L
    dur = torch.randint(0, 12, (B, L)) * (torch.arange(L)[None] < lens[:, None])
    dur[0, 1] = 40
    cum, mel_len, _ = ops.lr_durations(dur.to(DEV))
    T = int(mel_len.max()) if T_cut is None else T_cut
    dy = torch.randn(B, T, 256)
    x = torch.randn(B, L, 256, dtype=torch.float64, requires_grad=True)
    rows = []
    for b in range(B):
        r = torch.cat([x[b, i].expand(int(dur[b, i]), -1) for i in range(L)], 0)
        rows.append(F.pad(r, (0, 0, 0, max(0, T - r.shape[0])))[:T])
    ref, = torch.autograd.grad(torch.stack(rows), x, dy.double())
    g1 = ops.lr_backward(dy.to(DEV), cum, L)
    g2 = ops.lr_backward(dy.to(DEV), cum, L)
    torch.cuda.synchronize()
    assert torch.equal(g1, g2)
    assert float((g1.cpu().double() - ref).abs().max()) <= 1e-6 * float(ref.abs().max())


def test_variance_embed_ex_equals_torch(ops):
    """fs2_variance_embed_ex: bucket indices equal torch.bucketize (right=False) exactly, incl.
    values on a boundary and outside the range; out = x + table[idx] exact in f32."""
    torch.manual_seed(3)
    bins = torch.linspace(-2.0, 8.0, 255)
    table = torch.randn(256, 256)
    M = 2000
    v = torch.randn(M) * 4 + 3
    v[:10] = bins[:10]  # exactly on boundaries
    v[10:20] = torch.tensor([-1e9, 1e9, -2.0, 8.0, 8.5, -2.5, 0.0, 3.0, float(bins[100]), float(bins[254])])
    x = torch.randn(M, 256)
    out, idx = ops.variance_embed_ex(x.to(DEV), v.to(DEV), bins.to(DEV), table.to(DEV))
    ref_idx = torch.bucketize(v, bins)
    assert torch.equal(idx.cpu(), ref_idx)
    assert torch.equal(out.cpu(), x + table[ref_idx])


@pytest.mark.parametrize("frame_level", [False, True])
def test_loss_fused_equals_torch(ops, frame_level, monkeypatch):
    """FastSpeech2Loss on fs2_loss_fwd / _bwd against its torch statement (FS2_LOSS_FUSED=0): the six
    losses rtol 1e-5, every prediction gradient within 1e-6 of its scale (same sign / count
    arithmetic), incl. a mel target longer than the prediction (cropped) and an exact-zero error."""
    from fs2amd.loss import FastSpeech2Loss

    torch.manual_seed(7)
    B, L, T, C = 4, 23, 57, 80
    lvl = "frame_level" if frame_level else "phoneme_level"
    pc = {"preprocessing": {"pitch": {"feature": lvl}, "energy": {"feature": "phoneme_level"}}}
    src_lens, mel_lens = torch.tensor([23, 10, 1, 17]), torch.tensor([57, 30, 3, 44])
    src_m = (torch.arange(L)[None] >= src_lens[:, None]).to(DEV)
    mel_m = (torch.arange(T)[None] >= mel_lens[:, None]).to(DEV)

    def run(fused):
        monkeypatch.setenv("FS2_LOSS_FUSED", "1" if fused else "0")
        torch.manual_seed(8)
        mel = torch.randn(B, T, C, device=DEV, requires_grad=True)
        post = torch.randn(B, T, C, device=DEV, requires_grad=True)
        PL = T if frame_level else L
        pp = torch.randn(B, PL, device=DEV, requires_grad=True)
        ep = torch.randn(B, L, device=DEV, requires_grad=True)
        ld = torch.randn(B, L, device=DEV, requires_grad=True)
        tgt = torch.randn(B, T + 9, C, device=DEV)
        with torch.no_grad():
            tgt[0, 0, 0] = mel[0, 0, 0]  # exact zero error: zero L1 gradient
        inputs = (None,) * 9 + (tgt, mel_lens.to(DEV), T + 9, torch.randn(B, PL, device=DEV),
                                torch.randn(B, L, device=DEV), torch.randint(1, 9, (B, L), device=DEV))
        preds = (mel, post, pp, ep, ld, None, src_m, mel_m, None, None)
        losses = FastSpeech2Loss(pc, None)(inputs, preds)
        (losses[0] + 0.5 * losses[2] + 0.25 * losses[5]).backward()
        return [float(l) for l in losses], [t.grad.detach().clone() for t in (mel, post, pp, ep, ld)]

    lf, gf = run(True)
    lt, gt = run(False)
    np = pytest.importorskip("numpy")
    np.testing.assert_allclose(lf, lt, rtol=1e-5)
    for a, b in zip(gf, gt):
        assert float((a - b).abs().max()) <= 1e-6 * max(1e-3, float(b.abs().max()))


@pytest.mark.parametrize("C,use_tanh,p", [(512, True, 0.5), (80, False, 0.5), (512, True, 0.0)])
def test_bn_train_fwd_bwd(ops, C, use_tanh, p):
    """fs2_bn_train_fwd / _bwd (a PostNet layer in train mode: BatchNorm1d on batch statistics with
    the running-stat update, tanh, dropout; transformer/Layers.py:92-137) against float64 autograd
    of F.batch_norm(training=True) with the kernel's keep mask (read back with gamma = 0, beta = 1):
    y within 2e-5 (f32 path) / 1e-2 (bf16 copy) of its scale, running stats rtol 1e-5, dz within
    1e-2 (bf16), dgamma / dbeta rtol 1e-4."""
    torch.manual_seed(C + int(use_tanh))
    R = 3 * 37
    z = torch.randn(R, C) * 2 + 0.5
    g, b = 1 + 0.1 * torch.randn(C), 0.1 * torch.randn(C)
    res = torch.randn(R, C)
    seed = torch.tensor([77], dtype=torch.int64, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yb, yf, mean, rstd = ops.bn_train_fwd(z.to(DEV), g.to(DEV), b.to(DEV), 1e-5, 0.1, rm, rv, use_tanh, p, seed, 3,
                                          residual=None if use_tanh else res.to(DEV), want_bf16=True, want_f32=True)
    if p > 0:
        kb, kf, _, _ = ops.bn_train_fwd(z.to(DEV), torch.zeros(C, device=DEV), torch.ones(C, device=DEV), 1e-5, 0.1,
                                        None, None, True, p, seed, 3, want_bf16=False, want_f32=True)
        keep = (kf != 0).cpu()
        assert abs(float(keep.float().mean()) - (1 - p)) < 0.02
    else:
        keep = torch.ones(R, C, dtype=torch.bool)
    zd = z.double().requires_grad_()
    gd, bd = g.double().requires_grad_(), b.double().requires_grad_()
    rmr, rvr = torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    v = F.batch_norm(zd, rmr, rvr, gd, bd, True, 0.1, 1e-5)
    if use_tanh:
        v = torch.tanh(v)
    ref = v * keep / (1 - p) + (0 if use_tanh else res.double())
    torch.cuda.synchronize()
    sc = float(ref.abs().max())
    assert float((yf.cpu().double() - ref).abs().max()) <= 2e-5 * sc
    assert float((yb.cpu().double() - ref).abs().max()) <= 1e-2 * sc
    assert torch.allclose(rm.cpu().double(), rmr, rtol=1e-5, atol=1e-6)
    assert torch.allclose(rv.cpu().double(), rvr, rtol=1e-5, atol=1e-6)
    dy = torch.randn(R, C)
    ref.backward(dy.double())
    dz, dg, dbe = ops.bn_train_bwd(dy.to(DEV), z.to(DEV), g.to(DEV), b.to(DEV), mean, rstd, use_tanh, p, seed, 3)
    torch.cuda.synchronize()
    assert float((dz.cpu().double() - zd.grad).abs().max()) <= 1e-2 * float(zd.grad.abs().max())
    assert torch.allclose(dg.cpu().double(), gd.grad, rtol=1e-4, atol=1e-4 * float(gd.grad.abs().max()))
    assert torch.allclose(dbe.cpu().double(), bd.grad, rtol=1e-4, atol=1e-4 * float(bd.grad.abs().max()))


@pytest.mark.parametrize("capturable,wd", [(True, 0.0), (False, 0.01)])
def test_adam_flat_equals_torch(ops, capturable, wd):
    """fs2_adam_flat (clip_grad_norm_ + Adam over the flat gradient buffer, two launches) against
    nn.utils.clip_grad_norm_ + torch.optim.Adam(fused=True) over 3 steps, clipping active on the
    first: parameters and exp_avg / exp_avg_sq within 1e-5 relative (+1e-7), steps equal, the
    clipped gradients written back like clip_grad_norm_'s."""
    import copy
    from fs2amd.optimizer import ScheduledOptim

    torch.manual_seed(9)
    shapes = [(33,), (256, 256), (80, 512, 5), (7,), (1024,)]
    ps = [torch.randn(s, device=DEV) * 0.1 for s in shapes]
    tc = {"optimizer": {"betas": [0.9, 0.98], "eps": 1e-9, "weight_decay": wd, "warm_up_step": 4000,
                        "anneal_steps": [], "anneal_rate": 0.3, "grad_acc_step": 1, "grad_clip_thresh": 1.0}}
    mc = {"transformer": {"encoder_hidden": 256}}

    class M(torch.nn.Module):
        def __init__(self, init):
            super().__init__()
            self.ps = torch.nn.ParameterList([torch.nn.Parameter(t.clone()) for t in init])

    ma, mb = M(ps), M(ps)
    oa = ScheduledOptim(ma, tc, mc, 0, capturable=capturable)
    ob = ScheduledOptim(mb, tc, mc, 0, capturable=capturable)
    # the trainer's layout: each gradient starts on a 16-byte boundary, zero gaps after the
    # ragged sizes (33, 7) -- exercises the kernel's vector groups, ragged ends and gaps
    offs, n = [], 0
    for p in ma.parameters():
        offs.append(n)
        n += (p.numel() + 3) // 4 * 4
    flat = torch.zeros(n, device=DEV)
    for p, off in zip(ma.parameters(), offs):
        p.grad = flat[off:off + p.numel()].view_as(p)
    for step in range(3):
        gs = [torch.randn(s, device=DEV) * (3.0 if step == 0 else 0.001) for s in shapes]
        for p, g in zip(ma.parameters(), gs):
            p.grad.copy_(g)
        for p, g in zip(mb.parameters(), gs):
            p.grad = g.clone()
        oa._update_learning_rate()
        oa.flat_step(flat, list(ma.parameters()), 1.0)
        ob._update_learning_rate()
        torch.nn.utils.clip_grad_norm_(mb.parameters(), 1.0)
        ob._optimizer.step()
        torch.cuda.synchronize()
        for pa, pb in zip(ma.parameters(), mb.parameters()):
            assert torch.allclose(pa.grad, pb.grad, rtol=1e-5, atol=1e-7)
            assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-7), step
            sa, sb = oa._optimizer.state[pa], ob._optimizer.state[pb]
            assert torch.allclose(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-9)
            assert torch.allclose(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-12)
            assert float(sa["step"]) == float(sb["step"]) == step + 1
        used = torch.zeros(n, dtype=torch.bool, device=DEV)
        for p, off in zip(ma.parameters(), offs):
            used[off:off + p.numel()] = True
        assert not flat[~used].any()


def test_deferred_reductions_bit_identical(ops):
    """defer= (partials only, one fs2_reduce_batch_launch afterwards) equals the immediate finishes
    for fs2_conv_wgrad (Q|K|V parts + biases, a k=9 conv) and fs2_res_ln_bwd within f32 rounding of
    the different (but fixed) summation order: 1e-6 of each output's scale; two deferred runs are
    bit-identical."""
    torch.manual_seed(10)
    B, T = 3, 70
    dy = torch.randn(B, T, 768, device=DEV)
    x = torch.randn(B, T, 256, device=DEV).to(torch.bfloat16)
    mk = lambda: ([torch.ones(256, 256, device=DEV) for _ in range(3)], [torch.ones(256, device=DEV) for _ in range(3)])
    p1, p2 = mk(), mk()
    ops.conv_wgrad(dy, x, 1, 0, parts=p1, accumulate=True)
    q = []
    ops.conv_wgrad(dy, x, 1, 0, parts=p2, accumulate=True, defer=q)
    dy9 = torch.randn(B, T, 1024, device=DEV).to(torch.bfloat16)
    w9a, b9a = ops.conv_wgrad(dy9, x, 9, 4, want_db=True)
    w9b, b9b = torch.zeros(1024, 256, 9, device=DEV), torch.zeros(1024, device=DEV)
    ops.conv_wgrad(dy9, x, 9, 4, dw=w9b, db=b9b, defer=q)
    a = torch.randn(B, T, 256, device=DEV)
    lens = torch.tensor([70, 33, 1], device=DEV)
    g = torch.rand(256, device=DEV) + 0.5
    y, yb, xh, rs = ops.res_ln_fwd(a, torch.randn_like(a), g, torch.zeros(256, device=DEV), 1e-5, lens)
    dyl = torch.randn_like(a)
    _, _, ga, ba, bia = ops.res_ln_bwd(dyl, xh, rs, g, lens)
    gb, bb, bib = (torch.zeros(256, device=DEV) for _ in range(3))
    ops.res_ln_bwd(dyl, xh, rs, g, lens, dgamma=gb, dbeta=bb, dbias=bib, defer=q)
    assert len(q) == 5
    ops.reduce_flush(q, dy)
    w9c = torch.zeros_like(w9b)
    ops.conv_wgrad(dy9, x, 9, 4, dw=w9c, defer=q)
    ops.reduce_flush(q, dy)
    torch.cuda.synchronize()
    close = lambda u, v: float((u - v).abs().max()) <= 1e-6 * max(1.0, float(u.abs().max()))
    for t1, t2 in zip(p1[0] + p1[1], p2[0] + p2[1]):
        assert close(t1, t2)
    assert close(w9a, w9b) and close(b9a, b9b) and torch.equal(w9b, w9c)
    assert close(ga, gb) and close(ba, bb) and close(bia, bib)


@pytest.mark.parametrize("B,Lx,spk,emo", [(16, 64, True, True), (5, 37, True, True), (7, 20, False, True),
                                          (3, 11, True, False)])
def test_cond_fn_fwd_bwd(ops, B, Lx, spk, emo):
    """training.CondFn (fs2_cond_vectors + the two adds; backward fs2_cond_bwd): y = x + spk[s] +
    relu(W cat(emo[e], aro[a], val[v]) + b) (model/fastspeech2.py:101-110) and the gradients of x,
    the four tables, W and b against float64 autograd; repeated ids (their rows summed), relu-dead
    channels (bias shifted negative), accumulation into existing gradients through the sink path's
    fs2_cond_bwd call; two backward calls bit-identical."""
    from fs2amd.training import CondFn

    torch.manual_seed(B * 100 + Lx)
    D = 256
    x = torch.randn(B, Lx, D)
    ts = torch.randn(5, D)
    te, ta, tv = torch.randn(7, 128), torch.randn(3, 64), torch.randn(4, 64)
    W, bl = torch.randn(D, 256) / 16, torch.randn(D) - 0.5
    s_id = torch.randint(0, 5, (B,))
    e_id, a_id, v_id = torch.randint(0, 7, (B,)), torch.randint(0, 3, (B,)), torch.randint(0, 4, (B,))
    dev = lambda t: t.to(DEV).contiguous()
    params = [dev(t).requires_grad_() if on else None
              for t, on in ((ts, spk), (te, emo), (ta, emo), (tv, emo), (W, emo), (bl, emo))]
    xg = dev(x).requires_grad_()
    y = CondFn.apply(xg, dev(s_id) if spk else None, dev(e_id) if emo else None, dev(a_id) if emo else None,
                     dev(v_id) if emo else None, *params)
    dy = torch.randn(B, Lx, D)
    y.backward(dev(dy))
    torch.cuda.synchronize()
    # float64 reference
    ref_p = [t.double().requires_grad_() if on else None
             for t, on in ((ts, spk), (te, emo), (ta, emo), (tv, emo), (W, emo), (bl, emo))]
    xd = x.double().requires_grad_()
    r = xd
    if spk:
        r = r + ref_p[0][s_id].unsqueeze(1)
    if emo:
        cat = torch.cat([ref_p[1][e_id], ref_p[2][a_id], ref_p[3][v_id]], -1)
        r = r + torch.relu(cat @ ref_p[4].t() + ref_p[5]).unsqueeze(1)
    r.backward(dy.double())
    assert float((y.detach().cpu().double() - r.detach()).abs().max()) <= 1e-5 * float(r.detach().abs().max())
    assert torch.equal(xg.grad.cpu(), dy)
    for got, want in zip(params, ref_p):
        if got is None:
            continue
        g = got.grad.cpu().double()
        assert float((g - want.grad).abs().max()) <= 2e-5 * max(1.0, float(want.grad.abs().max())), \
            (tuple(got.shape), float((g - want.grad).abs().max()))
    # accumulation (the sink path): into existing gradients, deterministic
    if emo:
        dt = torch.zeros(ta.shape, device=DEV)
        dw = [torch.full_like(W, 0.5, device=DEV) for _ in range(2)]
        for k in range(2):
            ops.cond_bwd(dev(dy), dev(s_id) if spk else None, params[0], dev(e_id), dev(a_id), dev(v_id),
                         params[1], params[2], params[3], params[4],
                         ops.cond_vectors(dev(s_id) if spk else None, params[0], dev(e_id), dev(a_id), dev(v_id),
                                          params[1], params[2], params[3], params[4], params[5], D)[1].detach(),
                         d_aro=dt if k == 0 else None, d_w=dw[k])
        torch.cuda.synchronize()
        assert torch.equal(dw[0], dw[1])
        assert torch.allclose(dw[0].cpu().double(), ref_p[4].grad + 0.5, rtol=1e-5, atol=2e-5 * float(ref_p[4].grad.abs().max()))
        assert torch.allclose(dt.cpu().double(), ref_p[2].grad, rtol=1e-5, atol=2e-5 * float(ref_p[2].grad.abs().max()))
