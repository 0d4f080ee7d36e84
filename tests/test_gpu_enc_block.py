"""fs2_enc_attn_block — the encoder FFT block's attention sub-layer in one launch
(transformer/SubLayers.py:29-57 + Modules.py:14-25 + Layers.py:25), bf16.

* against the three launches it replaces (fs2_conv1d Q|K|V, fs2_attention, fs2_conv1d fc +
  residual + LayerNorm with the row mask) on the same operands: Q|K|V and the attention output
  round identically (same MFMA k order, attn_bf16_kernel's per-wave arithmetic), only the
  LayerNorm statistics are summed in another order -> within 2 bf16 ulps;
* against a float64 statement of the sub-layer on the same bf16 weights: bf16 tolerance;
* padded rows (t >= len) exactly zero; lengths 0, 1, L; L = 64, 37, 1.
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


def _weights(g, D=256):
    wqkv = torch.randn(3 * D, D, device=DEV, generator=g) / D ** 0.5
    bqkv = 0.1 * torch.randn(3 * D, device=DEV, generator=g)
    wfc = torch.randn(D, D, device=DEV, generator=g) / D ** 0.5
    bfc = 0.1 * torch.randn(D, device=DEV, generator=g)
    gam = 1 + 0.1 * torch.randn(D, device=DEV, generator=g)
    bet = 0.1 * torch.randn(D, device=DEV, generator=g)
    return wqkv, bqkv, wfc, bfc, gam, bet


def _ref64(x, lens, wqkv, bqkv, wfc, bfc, gam, bet, eps=1e-5, H=2, dk=128):
    """float64 statement of the sub-layer on the bf16-rounded weights / input."""
    xd = x.double()
    B, L, D = x.shape
    qkv = xd @ wqkv.to(torch.bfloat16).double().t() + bqkv.double()
    q, k, v = qkv.split(D, -1)
    heads = lambda t: t.view(B, L, H, dk).transpose(1, 2)
    s = heads(q) @ heads(k).transpose(-1, -2) / dk ** 0.5
    keymask = torch.arange(L, device=DEV)[None, :] >= lens[:, None]
    s = s.masked_fill(keymask[:, None, None, :], float("-inf"))
    a = torch.softmax(s, -1).nan_to_num(0.0)
    o = (a @ heads(v)).transpose(1, 2).reshape(B, L, D)
    y = o @ wfc.to(torch.bfloat16).double().t() + bfc.double() + xd
    y = torch.nn.functional.layer_norm(y, (D,), gam.double(), bet.double(), eps)
    return y.masked_fill(keymask[..., None], 0.0)


@pytest.mark.parametrize("B,L,seed", [(64, 64, 1), (5, 37, 2), (3, 1, 3), (7, 64, 4)])
def test_enc_attn_block_matches_three_launches_and_float64(gpu, B, L, seed):
    ops, Lb = gpu
    g = torch.Generator(device=DEV).manual_seed(seed)
    wqkv, bqkv, wfc, bfc, gam, bet = _weights(g)
    x = torch.randn(B, L, 256, device=DEV, generator=g).to(torch.bfloat16)
    lens = torch.randint(0, L + 1, (B,), generator=torch.Generator().manual_seed(seed)).to(DEV)
    lens[0] = L
    if B > 2:
        lens[1], lens[2] = 0, 1
    ln = (gam, bet, 1e-5)
    got = ops.enc_attn_block(x, lens, ops.pack_frag_rows(wqkv), bqkv, ops.pack_frag_rows(wfc), bfc, ln, 2, 128,
                             128 ** 0.5)
    qkv = ops.conv1d(x, ops.pack_conv_weight(wqkv, Lb.FS2_BF16), bqkv, cin=256, ks=1, pad=0, compute=Lb.FS2_BF16,
                     epilogue=Lb.EPI_BIAS, out_dtype=Lb.FS2_BF16)
    att = ops.attention(qkv, lens, 2, 128, 128 ** 0.5)
    three = ops.conv1d(att, ops.pack_conv_weight(wfc, Lb.FS2_BF16), bfc, cin=256, ks=1, pad=0, compute=Lb.FS2_BF16,
                       epilogue=Lb.EPI_RES_LN, out_dtype=Lb.FS2_BF16, residual=x, ln=ln, lens=lens)
    torch.cuda.synchronize()
    pad = torch.arange(L, device=DEV)[None, :] >= lens[:, None]
    assert bool((got[pad] == 0).all()), "padded rows must be zero"
    d = (got.float() - three.float()).abs()
    ulp = three.float().abs().clamp(min=2 ** -6) * 2 ** -7
    assert bool((d <= 2 * ulp).all()), float((d - 2 * ulp).max())
    ref = _ref64(x, lens, wqkv, bqkv, wfc, bfc, gam, bet)
    err = (got.double() - ref).abs()
    assert float(err.max()) <= 0.06 and float(err.mean()) <= 4e-3, (float(err.max()), float(err.mean()))


def test_enc_attn_block_rejects(gpu):
    ops, Lb = gpu
    g = torch.Generator(device=DEV).manual_seed(9)
    wqkv, bqkv, wfc, bfc, gam, bet = _weights(g)
    x = torch.randn(2, 65, 256, device=DEV, generator=g).to(torch.bfloat16)
    lens = torch.tensor([65, 3], device=DEV)
    with pytest.raises(RuntimeError):  # L > 64: the three-launch path covers it
        ops.enc_attn_block(x, lens, ops.pack_frag_rows(wqkv), bqkv, ops.pack_frag_rows(wfc), bfc, (gam, bet, 1e-5), 2,
                           128, 128 ** 0.5)
    with pytest.raises(AssertionError):
        ops.enc_attn_block(x.float(), lens, ops.pack_frag_rows(wqkv), bqkv, ops.pack_frag_rows(wfc), bfc,
                           (gam, bet, 1e-5), 2, 128, 128 ** 0.5)


@pytest.mark.parametrize("B,L,seed", [(64, 64, 5), (5, 37, 6), (3, 1, 7)])
def test_enc_embed_attn_block_equals_embed_then_block(gpu, B, L, seed):
    """fs2_enc_embed_attn_block (the first encoder block builds x = bf16(emb[tok] + pe) itself and
    writes both masks) equals fs2_embed_pe + fs2_enc_attn_block BIT-EXACTLY, the masks equal
    fs2_length_masks, and an out-of-vocabulary id gives a NaN input row and counts once."""
    ops, Lb = gpu
    g = torch.Generator(device=DEV).manual_seed(seed)
    wqkv, bqkv, wfc, bfc, gam, bet = _weights(g)
    vocab = 50
    table = torch.randn(vocab, 256, device=DEV, generator=g)
    pe = torch.randn(L + 3, 256, device=DEV, generator=g)
    tok = torch.randint(0, vocab, (B, L), device=DEV, generator=g)
    lens = torch.randint(0, L + 1, (B,), generator=torch.Generator().manual_seed(seed)).to(DEV)
    lens[0] = L
    mel_lens = torch.randint(-2, 90, (B,), generator=torch.Generator().manual_seed(seed + 1)).to(DEV)
    ln = (gam, bet, 1e-5)
    wq, wf = ops.pack_frag_rows(wqkv), ops.pack_frag_rows(wfc)
    x = ops.embed_pe(tok, table, pe, Lb.FS2_BF16)
    two = ops.enc_attn_block(x, lens, wq, bqkv, wf, bfc, ln, 2, 128, 128 ** 0.5)
    sm = torch.empty(B, L, device=DEV, dtype=torch.bool)
    mm = torch.empty(B, 77, device=DEV, dtype=torch.bool)
    one = ops.enc_attn_block(None, lens, wq, bqkv, wf, bfc, ln, 2, 128, 128 ** 0.5, embed=(tok, table, pe),
                             masks=(sm, mel_lens, mm))
    torch.cuda.synchronize()
    assert torch.equal(one, two), float((one.float() - two.float()).abs().max())
    assert torch.equal(sm, ops.length_mask(lens, L)) and torch.equal(mm, ops.length_mask(mel_lens, 77))
    if B > 1 and L > 1:
        bad = ops.bad_id_counter(torch.device(DEV))
        before = int(bad.item())
        tok[1, 0] = vocab + 3
        lens[1] = L
        out = ops.enc_attn_block(None, lens, wq, bqkv, wf, bfc, ln, 2, 128, 128 ** 0.5, embed=(tok, table, pe))
        torch.cuda.synchronize()
        assert int(bad.item()) == before + 1
        assert bool(torch.isnan(out[1].float()).any()) and not bool(torch.isnan(out[0].float()).any())
        bad.zero_()


@pytest.mark.parametrize("B,L,seed", [(64, 64, 11), (13, 37, 12), (3, 1, 13)])
def test_enc_attn_block_head_split_equals_one_workgroup(gpu, B, L, seed, monkeypatch):
    """The head-split form (two workgroups per utterance, f32 fc halves summed head 0 + head 1 by
    the last arriver through the split-K workspace) against the one-workgroup form: the same
    Q|K|V, attention and o; the fc sum regrouped (k 0..127 + k 128..255 instead of one chain) ->
    within 2 bf16 ulps; run twice (the arrival counters must be left zero); B not a multiple of 8."""
    ops, Lb = gpu
    g = torch.Generator(device=DEV).manual_seed(seed)
    wqkv, bqkv, wfc, bfc, gam, bet = _weights(g)
    x = torch.randn(B, L, 256, device=DEV, generator=g).to(torch.bfloat16)
    lens = torch.randint(0, L + 1, (B,), generator=torch.Generator().manual_seed(seed)).to(DEV)
    lens[0] = L
    ln = (gam, bet, 1e-5)
    wq, wf = ops.pack_frag_rows(wqkv), ops.pack_frag_rows(wfc)
    monkeypatch.setenv("FS2_ENC_HALF", "0")
    one = ops.enc_attn_block(x, lens, wq, bqkv, wf, bfc, ln, 2, 128, 128 ** 0.5)
    monkeypatch.setenv("FS2_ENC_HALF", "1")
    two = ops.enc_attn_block(x, lens, wq, bqkv, wf, bfc, ln, 2, 128, 128 ** 0.5)
    again = ops.enc_attn_block(x, lens, wq, bqkv, wf, bfc, ln, 2, 128, 128 ** 0.5)
    torch.cuda.synchronize()
    assert torch.equal(two, again)
    assert int(ops.splitk_workspace(torch.device(DEV))[:4096].view(torch.int32)[:B].abs().sum()) == 0
    d = (two.float() - one.float()).abs()
    ulp = one.float().abs().clamp(min=2 ** -6) * 2 ** -7
    assert bool((d <= 2 * ulp).all()), float((d - 2 * ulp).max())


def test_enc_embed_block_conditioning_tiles_equal_cond_vectors(gpu):
    """The conditioning vectors computed by extra workgroups of the first encoder block's launch
    (cond.h tiles on otherwise idle CUs) equal fs2_cond_vectors BIT-EXACTLY (the same tile code),
    ids clamped as there; the block output is unchanged by them."""
    ops, Lb = gpu
    g = torch.Generator(device=DEV).manual_seed(21)
    B, L = 13, 40
    wqkv, bqkv, wfc, bfc, gam, bet = _weights(g)
    table = torch.randn(30, 256, device=DEV, generator=g)
    pe = torch.randn(L, 256, device=DEV, generator=g)
    tok = torch.randint(0, 30, (B, L), device=DEV, generator=g)
    lens = torch.randint(1, L + 1, (B,), generator=torch.Generator().manual_seed(3)).to(DEV)
    spk_t = torch.randn(10, 256, device=DEV, generator=g)
    emo_t, aro_t, val_t = (torch.randn(n, d, device=DEV, generator=g) for n, d in ((5, 128), (7, 64), (7, 64)))
    lin_w = torch.randn(256, 256, device=DEV, generator=g) / 16
    lin_b = torch.randn(256, device=DEV, generator=g)
    ids = lambda n, hi: torch.randint(-1, hi + 1, (n,), device=DEV, generator=g)
    spk, emo, aro, val = ids(B, 10), ids(B, 5), ids(B, 7), ids(B, 7)
    ln = (gam, bet, 1e-5)
    wq, wf = ops.pack_frag_rows(wqkv), ops.pack_frag_rows(wfc)
    out, sv, ev = ops.enc_attn_block(None, lens, wq, bqkv, wf, bfc, ln, 2, 128, 128 ** 0.5, embed=(tok, table, pe),
                                     cond=(spk, spk_t, emo, aro, val, emo_t, aro_t, val_t, lin_w, lin_b))
    plain = ops.enc_attn_block(None, lens, wq, bqkv, wf, bfc, ln, 2, 128, 128 ** 0.5, embed=(tok, table, pe))
    rs, re = ops.cond_vectors(spk, spk_t, emo, aro, val, emo_t, aro_t, val_t, lin_w, lin_b, 256)
    torch.cuda.synchronize()
    assert torch.equal(sv, rs) and torch.equal(ev, re)
    assert torch.equal(out, plain)
