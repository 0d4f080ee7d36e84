"""fs2_ffn — the fused PositionwiseFeedForward (conv-k9 + ReLU + conv-k1 + residual + LayerNorm +
mask in one launch, transformer/SubLayers.py:85-93 + Layers.py:28).

* against a float64 PyTorch statement of the same op on the same bf16 operands (the hidden f is
  rounded to bf16 exactly where the two-launch path stores it), bf16 tolerance;
* against the two fs2_conv1d launches it replaces (same bf16 rounding points; only the f32
  summation order of the k=9 product differs);
* packed rows (SeqLayout) bit-identical to padded rows: each output row depends only on its own
  input rows and the per-row k order, not on where the 112-row tile boundaries fall;
* ragged lengths 0 / 1 / < the 4-row tap reach / exact tile multiples, row counts that are not
  multiples of 112, a padded launch with speaker / emotion vectors;
* the split-hidden form (nsplit 2 / 4 workgroups per tile, partials summed by the last arriver):
  against float64 and the unsplit launch, bit-identical across repeated launches (fixed split
  order, self-resetting counters), packed == padded at equal nsplit, invalid splits refused.
"""
import numpy as np
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


def _weights(ops, L, F=1024, ks=9, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    w1 = torch.randn(F, 256, ks, device=DEV, generator=g) / (256 * ks) ** 0.5
    w2 = torch.randn(256, F, 1, device=DEV, generator=g) / F ** 0.5
    b1 = 0.1 * torch.randn(F, device=DEV, generator=g)
    b2 = 0.1 * torch.randn(256, device=DEV, generator=g)
    ln = (1 + 0.1 * torch.randn(256, device=DEV, generator=g), 0.1 * torch.randn(256, device=DEV, generator=g), 1e-5)
    return dict(w1=w1, w2=w2, b1=b1, b2=b2, ln=ln, p1=ops.pack_conv_weight(w1, L.FS2_BF16),
                p2=ops.pack_conv_weight(w2, L.FS2_BF16), w12=ops.pack_ffn_weights(w1, w2), ks=ks)


def _ref(x, lens, W, addvecs=()):
    """float64 statement: per-sequence conv (zero taps outside [0, T)), f rounded to bf16 like the
    stored hidden, LN(f w2^T + b2 + x), rows t >= len -> 0, + addvecs."""
    ks = W["ks"]
    xd = x.double()
    w1 = W["w1"].to(torch.bfloat16).double()
    w2 = W["w2"].to(torch.bfloat16).double()[:, :, 0]
    f = torch.nn.functional.conv1d(xd.transpose(1, 2), w1, W["b1"].double(), padding=(ks - 1) // 2).transpose(1, 2)
    f = torch.relu(f).to(torch.bfloat16).double()
    y = f @ w2.t() + W["b2"].double() + xd
    g, b, eps = W["ln"]
    y = torch.nn.functional.layer_norm(y, (256,), g.double(), b.double(), eps)
    T = x.shape[1]
    if lens is not None:
        y = y * (torch.arange(T, device=DEV)[None, :, None] < lens[:, None, None])
    for v in addvecs:
        y = y + v.double()[:, None, :]
    return y


def _pack(lay, x):
    """padded [B, T, C] -> packed [B*T, C] capacity rows (rows past cu[B] zero)."""
    rm = lay.rowmap.long()
    out = x.new_zeros(lay.capacity, x.shape[-1])
    ok = rm >= 0
    out[rm[ok]] = x.reshape(-1, x.shape[-1])[ok]
    return out


def _x(B, T, lens, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    valid = (torch.arange(T, device=DEV)[None, :] < lens[:, None])[..., None]
    return (torch.randn(B, T, 256, device=DEV, generator=g) * valid).to(torch.bfloat16)


@pytest.mark.parametrize("B,T,seed", [(8, 130, 1), (3, 37, 2), (40, 300, 3)])
def test_ffn_matches_float64(gpu, B, T, seed):
    ops, L = gpu
    W = _weights(ops, L, seed=seed)
    rng = np.random.default_rng(seed)
    lens_l = rng.integers(0, T + 1, B).tolist()
    lens_l[0] = T
    if B > 2:
        lens_l[1], lens_l[2] = 1, 3  # shorter than the taps' reach on both sides
    lens = torch.tensor(lens_l, dtype=torch.int64, device=DEV)
    x = _x(B, T, lens, seed)
    got = ops.ffn(x, W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], lens=lens)
    ref = _ref(x, lens, W)
    err = (got.double() - ref).abs()
    # bf16 output rounding (|y| <~ 4: 1.6e-2) plus rare 1-ulp flips of a bf16 hidden value
    assert float(err.max()) <= 3e-2, float(err.max())
    assert float(err.mean()) <= 2e-3, float(err.mean())


def test_ffn_matches_two_launch_path(gpu):
    ops, L = gpu
    B, T = 64, 430
    W = _weights(ops, L, seed=7)
    g = torch.Generator(device="cpu").manual_seed(7)
    lens = torch.randint(200, T + 1, (B,), generator=g).to(DEV)
    x = _x(B, T, lens, 7)
    fused = ops.ffn(x, W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], lens=lens)
    kw = dict(compute=L.FS2_BF16, out_dtype=L.FS2_BF16)
    f = ops.conv1d(x, W["p1"], W["b1"], cin=256, ks=9, pad=4, epilogue=L.EPI_BIAS_RELU, **kw)
    two = ops.conv1d(f, W["p2"], W["b2"], cin=1024, ks=1, pad=0, epilogue=L.EPI_RES_LN, residual=x, ln=W["ln"],
                     lens=lens, **kw)
    d = (fused.float() - two.float()).abs()
    assert float(d.max()) <= 3e-2 and float(d.mean()) <= 1e-3, (float(d.max()), float(d.mean()))


@pytest.mark.parametrize("tile_rows,nsplit", [(112, 1), (112, 2), (112, 4), (96, 2), (64, 1), (64, 4)])
@pytest.mark.parametrize("lens_l,T", [([37, 0, 130, 1, 64, 129, 130, 5], 130),
                                      ([430] * 3 + [2, 3, 4, 111, 112, 113, 224, 225], 430)])
def test_ffn_packed_equals_padded(gpu, lens_l, T, tile_rows, nsplit):
    ops, L = gpu
    W = _weights(ops, L, seed=11)
    lens = torch.tensor(lens_l, dtype=torch.int64, device=DEV)
    B = len(lens_l)
    x = _x(B, T, lens, 11)
    lay = ops.SeqLayout(lens, T)
    rm = lay.rowmap.long()
    ok = rm >= 0
    xp = x.new_zeros(lay.capacity, 256)
    xp[rm[ok]] = x.reshape(-1, 256)[ok]
    kw = dict(ks=9, pad=4, ln=W["ln"], nsplit=nsplit, tile_rows=tile_rows)
    ref = ops.ffn(x, W["w12"], W["b1"], W["b2"], lens=lens, **kw)
    got = ops.ffn(xp, W["w12"], W["b1"], W["b2"], layout=lay, **kw)
    torch.cuda.synchronize()
    R = int(lay.cu[-1])
    assert torch.equal(got[:R], ref.reshape(-1, 256)[ok])
    assert not torch.isnan(got[:R].float()).any()


def test_ffn_addvecs_and_narrow_hidden(gpu):
    """Padded rows with the speaker / emotion adds of the last encoder block, F = 512 (two chunks)
    and a k=3 first conv."""
    ops, L = gpu
    B, T = 5, 61
    W = _weights(ops, L, F=512, ks=3, seed=13)
    lens = torch.tensor([61, 17, 0, 2, 40], dtype=torch.int64, device=DEV)
    x = _x(B, T, lens, 13)
    g = torch.Generator(device=DEV).manual_seed(14)
    a1, a2 = torch.randn(B, 256, device=DEV, generator=g), torch.randn(B, 256, device=DEV, generator=g)
    got = ops.ffn(x, W["w12"], W["b1"], W["b2"], ks=3, pad=1, ln=W["ln"], lens=lens, addvec1=a1, addvec2=a2)
    ref = _ref(x, lens, W, (a1, a2))
    err = (got.double() - ref).abs()
    assert float(err.max()) <= 5e-2 and float(err.mean()) <= 3e-3, (float(err.max()), float(err.mean()))


def test_ffn_rejects_bad_shapes(gpu):
    ops, L = gpu
    W = _weights(ops, L, seed=1)
    x = torch.zeros(2, 8, 256, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):  # out aliasing x: other tiles re-read x rows
        ops.ffn(x, W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], out=x)
    with pytest.raises(TypeError):
        ops.ffn(x.float(), W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"])
    with pytest.raises(AssertionError):  # w_1 | w_2 buffer of another shape
        ops.ffn(x, W["w12"][:-1], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"])


@pytest.mark.parametrize("F,ks,nsplit,tile_rows", [(1024, 9, 2, 112), (1024, 9, 4, 112), (512, 3, 2, 112),
                                                   (1024, 9, 4, 64), (1024, 9, 2, 64), (1024, 9, 1, 64),
                                                   (1024, 9, 2, 96)])
@pytest.mark.parametrize("packed", [False, True])
def test_ffn_split_hidden(gpu, F, ks, nsplit, tile_rows, packed):
    """Split-hidden fs2_ffn: encoder-like padded rows with lens + speaker / emotion vectors, or
    packed rows (rows_dev: tiles past the active rows exit before touching a counter)."""
    ops, L = gpu
    B, T = 37, 111
    W = _weights(ops, L, F=F, ks=ks, seed=21 + nsplit)
    g = torch.Generator(device="cpu").manual_seed(nsplit)
    lens = torch.randint(0, T + 1, (B,), generator=g)
    lens[0], lens[1], lens[2] = T, 1, 0
    lens = lens.to(DEV)
    x = _x(B, T, lens, 5)
    pad = (ks - 1) // 2
    kw = dict(ks=ks, pad=pad, ln=W["ln"], tile_rows=tile_rows)
    if packed:
        lay = ops.SeqLayout(lens, T)
        rm = lay.rowmap.long()
        ok = rm >= 0
        xp = x.new_zeros(lay.capacity, 256)
        xp[rm[ok]] = x.reshape(-1, 256)[ok]
        outs = [ops.ffn(xp, W["w12"], W["b1"], W["b2"], layout=lay, nsplit=nsplit, **kw) for _ in range(4)]
        one = ops.ffn(xp, W["w12"], W["b1"], W["b2"], layout=lay, nsplit=1, ks=ks, pad=pad, ln=W["ln"])
        R = int(lay.cu[-1])
        got, one = outs[0][:R], one[:R]
        ref = _ref(x, lens, W).reshape(-1, 256)[ok]
        outs = [o[:R] for o in outs]
    else:
        a1 = torch.randn(B, 256, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
        outs = [ops.ffn(x, W["w12"], W["b1"], W["b2"], lens=lens, addvec1=a1, nsplit=nsplit, **kw) for _ in range(4)]
        one = ops.ffn(x, W["w12"], W["b1"], W["b2"], lens=lens, addvec1=a1, nsplit=1, ks=ks, pad=pad, ln=W["ln"])
        got = outs[0]
        ref = _ref(x, lens, W, (a1,))
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, got)  # fixed summation order, counters reset themselves
    err = (got.double() - ref).abs()
    assert float(err.max()) <= 5e-2 and float(err.mean()) <= 2e-3, (float(err.max()), float(err.mean()))
    d = (got.float() - one.float()).abs()
    assert float(d.max()) <= 3e-2 and float(d.mean()) <= 1e-3, (float(d.max()), float(d.mean()))


def test_ffn_split_rejects(gpu):
    ops, L = gpu
    x = torch.zeros(2, 8, 256, device=DEV, dtype=torch.bfloat16)
    W = _weights(ops, L, F=512, ks=3, seed=1)
    with pytest.raises(RuntimeError):  # 4 splits of a 2-chunk hidden
        ops.ffn(x, W["w12"], W["b1"], W["b2"], ks=3, pad=1, ln=W["ln"], nsplit=4)
    with pytest.raises(RuntimeError):  # not a power of two
        ops.ffn(x, W["w12"], W["b1"], W["b2"], ks=3, pad=1, ln=W["ln"], nsplit=3)


def test_ffn_form_rule(gpu):
    ops, L = gpu
    assert ops.ffn_form(24883, 1024) == (112, 1)  # cfg2 decoder: 223 tiles fill the chip
    tr, ns = ops.ffn_form(4096, 1024)            # encoder: 37 tiles of 112 -> a split form
    assert ns > 1 and -(-4096 // tr) * ns <= ops.FFN_SLOTS
    for rows in (1, 500, 4096, 11141, 24883, 200000):
        tr, ns = ops.ffn_form(rows, 1024)
        assert tr in (112, 96, 64) and ns in (1, 2, 4) and (tr != 96 or ns == 2)
        assert ns == 1 or 4096 + -(-rows // tr) * ns * ops.ffn_part_bytes(tr) <= ops.SPLITK_WS_BYTES
    with ops.splitk_enabled(False):
        assert ops.ffn_form(4096, 1024) == (112, 1)
    # a free-running cfg2 decoder (~9-12k rows): 96-row tiles x 2 hidden splits (~230 workgroups)
    assert ops.ffn_form(10240, 1024) == (96, 2) and ops.ffn_form(11264, 1024) == (96, 2)


@pytest.mark.parametrize("B,T,seed", [(64, 180, 71), (8, 130, 72), (3, 37, 73)])
def test_ffn_pre_packed_split_96(gpu, B, T, seed):
    """The free-running decoder's form: packed rows, 96-row tiles x 2 hidden splits, the fc + residual
    + LN prologue computed by both splits of a tile (round 6). Against the unsplit 112-row PRE launch
    (the same h up to the prologue's per-tile halo rounding; the split partials summed in split
    order: within 2 bf16 ulps) and a float64 statement within the FFN's bf16 tolerance; repeated
    launches identical (counters reset themselves)."""
    ops, L = gpu
    W = _weights(ops, L, seed=seed)
    g = torch.Generator(device=DEV).manual_seed(seed + 7)
    lens = torch.randint(T // 2, T + 1, (B,), device=DEV, generator=g)
    lens[0] = T
    if B > 2:
        lens[1], lens[2] = 0, 1
    x = _x(B, T, lens, seed + 1)
    att = _x(B, T, lens, seed + 2)
    wfc = torch.randn(256, 256, device=DEV, generator=g) / 16
    bfc = 0.1 * torch.randn(256, device=DEV, generator=g)
    ln1 = (1 + 0.1 * torch.randn(256, device=DEV, generator=g), 0.1 * torch.randn(256, device=DEV, generator=g), 1e-5)
    lay = ops.SeqLayout(lens, T)
    pk = lambda t: _pack(lay, t)
    pre = (pk(att), ops.pack_frag_rows(wfc), bfc, ln1)
    kw = dict(ks=9, pad=4, ln=W["ln"], layout=lay, pre=pre)
    outs = [ops.ffn(pk(x), W["w12"], W["b1"], W["b2"], tile_rows=96, nsplit=2, **kw) for _ in range(3)]
    ref112 = ops.ffn(pk(x), W["w12"], W["b1"], W["b2"], tile_rows=112, nsplit=1, **kw)
    torch.cuda.synchronize()
    R = int(lay.cu[-1])
    got = outs[0][:R]
    for o in outs[1:]:
        assert torch.equal(o[:R], got)
    d = (got.float() - ref112[:R].float()).abs()
    ulp = ref112[:R].float().abs().clamp(min=2 ** -8) * 2 ** -7
    assert float((d / ulp).max()) <= 2.0, float((d / ulp).max())
    h = torch.nn.functional.layer_norm(att.double() @ wfc.to(torch.bfloat16).double().t() + bfc.double() + x.double(),
                                       (256,), ln1[0].double(), ln1[1].double(), ln1[2])
    valid = (torch.arange(T, device=DEV)[None, :] < lens[:, None])
    h = (h * valid[..., None]).to(torch.bfloat16)
    refp = _ref(h, lens, W).reshape(-1, 256)[valid.reshape(-1)]
    err = (got.double() - refp).abs()
    assert float(err.max()) <= 0.1 and float(err.mean()) <= 6e-3, (float(err.max()), float(err.mean()))


@pytest.mark.parametrize("tile_rows,nsplit,packed", [(112, 1, True), (64, 4, False), (112, 2, True), (64, 1, False)])
def test_ffn_next_qkv_epilogue(gpu, tile_rows, nsplit, packed):
    """fs2_ffn with the next block's Q|K|V projection in its epilogue: qkv = bf16(y . W^T + b) on
    the kernel's own bf16 output rows (float64 reference of the same operands: bf16 output
    rounding), y unchanged by the extra epilogue, rows past the active packed rows untouched."""
    ops, L = gpu
    B, T = 19, 140
    W = _weights(ops, L, seed=31)
    g = torch.Generator(device="cpu").manual_seed(9)
    lens = torch.randint(1, T + 1, (B,), generator=g)
    lens[0] = T
    lens = lens.to(DEV)
    x = _x(B, T, lens, 31)
    gd = torch.Generator(device=DEV).manual_seed(32)
    wq = torch.randn(768, 256, device=DEV, generator=gd) / 16
    bq = 0.1 * torch.randn(768, device=DEV, generator=gd)
    wqf = ops.pack_frag_rows(wq)
    kw = dict(ks=9, pad=4, ln=W["ln"], nsplit=nsplit, tile_rows=tile_rows)
    if packed:
        lay = ops.SeqLayout(lens, T)
        rm = lay.rowmap.long()
        ok = rm >= 0
        xp = x.new_zeros(lay.capacity, 256)
        xp[rm[ok]] = x.reshape(-1, 256)[ok]
        y0 = ops.ffn(xp, W["w12"], W["b1"], W["b2"], layout=lay, **kw)
        y, qkv = ops.ffn(xp, W["w12"], W["b1"], W["b2"], layout=lay, next_qkv=(wqf, bq), **kw)
        R = int(lay.cu[-1])
        y0, y, qkv = y0[:R], y[:R], qkv[:R]
    else:
        y0 = ops.ffn(x, W["w12"], W["b1"], W["b2"], lens=lens, **kw)
        y, qkv = ops.ffn(x, W["w12"], W["b1"], W["b2"], lens=lens, next_qkv=(wqf, bq), **kw)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    ref = y.double().reshape(-1, 256) @ wq.to(torch.bfloat16).double().t() + bq.double()
    err = (qkv.double().reshape(-1, 768) - ref).abs()
    scale = float(ref.abs().max())
    assert float(err.max()) <= 1e-2 * scale, (float(err.max()), scale)
    assert float(err.mean()) <= 1e-3 * scale, (float(err.mean()), scale)


@pytest.mark.parametrize("B,T,seed,tile", [(64, 430, 31, 112), (8, 130, 32, 112), (3, 37, 33, 112),
                                          (64, 430, 34, 64), (8, 130, 35, 64), (3, 37, 36, 64)])
def test_ffn_pre_fc_ln_prologue(gpu, B, T, seed, tile):
    """fs2_ffn with pre_att: the FFT block's attention output projection + residual + LayerNorm
    (SubLayers.py:54-55) computed in the fused FFN's prologue for each tile and its 4+4 halo rows,
    then the FFN (packed rows; ragged lengths incl. 0 and 1). Against a float64 statement of the
    whole sequence (h rounded to bf16 where the two-launch path stores it) within the FFN's bf16
    tolerance, and against the two launches (fc + LN on fs2_conv1d, then fs2_ffn) within 2 bf16 ulps
    (the h rounding can move by one ulp with the summation order). Also with the next block's
    Q|K|V in the epilogue. Both packed unsplit tile forms: 112 rows (teacher-forced decoder) and
    64 rows (free-running decoder)."""
    ops, L = gpu
    W = _weights(ops, L, seed=seed)
    g = torch.Generator(device=DEV).manual_seed(seed + 7)
    lens = torch.randint(T // 2, T + 1, (B,), device=DEV, generator=g)
    lens[0] = T
    if B > 2:
        lens[1], lens[2] = 0, 1
    x = _x(B, T, lens, seed + 1)
    att = _x(B, T, lens, seed + 2)
    wfc = torch.randn(256, 256, device=DEV, generator=g) / 16
    bfc = 0.1 * torch.randn(256, device=DEV, generator=g)
    ln1 = (1 + 0.1 * torch.randn(256, device=DEV, generator=g), 0.1 * torch.randn(256, device=DEV, generator=g), 1e-5)
    lay = ops.SeqLayout(lens, T)
    pk = lambda t: _pack(lay, t)
    with ops.splitk_enabled(False):  # the 112-row unsplit form the prologue covers
        h2 = ops.conv1d(pk(att), ops.pack_conv_weight(wfc, L.FS2_BF16), bfc, cin=256, ks=1, pad=0, compute=L.FS2_BF16,
                        epilogue=L.EPI_RES_LN, out_dtype=L.FS2_BF16, residual=pk(x), ln=ln1, layout=lay)
        tf = dict(tile_rows=tile, nsplit=1)
        two = ops.ffn(h2, W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], layout=lay, **tf)
        one = ops.ffn(pk(x), W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], layout=lay,
                      pre=(pk(att), ops.pack_frag_rows(wfc), bfc, ln1), **tf)
        wq = torch.randn(768, 256, device=DEV, generator=g) / 16
        bq = 0.1 * torch.randn(768, device=DEV, generator=g)
        one_q, qkv = ops.ffn(pk(x), W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], layout=lay,
                             pre=(pk(att), ops.pack_frag_rows(wfc), bfc, ln1), next_qkv=(ops.pack_frag_rows(wq), bq), **tf)
    torch.cuda.synchronize()
    R = int(lay.cu[-1])
    # float64 reference on the padded rows
    h = torch.nn.functional.layer_norm(att.double() @ wfc.to(torch.bfloat16).double().t() + bfc.double() + x.double(),
                                       (256,), ln1[0].double(), ln1[1].double(), ln1[2])
    valid = (torch.arange(T, device=DEV)[None, :] < lens[:, None])
    h = (h * valid[..., None]).to(torch.bfloat16)
    ref = _ref(h, lens, W)
    refp = ref.reshape(-1, 256)[valid.reshape(-1)]
    err = (one[:R].double() - refp).abs()
    assert float(err.max()) <= 0.1 and float(err.mean()) <= 6e-3, (float(err.max()), float(err.mean()))
    d = (one[:R].float() - two[:R].float()).abs()
    ulp = two[:R].float().abs().clamp(min=2 ** -8) * 2 ** -7
    assert float((d / ulp).max()) <= 2.0 or float(err.max()) <= 0.05, float((d / ulp).max())
    assert torch.equal(one_q[:R], one[:R])
    qref = (one[:R].double() @ wq.to(torch.bfloat16).double().t() + bq.double())
    assert float((qkv[:R].double() - qref).abs().max()) <= 0.05 * max(1.0, float(qref.abs().max()))


@pytest.mark.parametrize("B,T,nsplit,seed", [(64, 64, 4, 41), (8, 37, 4, 42), (5, 50, 2, 43)])
def test_ffn_pre_padded_split_form(gpu, B, T, nsplit, seed):
    """The encoder's form of the fc + residual + LN prologue: padded [B, T] rows with lengths, 64-row
    tiles in the split-hidden form (every split recomputes its tile's h; padded rows of h are zeroed
    as masked_fill does, Layers.py:25-26), the speaker / emotion vectors in the LN epilogue and the
    next block's Q|K|V. Against the two launches it replaces (fc + LN + mask on fs2_conv1d, then
    fs2_ffn on the same form): the h rounding can move by one bf16 ulp with the summation order,
    which moves the output by a fraction of the LN scale, so valid rows within 0.05 absolute (max)
    and 1e-3 (mean), at most 0.5 % of the elements beyond 2 ulps of the output; padded rows (zeros
    + the speaker / emotion vectors) exactly."""
    ops, L = gpu
    W = _weights(ops, L, seed=seed)
    g = torch.Generator(device=DEV).manual_seed(seed + 7)
    lens = torch.randint(T // 2, T + 1, (B,), device=DEV, generator=g)
    lens[0] = T
    if B > 2:
        lens[1], lens[2] = 1, T - 1
    x = _x(B, T, lens, seed + 1)
    att = torch.randn(B, T, 256, device=DEV, generator=g).to(torch.bfloat16)
    wfc = torch.randn(256, 256, device=DEV, generator=g) / 16
    bfc = 0.1 * torch.randn(256, device=DEV, generator=g)
    ln1 = (1 + 0.1 * torch.randn(256, device=DEV, generator=g), 0.1 * torch.randn(256, device=DEV, generator=g), 1e-5)
    av1 = torch.randn(B, 256, device=DEV, generator=g)
    av2 = torch.randn(B, 256, device=DEV, generator=g)
    wq = torch.randn(768, 256, device=DEV, generator=g) / 16
    bq = 0.1 * torch.randn(768, device=DEV, generator=g)
    kw = dict(ks=9, pad=4, ln=W["ln"], lens=lens, addvec1=av1, addvec2=av2, nsplit=nsplit, tile_rows=64,
              next_qkv=(ops.pack_frag_rows(wq), bq))
    h2 = ops.conv1d(att, ops.pack_conv_weight(wfc, L.FS2_BF16), bfc, cin=256, ks=1, pad=0, compute=L.FS2_BF16,
                    epilogue=L.EPI_RES_LN, out_dtype=L.FS2_BF16, residual=x, ln=ln1, lens=lens)
    two, q2 = ops.ffn(h2, W["w12"], W["b1"], W["b2"], **kw)
    one, q1 = ops.ffn(x, W["w12"], W["b1"], W["b2"], pre=(att, ops.pack_frag_rows(wfc), bfc, ln1), **kw)
    torch.cuda.synchronize()
    valid = torch.arange(T, device=DEV)[None, :] < lens[:, None]
    d = (one.float() - two.float()).abs()[valid]
    ulp = two.float().abs().clamp(min=2 ** -8)[valid] * 2 ** -7
    far = float((d > 2 * ulp).float().mean())
    print(f"pre padded split: max {float(d.max()):.4f} mean {float(d.mean()):.2e} beyond 2 ulps {far:.2e}")
    assert float(d.max()) <= 0.05 and float(d.mean()) <= 1e-3 and far <= 5e-3, (float(d.max()), float(d.mean()), far)
    assert torch.equal(one[~valid], two[~valid])
    dq = (q1.float() - q2.float()).abs()
    assert float(dq.max()) <= 0.05 * max(1.0, float(q2.float().abs().max())), float(dq.max())


# ---- fs2_ffn_wide (the small-row-count form: conv-k9 on 256-row x 64-column tiles into a bf16 hidden,
# then the k=1 conv + LN finished by the last of 4 column quarters)
@pytest.mark.parametrize("B,T,seed,F,ks", [(64, 64, 51, 1024, 9), (8, 130, 52, 1024, 9), (3, 37, 53, 1024, 9),
                                          (5, 50, 54, 512, 3), (1, 300, 55, 1024, 9)])
def test_ffn_wide_matches_float64_and_fused(gpu, B, T, seed, F, ks):
    """fs2_ffn_wide against the float64 statement (bf16 tolerance, as the fused launch) and against
    the unsplit fused launch. The wide form's conv-k loop runs channel-chunk-major (the x tile streams
    into LDS chunk by chunk) where the fused kernel runs tap-major, so the f32 hidden sums round
    differently: a hidden value can land one bf16 ulp apart, and the LayerNorm row statistics are
    summed in another order -- measured within 2 bf16 ulps of |y| <~ 4 on a few percent of the
    elements. Ragged lengths (0 / 1 / shorter than the taps' reach), rows past the last 256-row tile,
    repeated launches identical."""
    ops, L = gpu
    W = _weights(ops, L, F=F, ks=ks, seed=seed)
    rng = np.random.default_rng(seed)
    lens_l = rng.integers(0, T + 1, B).tolist()
    lens_l[0] = T
    if B > 2:
        lens_l[1], lens_l[2] = 1, 3
    lens = torch.tensor(lens_l, dtype=torch.int64, device=DEV)
    x = _x(B, T, lens, seed)
    pad = (ks - 1) // 2
    got = ops.ffn_wide(x, W["w12"], W["b1"], W["b2"], ks=ks, pad=pad, ln=W["ln"], lens=lens)
    again = ops.ffn_wide(x, W["w12"], W["b1"], W["b2"], ks=ks, pad=pad, ln=W["ln"], lens=lens)
    fused = ops.ffn(x, W["w12"], W["b1"], W["b2"], ks=ks, pad=pad, ln=W["ln"], lens=lens, tile_rows=112, nsplit=1)
    torch.cuda.synchronize()
    assert torch.equal(got, again)
    ref = _ref(x, lens, W)
    err = (got.double() - ref).abs()
    assert float(err.max()) <= 3e-2 and float(err.mean()) <= 2e-3, (float(err.max()), float(err.mean()))
    d = (got.float() - fused.float()).abs()
    assert float(d.max()) <= 3.2e-2 and float((d > 0).float().mean()) <= 0.05, (float(d.max()), float((d > 0).float().mean()))


def test_ffn_wide_addvecs_packed_and_form_rule(gpu):
    """fs2_ffn_wide with speaker / emotion vectors (added after the mask, every row), on packed rows
    of a SeqLayout (rows_dev, row positions: packed == padded bit-identical, as fs2_ffn), and the
    runtime picks it for the cfg2 encoder's 4,096 rows only (cfg4's 41k keep the fused launch)."""
    ops, L = gpu
    from fs2amd import runtime

    W = _weights(ops, L, seed=61)
    B, T = 6, 70
    lens = torch.tensor([70, 0, 1, 33, 69, 12], dtype=torch.int64, device=DEV)
    x = _x(B, T, lens, 61)
    g = torch.Generator(device=DEV).manual_seed(62)
    v1, v2 = (torch.randn(B, 256, device=DEV, generator=g) for _ in range(2))
    got = ops.ffn_wide(x, W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], lens=lens, addvec1=v1, addvec2=v2)
    ref = _ref(x, lens, W, (v1, v2))
    assert float((got.double() - ref).abs().max()) <= 3e-2
    lay = ops.SeqLayout(lens, T)
    xp = _pack(lay, x)
    gp = ops.ffn_wide(xp, W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], layout=lay)
    gd = ops.ffn_wide(x, W["w12"], W["b1"], W["b2"], ks=9, pad=4, ln=W["ln"], lens=lens)
    torch.cuda.synchronize()
    rm = lay.rowmap.long()
    ok = rm >= 0
    R = int(lay.cu[-1])
    assert torch.equal(gp[:R], gd.reshape(-1, 256)[ok])
    assert ops.ffn_wide_ok(64 * 64, 1024, 9) and not ops.ffn_wide_ok(256 * 160, 1024, 9)
