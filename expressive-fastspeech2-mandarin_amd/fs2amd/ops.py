"""Torch-facing wrappers of the fs2hip C ABI: device tensors in, device tensors out.

Each wrapper validates shapes on the host, passes raw device pointers + sizes to
libfs2hip.so and launches on ``torch.cuda.current_stream()``. PyTorch only provides the
memory and the stream; every arithmetic op below runs in a hand-written HIP kernel. There
is no CPU path: CPU tensors raise.
"""
import ctypes
import os

import torch

from . import _lib as L

_lib = L.load()


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _dt(t):
    if t.dtype == torch.bfloat16:
        return L.FS2_BF16
    if t.dtype == torch.float32:
        return L.FS2_F32
    if t.dtype == torch.float8_e4m3fn:
        return L.FS2_FP8
    raise TypeError(f"fs2amd: unsupported dtype {t.dtype} (float32 / bfloat16 / float8_e4m3fn only)")


FP8_MAX = 448.0  # e4m3fn


def torch_dtype(code):
    if code == L.FS2_FP8:
        return torch.float8_e4m3fn
    return torch.bfloat16 if code == L.FS2_BF16 else torch.float32


def _gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("fs2amd: the HIP backend needs ROCm device tensors (got a CPU tensor); "
                               "there is no CPU fallback")


def _rows(x, name):
    """Row stride (elements) of a [B, T, C] (or packed [rows, C]) tensor with evenly spaced rows."""
    if x.dim() == 2 and x.stride(1) == 1:
        return x.stride(0)
    if x.dim() != 3 or x.stride(2) != 1 or x.stride(0) != x.shape[1] * x.stride(1):
        raise ValueError(f"fs2amd: {name} must be a [B, T, C] or [rows, C] tensor with unit channel stride and "
                         f"evenly spaced rows")
    return x.stride(1)


def cin_pad(cin, compute):
    return _lib.fs2_conv_cin_pad(cin, compute)


def pack_conv_weight(w, compute, scale=None):
    """nn.Conv1d weight [N, Cin, KS] (or nn.Linear [N, Cin]) -> packed [N, KS, Cin_pad] in the
    compute dtype, optionally scaled per output channel (BatchNorm folding). fp8: use
    :func:`pack_conv_weight_fp8` (it also returns the per-channel scales)."""
    if w.dim() == 2:
        w = w.unsqueeze(-1)
    w = w.detach().float()
    if scale is not None:
        w = w * scale.detach().float().view(-1, 1, 1)
    N, cin, ks = w.shape
    cp = cin_pad(cin, compute)
    if cp == cin:  # one fused permute + cast copy
        return torch.empty(N, ks, cin, dtype=torch_dtype(compute), device=w.device).copy_(w.permute(0, 2, 1))
    out = torch.zeros(N, ks, cp, dtype=torch_dtype(compute), device=w.device)
    out[:, :, :cin] = w.permute(0, 2, 1).to(out.dtype)
    return out.contiguous()


class SeqLayout:
    """Packed-sequence layout (fs2_seq_layout): B sequences of clamp(lens[b], 0, T) frames stored
    back to back in a [B*T, C] buffer (capacity). ``cu`` int32 [B+1] (cu[B] = active rows, read on
    the device), ``row_pos`` int32 [B*T, 2] = (frame, length) per packed row, ``rowmap`` int32
    [B*T] padded row -> packed row (-1 = padding). Built with two launches, no host sync."""

    def __init__(self, lens, T, margin=0):
        """margin > 0: sequence b holds min(lens[b] + margin, T) frames, or all T when
        lens[b] + 2 * margin > T (fs2_seq_layout_margin: the PostNet valid-region rows)."""
        _gpu(lens)
        lens = lens.to(torch.int64).contiguous()
        self.B, self.T = int(lens.shape[0]), int(T)
        dev = lens.device
        self.cu = torch.empty(self.B + 1, device=dev, dtype=torch.int32)
        self.row_pos = torch.empty(self.B * self.T, 2, device=dev, dtype=torch.int32)
        self.rowmap = torch.empty(self.B * self.T, device=dev, dtype=torch.int32)
        if margin:
            L.check(_lib.fs2_seq_layout_margin(_ptr(lens), self.B, self.T, int(margin), _ptr(self.cu),
                                               _ptr(self.row_pos), _ptr(self.rowmap), _stream(lens)),
                    "fs2_seq_layout_margin")
        else:
            L.check(_lib.fs2_seq_layout(_ptr(lens), self.B, self.T, _ptr(self.cu), _ptr(self.row_pos),
                                        _ptr(self.rowmap), _stream(lens)), "fs2_seq_layout")

    @classmethod
    def deferred(cls, B, T, device):
        """Allocated, not computed: a launch that builds the layout itself fills cu / row_pos /
        rowmap (fs2_lr_fused)."""
        lay = cls.__new__(cls)
        lay.B, lay.T = int(B), int(T)
        lay.cu = torch.empty(lay.B + 1, device=device, dtype=torch.int32)
        lay.row_pos = torch.empty(lay.B * lay.T, 2, device=device, dtype=torch.int32)
        lay.rowmap = torch.empty(lay.B * lay.T, device=device, dtype=torch.int32)
        return lay

    @property
    def capacity(self):
        return self.B * self.T

    @property
    def rows_dev(self):
        return self.cu.data_ptr() + 4 * self.B

    def empty(self, C, dtype):
        return torch.empty(self.capacity, C, device=self.cu.device, dtype=dtype)

    def unpack(self, packed):
        """Packed [B*T, C] -> padded [B, T, C] with zeros at padding (test / debug helper)."""
        C = packed.shape[-1]
        rm = self.rowmap.long()
        out = packed.new_zeros(self.capacity, C)
        ok = rm >= 0
        out[ok] = packed[rm[ok]]
        return out.view(self.B, self.T, C)


def pack_conv_weight_split(w, blocks):
    """bf16x3 split-precision weights: w = hi + lo (bf16 parts); the packed [N, KS, len(blocks)*Cin]
    bf16 weight holds the part named by each block ('hi' / 'lo'), matching an input whose channel
    blocks hold x_hi / x_lo (y = x_hi w_hi + x_hi w_lo + x_lo w_hi, the x_lo w_lo term dropped)."""
    if w.dim() == 2:
        w = w.unsqueeze(-1)
    w = w.detach().float()
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    parts = {"hi": hi, "lo": lo}
    cat = torch.cat([parts[b] for b in blocks], dim=1)  # [N, len*Cin, KS]
    return pack_conv_weight(cat.float(), L.FS2_BF16)


def pack_conv_weight_fp8(w):
    """Per-output-channel e4m3fn quantisation: w[n] ~= q[n] * s[n], s[n] = max|w[n]| / 448.
    Returns (packed [N, KS, Cin_pad] float8_e4m3fn, s f32 [N])."""
    if w.dim() == 2:
        w = w.unsqueeze(-1)
    w = w.detach().float()
    N, cin, ks = w.shape
    s = (w.abs().amax(dim=(1, 2)) / FP8_MAX).clamp_min(1e-12)
    q = (w / s.view(-1, 1, 1)).clamp(-FP8_MAX, FP8_MAX)
    cp = cin_pad(cin, L.FS2_FP8)
    out = torch.zeros(N, ks, cp, dtype=torch.float8_e4m3fn, device=w.device)
    out[:, :, :cin] = q.permute(0, 2, 1).to(torch.float8_e4m3fn)
    return out.contiguous(), s.contiguous()


# fs2_conv_desc.splitk_ws: counters + f32 partial tiles (32 MiB covers the 128x128 kernel's tail
# segments on 256 CUs)
SPLITK_WS_BYTES = 4096 + (32 << 20)
_splitk_ws = {}
_splitk_slot = [0]
_splitk_on = [os.environ.get("FS2_CONV_SPLITK", "1") != "0"]


class splitk_enabled:
    """Turn the split-K tail on/off for the launches inside (it changes the f32 summation order,
    so paths that must agree bit-exactly with an unsplit launch run with it off)."""

    def __init__(self, flag):
        self.flag = bool(flag)

    def __enter__(self):
        self.prev = _splitk_on[0]
        _splitk_on[0] = self.flag

    def __exit__(self, *exc):
        _splitk_on[0] = self.prev


class splitk_slot:
    """Launches inside use split-K workspace `i` (one per concurrently running stream)."""

    def __init__(self, i):
        self.i = i

    def __enter__(self):
        self.prev = _splitk_slot[0]
        _splitk_slot[0] = self.i

    def __exit__(self, *exc):
        _splitk_slot[0] = self.prev


def splitk_workspace(device):
    """The split-K tail workspace of (device, current slot, current stream): launches on different
    streams never share one (concurrent users would race on its arrival counters and partial
    tiles). Allocated on first use; only the 4 KiB of counters are zeroed (they self-reset after
    every tile), so under graph capture the first use records one small memset node."""
    if device.type != "cuda" or not _splitk_on[0]:
        return None
    key = (device.index, _splitk_slot[0], torch.cuda.current_stream(device).cuda_stream)
    ws = _splitk_ws.get(key)
    if ws is None:
        ws = torch.empty(SPLITK_WS_BYTES, dtype=torch.uint8, device=device)
        ws[:4096].zero_()
        _splitk_ws[key] = ws
    return ws


def conv1d(x, w_packed, bias, *, cin, ks, pad, compute, epilogue, out_dtype=None, out=None, residual=None,
           ln=None, lens=None, addvec1=None, addvec2=None, dot=None, n=None, layout=None, src_layout=None,
           col_scale=None, out_scale=1.0, out2=None, out2_scale=1.0, cin_block=0, cin_src=(), out_split=False,
           dilation=1, act_slope=0.0, out2_act=False, out2_slope=0.0, residual2=None, out_div=1.0, group=None):
    """Implicit-GEMM Conv1d / Linear with a fused epilogue (fs2_conv1d).

    layout: x / residual / out are packed [B*T, C] in that SeqLayout. src_layout (KS == 1): x is
    packed in it, out is padded [B, T, N] (zeros in, i.e. bias out, at padding).
    Vocoder extensions: dilation (tap k reads row t + k*dilation - pad), act_slope (EPI_BIAS_LRELU),
    out2_act / out2_slope (out2 = leaky_relu(y)), out2 may be f32, residual2 / out_div (EPI_RES_SUM).
    group = (group_n, group_cin): output columns [g*group_n, ...) read x's channels + g*group_cin."""
    _gpu(x, w_packed, bias, residual, lens, addvec1, addvec2, residual2)
    if layout is not None or src_layout is not None:
        lay = layout if layout is not None else src_layout
        B, T = lay.B, lay.T
        # a src_layout's packed rows may sit in a larger buffer (the decoder of a longer T bucket,
        # fs2amd.graphs.SynthGraphs): only its first cu[B] <= capacity rows are read
        assert x.dim() == 2 and (x.shape[0] == lay.capacity or (layout is None and x.shape[0] >= lay.capacity)), \
            (tuple(x.shape), lay.capacity)
    else:
        B, T, _ = x.shape
    N = w_packed.shape[0] if n is None else n
    d = L.ConvDesc()
    d.x, d.x_dtype, d.x_row_stride = x.data_ptr(), _dt(x), _rows(x, "x")
    d.w = w_packed.data_ptr()
    d.bias = bias.data_ptr() if bias is not None else None
    d.B, d.T, d.Cin, d.Cin_pad, d.N, d.KS, d.pad = B, T, cin, w_packed.shape[-1], N, ks, pad
    d.compute, d.epilogue = compute, epilogue
    if residual is not None:
        d.residual, d.res_dtype, d.res_row_stride = residual.data_ptr(), _dt(residual), _rows(residual, "residual")
    if ln is not None:
        g, b, eps = ln
        d.ln_gamma, d.ln_beta, d.ln_eps = g.data_ptr(), b.data_ptr(), float(eps)
    if lens is not None:
        assert lens.dtype == torch.int64 and lens.numel() == B
        d.lens = lens.data_ptr()
    if addvec1 is not None:
        d.addvec1 = addvec1.data_ptr()
    if addvec2 is not None:
        d.addvec2 = addvec2.data_ptr()
    if cin_block:
        d.cin_block = int(cin_block)
        for i, c in enumerate(cin_src):
            d.cin_src[i] = int(c)
    d.out_split = 1 if out_split else 0
    if col_scale is not None:
        d.col_scale = col_scale.data_ptr()
    d.out_scale = float(out_scale)
    if out2 is not None:
        d.out2, d.out2_scale = out2.data_ptr(), float(out2_scale)
        d.out2_f32 = 1 if out2.dtype == torch.float32 else 0
        d.out2_act, d.out2_slope = (1 if out2_act else 0), float(out2_slope)
    d.dilation, d.act_slope, d.out_div = int(dilation), float(act_slope), float(out_div)
    if residual2 is not None:
        d.residual2 = residual2.data_ptr()
    if group is not None:
        d.group_n, d.group_cin = int(group[0]), int(group[1])
    if layout is not None:
        d.rows_dev, d.row_pos = layout.rows_dev, layout.row_pos.data_ptr()
    if src_layout is not None:
        d.a_rowmap = src_layout.rowmap.data_ptr()
    ws = splitk_workspace(x.device)
    if ws is not None:
        d.splitk_ws, d.splitk_ws_bytes = ws.data_ptr(), ws.numel()
    oshape = (B * T,) if layout is not None else (B, T)
    if epilogue == L.EPI_RELU_LN_DOT:
        dw, db = dot
        d.dot_w, d.dot_b = dw.data_ptr(), float(db)
        if out is None:
            out = torch.empty(*oshape, device=x.device, dtype=torch.float32)
        d.out, d.out_dtype, d.out_row_stride = out.data_ptr(), L.FS2_F32, 1
    else:
        if out is None:
            out = torch.empty(*oshape, 2 * N if out_split else N, device=x.device, dtype=torch_dtype(out_dtype))
        d.out, d.out_dtype, d.out_row_stride = out.data_ptr(), _dt(out), _rows(out, "out")
    L.check(_lib.fs2_conv1d(ctypes.byref(d), _stream(x)), "fs2_conv1d")
    return out


def pack_ffn_weights(w1, w2):
    """PositionwiseFeedForward weights -> the fs2_ffn buffer (flat bf16, fs2_ffn_weight_elems(KS, F)
    elements): both matrices in MFMA fragment order, so that one wave's weight k-step ("unit": 64
    weight rows x 32 channels) is 4 KiB contiguous and each 1 KiB row block is one fully coalesced
    16-byte-per-lane load straight into the A-operand registers (lane l = 16 * hi + r holds row r of
    the block, channels 8 * hi .. 8 * hi + 7 of the 32).

    w_1 (nn.Conv1d weight [F, D, KS]): [F/64 row quads][KS taps][D/32 k-steps][4 blocks][4 hi][16 r][8]
    w_2 ([D, F, 1]):                   [D/64 row quads][F/32 k-steps][4 blocks][4 hi][16 r][8]"""
    F, D, ks = w1.shape
    assert w2.shape[:2] == (D, F) and (w2.dim() == 2 or w2.shape[2] == 1), (tuple(w1.shape), tuple(w2.shape))
    assert F % 64 == 0 and D % 64 == 0, (F, D)
    a = w1.detach().float().permute(0, 2, 1)  # [F][KS][D]
    a = a.reshape(F // 64, 4, 16, ks, D // 32, 4, 8).permute(0, 3, 4, 1, 5, 2, 6)
    b = w2.detach().float().reshape(D // 64, 4, 16, F // 32, 4, 8).permute(0, 3, 1, 4, 2, 5)
    return torch.cat([a.reshape(-1), b.reshape(-1)]).to(torch.bfloat16).contiguous()


def pack_ffn8_weights(q1, q2):
    """The e4m3 FFN pair (pack_conv_weight_fp8 outputs: q1 [F, KS, 256], q2 [256, 1, F]) -> the
    fs2_ffn8 byte buffer: 8 KiB units of 64 rows x 128 k, each lane's 32 bytes as two 16-byte halves
    (include/fs2hip.h: [q][u][b][h][g][r][e], element = W[64q + 16b + r][128u + 32g + 16h + e])."""
    F, KS, D = q1.shape
    assert q2.shape[0] == D and q2.shape[-1] == F and D % 128 == 0 and F % 128 == 0, (tuple(q1.shape), tuple(q2.shape))
    perm = (0, 3, 1, 5, 4, 2, 6)
    b1 = q1.contiguous().view(torch.uint8).reshape(F // 64, 4, 16, KS * D // 128, 4, 2, 16).permute(*perm)
    b2 = q2.contiguous().view(torch.uint8).reshape(D // 64, 4, 16, F // 128, 4, 2, 16).permute(*perm)
    return torch.cat([b1.reshape(-1), b2.reshape(-1)]).contiguous()


def ffn8(x8, res, w8, cs1, b1, inv_sf, cs2, b2, *, ln, layout, out=None, out8=None, out8_scale=1.0, ks=9, pad=4):
    """fs2_ffn8: the fused FFN on e4m3 MFMA (cfg5) over packed rows: x8 the e4m3 input [B*T, 256], res
    the bf16 LayerNorm residual (the same rows), w8 from :func:`pack_ffn8_weights`; out bf16 and
    optionally out8 = e4m3(out * out8_scale) (the next block's fp8 Q|K|V input)."""
    _gpu(x8, res, w8, cs1, b1, cs2, b2)
    assert layout is not None and x8.dim() == 2 and x8.shape[0] == layout.capacity and res.shape == x8.shape
    F = b1.numel()
    assert w8.numel() == _lib.fs2_ffn8_weight_bytes(ks, F)
    if out is None:
        out = torch.empty(res.shape, device=res.device, dtype=torch.bfloat16)
    d = L.Ffn8Desc()
    d.x8, d.x8_row_stride = x8.data_ptr(), _rows(x8, "x8")
    d.res, d.res_row_stride = res.data_ptr(), _rows(res, "res")
    d.w, d.cs1, d.b1, d.inv_sf, d.cs2, d.b2 = w8.data_ptr(), cs1.data_ptr(), b1.data_ptr(), float(inv_sf), \
        cs2.data_ptr(), b2.data_ptr()
    d.B, d.T, d.D, d.F, d.KS, d.pad = layout.B, layout.T, x8.shape[1], F, ks, pad
    g, b, eps = ln
    d.ln_gamma, d.ln_beta, d.ln_eps = g.data_ptr(), b.data_ptr(), float(eps)
    d.out, d.out_row_stride = out.data_ptr(), _rows(out, "out")
    if out8 is not None:
        d.out8, d.out8_row_stride, d.out8_scale = out8.data_ptr(), _rows(out8, "out8"), float(out8_scale)
    d.rows_dev, d.row_pos = layout.rows_dev, layout.row_pos.data_ptr()
    hint = getattr(layout, "rows_hint", None)
    d.rows_max = int(hint) if hint else 0
    L.check(_lib.fs2_ffn8(ctypes.byref(d), _stream(x8)), "fs2_ffn8")
    return out


def pack_wconv_weight(w, scale=None):
    """nn.Conv1d weight [N, Cin, KS] (optionally scaled per output channel: BatchNorm folding, in
    f32 then rounded once like pack_conv_weight) -> the fs2_wconv buffer: K = (tap, channel)
    flattened (k = tap * Cin + c), zero-padded to a multiple of 32, in MFMA fragment order
    [N/64][K/32][4][4][16][8] (include/fs2hip.h; for Cin % 32 == 0 this is [N/64][KS][Cin/32]...)."""
    w = w.detach().float()
    if scale is not None:
        w = w * scale.detach().float().view(-1, 1, 1)
    N, cin, ks = w.shape
    assert N % 64 == 0 and cin % 8 == 0, (N, cin)
    k = w.permute(0, 2, 1).reshape(N, ks * cin)
    kp = -(-ks * cin // 32) * 32
    if kp != ks * cin:
        k = torch.cat([k, k.new_zeros(N, kp - ks * cin)], 1)
    return pack_frag_rows(k)


def pack_wconv_tail(w, scale=None):
    """The PostNet's last conv (nn.Conv1d [80, 512, 5], BatchNorm folded like pack_conv_weight) for
    fs2_wconv's FS2_EPI_BIAS_RES form: K = (tap, channel) flattened, k-step-major fragment order
    [K/32][N/16][4][16][8] (every wave reads all 80 columns of a k-step from the LDS ring)."""
    w = w.detach().float()
    if scale is not None:
        w = w * scale.detach().float().view(-1, 1, 1)
    N, cin, ks = w.shape
    assert N % 16 == 0 and (ks * cin) % 32 == 0, (N, cin, ks)
    k = w.permute(0, 2, 1).reshape(N, ks * cin)
    b = k.reshape(N // 16, 16, ks * cin // 32, 4, 8).permute(2, 0, 3, 1, 4)
    return b.reshape(-1).to(torch.bfloat16).contiguous()


def _wconv_rows(x, layout):
    """(B, T, cin, out row shape) of a fs2_wconv operand: padded [B, T, C] or packed [B*T, C]."""
    if layout is not None:
        assert x.dim() == 2 and x.shape[0] == layout.capacity, (tuple(x.shape), layout.capacity)
        return layout.B, layout.T, x.shape[1], (layout.capacity,)
    B, T, cin = x.shape
    return B, T, cin, (B, T)


def _wconv_layout(d, layout):
    if layout is not None:
        d.rows_dev, d.row_pos = layout.rows_dev, layout.row_pos.data_ptr()
        hint = getattr(layout, "rows_hint", None)
        d.rows_max = int(hint) if hint else 0


def wconv_tail(x, w_packed, bias, residual, *, ks=5, pad=2, out=None, layout=None):
    """PostNet last conv + residual: out f32 [B, T, 80] = conv(x; w) + bias + residual (fs2_wconv,
    FS2_EPI_BIAS_RES; w_packed from :func:`pack_wconv_tail`). layout: packed rows (ops.SeqLayout)."""
    _gpu(x, w_packed, bias, residual)
    if x.dtype != torch.bfloat16 or w_packed.dtype != torch.bfloat16 or residual.dtype != torch.float32:
        raise TypeError("fs2amd.wconv_tail: bf16 x / weights, f32 residual")
    B, T, cin, rs = _wconv_rows(x, layout)
    N = bias.numel()
    assert tuple(residual.shape) == (*rs, N) and w_packed.numel() == _lib.fs2_wconv_weight_elems(ks, cin, N)
    if out is None:
        out = torch.empty(*rs, N, device=x.device, dtype=torch.float32)
    d = L.WconvDesc()
    _wconv_layout(d, layout)
    d.x, d.x_row_stride = x.data_ptr(), _rows(x, "x")
    d.w, d.bias = w_packed.data_ptr(), bias.data_ptr()
    d.B, d.T, d.Cin, d.N, d.KS, d.pad, d.epilogue = B, T, cin, N, ks, pad, L.EPI_BIAS_RES
    d.out, d.out_row_stride = out.data_ptr(), _rows(out, "out")
    d.residual, d.res_row_stride = residual.data_ptr(), _rows(residual, "residual")
    L.check(_lib.fs2_wconv(ctypes.byref(d), _stream(x)), "fs2_wconv")
    return out


def hifigan_mrf(x, x_act, w_packed, bias, out_slope, out=None):
    """fs2_hifigan_mrf: one HiFi-GAN stage's multi-receptive-field block (3 ResBlock1 chains, their
    average, the next leaky_relu) in one launch: x / x_act = the upsampler's output and its
    leaky_relu, bf16 [B, T, C] (C = 32 / 64) -> lrelu(xs / 3, out_slope) bf16 [B, T, C]."""
    _gpu(x, x_act, w_packed, bias)
    B, T, C = x.shape
    assert x_act.shape == x.shape and x.dtype == torch.bfloat16 and x_act.dtype == torch.bfloat16
    assert w_packed.numel() == _lib.fs2_hifigan_mrf_weight_elems(C) and bias.numel() == 18 * C
    if out is None:
        out = torch.empty_like(x)
    L.check(_lib.fs2_hifigan_mrf(_ptr(x.contiguous()), _ptr(x_act.contiguous()), _ptr(w_packed), _ptr(bias), B, T, C,
                                 float(out_slope), _ptr(out), _stream(x)), "fs2_hifigan_mrf")
    return out


def hifigan_post(x, w, bias, out=None):
    """fs2_hifigan_post: conv_post (32 -> 1, k = 7, pad 3) + tanh (hifigan/models.py:145,159-162) on
    x bf16 [B, T, 32] -> f32 [B, T]. w: bf16 [7, 32] (conv_post.weight[0].T); bias: python float."""
    _gpu(x, w)
    B, T, C = x.shape
    ks = w.shape[0]
    assert x.dtype == torch.bfloat16 and x.is_contiguous() and w.dtype == torch.bfloat16 and w.is_contiguous()
    assert w.shape == (ks, C), (tuple(w.shape), C)
    if out is None:
        out = torch.empty(B, T, device=x.device, dtype=torch.float32)
    assert out.dtype == torch.float32 and out.is_contiguous() and out.shape == (B, T)
    L.check(_lib.fs2_hifigan_post(_ptr(x), _ptr(w), float(bias), B, T, C, ks, _ptr(out), _stream(x)),
            "fs2_hifigan_post")
    return out


def hifigan_pair(x, w1, b1, w2, b2, ks, dilation, *, xs=None, out_scale=1.0, out_slope=0.1, out_act=False, out=None):
    """fs2_hifigan_pair: one ResBlock1 dilation pair at C in {128, 64} in one launch (256-sample
    tiles at C = 128, 512-sample tiles at C = 64), y = conv2(lrelu(conv1_d(lrelu(x)) + b1)) + b2 + x
    (+ xs); returns y, or lrelu(y * out_scale, out_slope) with out_act. x / xs bf16 [B, T, C];
    w1 / w2 from :func:`pack_wconv_tail`."""
    _gpu(x, w1, b1, w2, b2)
    B, T, C = x.shape
    assert x.dtype == torch.bfloat16 and x.is_contiguous()
    assert w1.numel() == ks * C * C and w2.numel() == ks * C * C and b1.numel() == C and b2.numel() == C
    if xs is not None:
        assert xs.shape == x.shape and xs.dtype == torch.bfloat16 and xs.is_contiguous()
    if out is None:
        out = torch.empty_like(x)
    L.check(_lib.fs2_hifigan_pair(_ptr(x), _ptr(w1), _ptr(b1), _ptr(w2), _ptr(b2), B, T, C, int(ks), int(dilation),
                                  None if xs is None else _ptr(xs), float(out_scale), float(out_slope),
                                  1 if out_act else 0, _ptr(out), _stream(x)), "fs2_hifigan_pair")
    return out


def wconv(x, w_packed, bias, *, ks, pad, out=None, second=None, layout=None, tail=None):
    """PostNet Conv1d(512, 512, k=5) + folded BatchNorm + tanh on padded bf16 rows [B, T, 512]
    (fs2_wconv; w_packed from :func:`pack_wconv_weight`). second = (w2_packed, bias2): the next
    512 -> 512 conv applied in the same launch (the PostNet's layers 0 and 1, Cin = 80). tail =
    (w_tail from :func:`pack_wconv_tail`, bias_tail, residual f32): the PostNet's last conv +
    residual on this conv's output in the same launch (layers 3 and 4, Cin = 512): returns the f32
    [.., 80] PostNet output instead. layout: packed rows [B*T, C] (ops.SeqLayout; the valid-region
    PostNet)."""
    _gpu(x, w_packed, bias)
    if x.dtype != torch.bfloat16 or w_packed.dtype != torch.bfloat16:
        raise TypeError("fs2amd.wconv: bf16 activations and weights only")
    B, T, cin, rs = _wconv_rows(x, layout)
    N = bias.numel()
    assert w_packed.is_contiguous() and w_packed.numel() == _lib.fs2_wconv_weight_elems(ks, cin, N)
    if second is not None:
        _gpu(*second)
        assert second[0].numel() == _lib.fs2_wconv_weight_elems(ks, N, N) and second[1].numel() == N
    if tail is not None:
        wt, bt, res = tail
        _gpu(wt, bt, res)
        assert second is None and cin == 512 and N == 512 and bt.numel() == 80 and res.dtype == torch.float32
        assert wt.dtype == torch.bfloat16 and wt.numel() == _lib.fs2_wconv_weight_elems(ks, 512, 80)
        assert tuple(res.shape) == (*rs, 80), (tuple(res.shape), rs)
        if out is None:
            out = torch.empty(*rs, 80, device=x.device, dtype=torch.float32)
        d = L.WconvDesc()
        _wconv_layout(d, layout)
        d.x, d.x_row_stride = x.data_ptr(), _rows(x, "x")
        d.w, d.bias = w_packed.data_ptr(), bias.data_ptr()
        d.B, d.T, d.Cin, d.N, d.KS, d.pad, d.epilogue = B, T, cin, N, ks, pad, L.EPI_BIAS_TANH
        d.out, d.out_row_stride = out.data_ptr(), _rows(out, "out")
        d.w2, d.bias2 = wt.data_ptr(), bt.data_ptr()
        d.residual, d.res_row_stride = res.data_ptr(), _rows(res, "residual")
        L.check(_lib.fs2_wconv(ctypes.byref(d), _stream(x)), "fs2_wconv")
        return out
    if out is None:
        out = torch.empty(*rs, N, device=x.device, dtype=torch.bfloat16)
    d = L.WconvDesc()
    _wconv_layout(d, layout)
    d.x, d.x_row_stride = x.data_ptr(), _rows(x, "x")
    d.w, d.bias = w_packed.data_ptr(), bias.data_ptr()
    d.B, d.T, d.Cin, d.N, d.KS, d.pad, d.epilogue = B, T, cin, N, ks, pad, L.EPI_BIAS_TANH
    d.out, d.out_row_stride = out.data_ptr(), _rows(out, "out")
    if second is not None:
        d.w2, d.bias2 = second[0].data_ptr(), second[1].data_ptr()
    L.check(_lib.fs2_wconv(ctypes.byref(d), _stream(x)), "fs2_wconv")
    return out


FFN_SLOTS = 256  # workgroups resident at once (1 per CU)


def ffn_part_bytes(tile_rows):
    """f32 partial accumulators per (tile, split) of fs2_ffn's split-hidden form (ffn.hip part_bytes)."""
    return 4 * 4 * (tile_rows // 16) * 64 * 16


def rows_bucket(rows, capacity, step=1024):
    """A host-known active row count rounded up to a multiple of ``step`` (capped at the capacity):
    the upper bound packed launches are sized with (fs2_ffn rows_max), so that one captured graph
    serves every batch whose count falls in the bucket."""
    return min(capacity, -(-int(rows) // step) * step)


# fs2_ffn cost model (us, one round of workgroups at one per CU; graph-timed probes at the encoder
# shape, tools/kernel_probe.py enc_ffn): per 256-column hidden chunk, fixed cost (x tile, LN
# epilogue), and the split hand-off (partial stores, arrival counter, partial loads) per nsplit.
# Measured: 112-row tiles 90 / 59.6 / 45.8 us at nsplit 1 / 2 / 4; 64-row tiles 57.3 / 40.2 / 38.8.
# 96-row tiles only as 2 splits (round 6: a free-running decoder's 8-12k rows -> ~230 workgroups that
# each stream half the weights; the per-CU weight stream, ~5.2 MB at ~70 GB/s, bounds the 64-row form
# there), interpolated between the two measured tile heights.
FFN_COST = {112: (20.0, 10.0, {1: 0.0, 2: 10.0, 4: 16.0}), 96: (17.5, 8.5, {2: 10.0}),
            64: (13.0, 5.0, {1: 0.0, 2: 9.0, 4: 21.0})}


def ffn_form(rows, F):
    """fs2_ffn launch form (tile_rows, nsplit) for ``rows`` rows and hidden width F: the least
    modelled time (FFN_COST) over rounds of FFN_SLOTS workgroups. The cfg2 decoder (24.9k rows) ->
    (112, 1); the 4k-row encoder -> (64, 4); a free-running cfg2 decoder (11.1k rows) -> (64, 1).
    (112, 1) when the split-K workspace is off (ops.splitk_enabled(False): bit-exact comparisons)."""
    nch = F // 256
    if not _splitk_on[0]:
        return 112, 1
    best = None
    for tr, (chunk, base, over) in FFN_COST.items():
        tiles = -(-rows // tr)
        for s in (1, 2, 4):
            if s > nch or s not in over:
                continue
            if s > 1 and (tiles > 1024 or 4096 + tiles * s * ffn_part_bytes(tr) > SPLITK_WS_BYTES):
                continue
            t = -(-tiles * s // FFN_SLOTS) * (nch // s * chunk + base + over[s])
            if best is None or t < best[0] - 1e-9:
                best = (t, tr, s)
    return best[1], best[2]


def ffn_nsplit(rows, F):
    return ffn_form(rows, F)[1]


def pack_frag_rows(w):
    """A [N, K] weight (N, K multiples of 64 / 32) in the MFMA fragment order the fused kernels
    stream to registers: [N/64][K/32][4 blocks][4 hi][16 r][8] (fs2_ffn w_2, fs2_ffn wqkv)."""
    N, K = w.shape[0], w.shape[1]
    assert N % 64 == 0 and K % 32 == 0, (N, K)
    b = w.detach().float().reshape(N // 64, 4, 16, K // 32, 4, 8).permute(0, 3, 1, 4, 2, 5)
    return b.reshape(-1).to(torch.bfloat16).contiguous()


def ffn_launch_rows(x, layout):
    """The row count an fs2_ffn launch is sized for (the host's bound when it knows one)."""
    if layout is None:
        return x.shape[0] * x.shape[1]
    return getattr(layout, "rows_hint", None) or layout.capacity


def ffn_pre_ok(x, layout, F, ks):
    """fs2_ffn's fc + residual + LN prologue (pre_att) covers the k = 9, F = 1024 FFN as packed
    112- or 64-row unsplit launches (the decoder's) and, opt-in (FS2_FFN_PRE_ENC=1), as padded [B, T]
    launches on 64-row tiles (the encoder's split-hidden form; padded rows are masked in the
    prologue). Off by default: every split of a tile recomputes the prologue, and the encoder
    launch grew by more than the fc launch it replaces (51-53 vs 41.6 + 10.4 us per block in
    eager forwards, profiles/r5f)."""
    if ks != 9 or F != 1024:
        return False
    form = ffn_form(ffn_launch_rows(x, layout), F)
    if layout is not None:
        # packed launches: unsplit 112-row tiles (teacher-forced cfg2), 96-row tiles x 2 splits (a
        # free-running decoder of ~8-12k rows; every split computes the prologue) or unsplit 64-row
        # tiles; FS2_FFN_PRE64=0 keeps the fc launch for the smaller forms
        small = os.environ.get("FS2_FFN_PRE64", "1") != "0"
        return form == (112, 1) or (form in ((64, 1), (96, 2)) and small)
    return form[0] == 64 and os.environ.get("FS2_FFN_PRE_ENC", "0") == "1"


def ffn(x, w_packed, b1, b2, *, ks, pad, ln, lens=None, addvec1=None, addvec2=None, layout=None, out=None,
        nsplit=None, tile_rows=None, next_qkv=None, pre=None):
    """PositionwiseFeedForward + residual + LayerNorm + mask in one launch (fs2_ffn): bf16 rows of
    256 (padded [B, T, 256] or packed [B*T, 256] in ``layout``); ``w_packed`` from
    :func:`pack_ffn_weights`. The hidden [rows, F] never reaches HBM. ``tile_rows`` (112 / 96 / 64) and
    ``nsplit`` (workgroups per row tile): None = :func:`ffn_form` of the row count the host knows
    (``layout.rows_hint`` or the capacity). ``next_qkv`` = (wqkv in :func:`pack_frag_rows` order,
    bqkv f32): the epilogue also projects the output rows to the next block's Q|K|V; returns
    (out, qkv) then (qkv None otherwise). ``pre`` = (att, wfc in :func:`pack_frag_rows` order, bfc,
    (gamma1, beta1, eps1)): x is the FFT block's input and the FFN input h = LN1(att wfc^T + bfc + x)
    is computed in the launch's prologue (:func:`ffn_pre_ok` forms only)."""
    _gpu(x, w_packed, b1, b2, lens, addvec1, addvec2)
    if x.dtype != torch.bfloat16 or w_packed.dtype != torch.bfloat16:
        raise TypeError("fs2amd.ffn: bf16 activations and weights only")
    if layout is not None:
        B, T = layout.B, layout.T
        assert x.dim() == 2 and x.shape[0] == layout.capacity, (tuple(x.shape), layout.capacity)
    else:
        B, T, _ = x.shape
    D = x.shape[-1]
    F = b1.numel()
    assert w_packed.is_contiguous() and w_packed.numel() == _lib.fs2_ffn_weight_elems(ks, F), tuple(w_packed.shape)
    d = L.FfnDesc()
    d.x, d.x_row_stride = x.data_ptr(), _rows(x, "x")
    d.w, d.b1, d.b2 = w_packed.data_ptr(), b1.data_ptr(), b2.data_ptr()
    d.B, d.T, d.D, d.F, d.KS, d.pad = B, T, D, F, ks, pad
    g, b, eps = ln
    d.ln_gamma, d.ln_beta, d.ln_eps = g.data_ptr(), b.data_ptr(), float(eps)
    if lens is not None:
        assert lens.dtype == torch.int64 and lens.numel() == B
        d.lens = lens.data_ptr()
    if addvec1 is not None:
        d.addvec1 = addvec1.data_ptr()
    if addvec2 is not None:
        d.addvec2 = addvec2.data_ptr()
    if layout is not None:
        d.rows_dev, d.row_pos = layout.rows_dev, layout.row_pos.data_ptr()
    if out is None:
        out = torch.empty_like(x)
    d.out, d.out_row_stride = out.data_ptr(), _rows(out, "out")
    rows = ffn_launch_rows(x, layout)
    if layout is not None and rows < layout.capacity:
        d.rows_max = int(rows)  # free-running: the active rows from the one host read
    tr, ns = ffn_form(rows, F)
    if tile_rows is None:
        tile_rows = tr if nsplit is None else 112
    if nsplit is None:
        nsplit = ns
    d.tile_rows = int(tile_rows)
    if nsplit > 1:
        ws = splitk_workspace(x.device)
        if ws is None:
            raise RuntimeError("fs2amd.ffn: nsplit > 1 needs the split-K workspace (ops.splitk_enabled)")
        d.nsplit, d.splitk_ws, d.splitk_ws_bytes = int(nsplit), ws.data_ptr(), ws.numel()
    qkv = None
    if next_qkv is not None:
        wq, bq = next_qkv
        nq = bq.numel()
        assert wq.is_contiguous() and wq.numel() == nq * D, (tuple(wq.shape), nq, D)
        qkv = torch.empty(*x.shape[:-1], nq, device=x.device, dtype=torch.bfloat16)
        d.wqkv, d.bqkv, d.qkv_out, d.qkv_row_stride, d.nqkv = wq.data_ptr(), bq.data_ptr(), qkv.data_ptr(), nq, nq
    if pre is not None:
        att, wfc, bfc, (g1, b1n, eps1) = pre
        _gpu(att, wfc, bfc, g1, b1n)
        assert att.shape == x.shape and att.dtype == torch.bfloat16 and wfc.numel() == D * D
        d.pre_att, d.pre_att_row_stride = att.data_ptr(), _rows(att, "att")
        d.pre_w, d.pre_b, d.pre_gamma, d.pre_beta, d.pre_eps = wfc.data_ptr(), bfc.data_ptr(), g1.data_ptr(), \
            b1n.data_ptr(), float(eps1)
    L.check(_lib.fs2_ffn(ctypes.byref(d), _stream(x)), "fs2_ffn")
    return (out, qkv) if next_qkv is not None else out


WIDE_MAX_ROWS = 16384  # fs2_ffn_wide below this many rows (the fused 112-row tiles fill the chip above it)


def ffn_wide_ok(rows, F, ks):
    """fs2_ffn_wide's shapes: F in {512, 1024}, kernel 9 or 3, rows within its workspace (the
    f32 pre-norm rows: 1 KiB per row in the split-K workspace) and below WIDE_MAX_ROWS.
    FS2_FFN_WIDE=0 keeps the fused split-hidden launch (A/B)."""
    return (os.environ.get("FS2_FFN_WIDE", "1") != "0" and _splitk_on[0] and F in (512, 1024) and ks in (3, 9)
            and 0 < rows <= WIDE_MAX_ROWS and 4096 + rows * 1024 <= SPLITK_WS_BYTES)


def ffn_wide(x, w_packed, b1, b2, *, ks, pad, ln, lens=None, addvec1=None, addvec2=None, layout=None, out=None):
    """fs2_ffn_wide: the FFN of :func:`ffn` (same weights, masks, addvecs, padded or packed rows) as
    two wide-tile launches for small row counts: the [rows, F] hidden goes through a bf16 buffer
    (8 MB at the cfg2 encoder's 4k rows, L2 / MALL resident) and the LayerNorm is finished by the
    last of 4 column-quarter workgroups per 64-row tile."""
    _gpu(x, w_packed, b1, b2, lens, addvec1, addvec2)
    if x.dtype != torch.bfloat16 or w_packed.dtype != torch.bfloat16:
        raise TypeError("fs2amd.ffn_wide: bf16 activations and weights only")
    if layout is not None:
        B, T = layout.B, layout.T
        assert x.dim() == 2 and x.shape[0] == layout.capacity, (tuple(x.shape), layout.capacity)
    else:
        B, T, _ = x.shape
    D = x.shape[-1]
    F = b1.numel()
    assert w_packed.is_contiguous() and w_packed.numel() == _lib.fs2_ffn_weight_elems(ks, F), tuple(w_packed.shape)
    d = L.FfnDesc()
    d.x, d.x_row_stride = x.data_ptr(), _rows(x, "x")
    d.w, d.b1, d.b2 = w_packed.data_ptr(), b1.data_ptr(), b2.data_ptr()
    d.B, d.T, d.D, d.F, d.KS, d.pad = B, T, D, F, ks, pad
    g, b, eps = ln
    d.ln_gamma, d.ln_beta, d.ln_eps = g.data_ptr(), b.data_ptr(), float(eps)
    if lens is not None:
        assert lens.dtype == torch.int64 and lens.numel() == B
        d.lens = lens.data_ptr()
    if addvec1 is not None:
        d.addvec1 = addvec1.data_ptr()
    if addvec2 is not None:
        d.addvec2 = addvec2.data_ptr()
    if layout is not None:
        d.rows_dev, d.row_pos = layout.rows_dev, layout.row_pos.data_ptr()
    if out is None:
        out = torch.empty_like(x)
    d.out, d.out_row_stride = out.data_ptr(), _rows(out, "out")
    rows = ffn_launch_rows(x, layout)
    if layout is not None and rows < layout.capacity:
        d.rows_max = int(rows)
    ws = splitk_workspace(x.device)
    if ws is None or not ffn_wide_ok(rows, F, ks):
        raise RuntimeError(f"fs2amd.ffn_wide: {rows} rows / F {F} / k {ks} not covered (ops.ffn_wide_ok)")
    d.splitk_ws, d.splitk_ws_bytes = ws.data_ptr(), ws.numel()
    hidden = torch.empty(rows, F, device=x.device, dtype=torch.bfloat16)
    L.check(_lib.fs2_ffn_wide(ctypes.byref(d), hidden.data_ptr(), hidden.numel() * 2, _stream(x)), "fs2_ffn_wide")
    return out


def _check_attention_args(qkv, lens, B, n_head, d_k, layout):
    """The kernels read int64 key lengths, B of them, and a fused Q|K|V row of 3*H*dk values: a
    mismatch would read the wrong lengths or past the buffers, so it raises here."""
    if qkv.shape[-1] != 3 * n_head * d_k:
        raise ValueError(f"attention: qkv has {qkv.shape[-1]} columns, expected 3*n_head*d_k = {3 * n_head * d_k}")
    if layout is None:
        if lens is None or lens.dtype != torch.int64 or lens.dim() != 1 or lens.numel() != B:
            raise ValueError(f"attention: lens must be an int64 vector of the B = {B} key lengths, got "
                             f"{None if lens is None else (lens.dtype, tuple(lens.shape))}")


def attention(qkv, lens, n_head, d_k, temperature, out=None, layout=None, lse=None):
    """Key-padding-masked multi-head self-attention over a fused [B, T, 3*H*dk] projection
    (or packed [B*T, 3*H*dk] rows of a SeqLayout: lens unused). lse: optional f32 [rows, H] that
    receives the softmax statistics for :func:`attention_bwd`."""
    _gpu(qkv, lens)
    if layout is not None:
        B, T = layout.B, layout.T
        shape = (layout.capacity, n_head * d_k)
    else:
        B, T, _ = qkv.shape
        shape = (B, T, n_head * d_k)
    _check_attention_args(qkv, lens, B, n_head, d_k, layout)
    if out is None:
        out = torch.empty(*shape, device=qkv.device, dtype=qkv.dtype)
    ws, ws_bytes, rows_max = None, 0, 0
    if attention_split_on(B, T, n_head, layout, lse, qkv.dtype):
        ws, ws_bytes, rows_max = _attn_split_items(layout, B, T, n_head, qkv)
    L.check(_lib.fs2_attention_ex(_ptr(qkv), _dt(qkv), _rows(qkv, "qkv"), _ptr(lens), B, T, n_head, d_k,
                                  float(temperature), _ptr(out), _rows(out, "out"),
                                  _ptr(layout.cu) if layout is not None else None, _ptr(lse),
                                  attention_waves(B, T, layout), _ptr(ws), ws_bytes, rows_max, _stream(qkv)),
            "fs2_attention_ex")
    return out


def attention_split_on(B, T, H, layout, lse, dtype):
    """Key-split attention (fs2_attention_ex split_ws): packed rows whose active row count the host
    knows (free-running synthesis sets layout.rows_hint), 256 < T <= 2048, bf16, inference (no lse).
    The split arithmetic depends on each sequence's length only, so every T bucket of a batch gives
    the same result. FS2_ATTN_SPLIT=0 turns it off."""
    if os.environ.get("FS2_ATTN_SPLIT", "1") == "0" or lse is not None or dtype != torch.bfloat16:
        return False
    if layout is None or getattr(layout, "rows_hint", None) is None:
        return False
    return _lib.fs2_attention_split_ws_bytes(B, T, H, int(layout.rows_hint)) > 0


def _attn_split_items(layout, B, T, H, like):
    """The layout's key-split workspace with its work list (fs2_attention_items: one launch per
    layout, reused by every layer; it also zeroes the arrival counters). The workspace is owned by
    the layout, so a captured graph keeps its own."""
    rows_max = int(layout.rows_hint)
    nbytes = _lib.fs2_attention_split_ws_bytes(B, T, H, rows_max)
    st = getattr(layout, "_attn_split", None)
    if st is None or st[1] != nbytes:
        ws = torch.empty(nbytes, device=like.device, dtype=torch.uint8)
        L.check(_lib.fs2_attention_items(_ptr(layout.cu), B, T, H, _ptr(ws), nbytes, rows_max, _stream(like)),
                "fs2_attention_items")
        st = layout._attn_split = (ws, nbytes)
    return st[0], nbytes, rows_max


def attention_waves(B, T, layout=None):
    """fs2_attention_ex's work-shape hint: 8 waves (256-query tiles) for long, dense sequences —
    64 < T <= 512 and, when the host knows the packed row count (free-running synthesis sets
    layout.rows_hint), at least 70 % of B * T valid; else 4. (Teacher-forced batches, whose row
    count the host does not see, are taken as dense.) Results do not depend on it."""
    if not 64 < T <= 512:
        return 4
    rows = getattr(layout, "rows_hint", None) if layout is not None else None
    return 8 if rows is None or rows >= 0.7 * B * T else 4


def enc_attn_block(x, lens, wqkv_frag, bqkv, wfc_frag, bfc, ln, n_head, d_k, temperature, out=None, embed=None,
                   masks=None, cond=None):
    """fs2_enc_attn_block: the encoder FFT block's attention sub-layer (Q|K|V projection, masked
    2-head attention, fc + residual + LayerNorm, padded rows zeroed) in one launch, bf16
    [B, L <= 64, 256] -> bf16 [B, L, 256]. Weights in fragment order (:func:`pack_frag_rows`).
    embed = (tokens int64 [B, L], table f32 [vocab, 256], pe f32 [>= L, 256]) instead of x
    (fs2_enc_embed_attn_block: the first block builds its input as fs2_embed_pe would); masks =
    (src_mask bool [B, L], mel_lens | None, mel_mask bool [B, T_mel] | None) filled as
    fs2_length_masks by that launch. cond (with embed) = the arguments of :func:`cond_vectors`
    (speakers, spk_table, emotions, arousals, valences, emo_table, aro_table, val_table, lin_w,
    lin_b): extra workgroups of the same launch compute them; returns (out, spk_vec, emo_vec)."""
    if embed is not None:
        tokens, table, pe = embed
        _gpu(tokens, table, pe, lens, wqkv_frag, bqkv, wfc_frag, bfc)
        B, Lx = tokens.shape
        D = table.shape[1]
        assert tokens.dtype == torch.int64 and tokens.is_contiguous() and table.dtype == torch.float32 \
            and pe.dtype == torch.float32 and pe.shape[0] >= Lx and D == n_head * d_k
        assert lens.dtype == torch.int64 and lens.numel() == B, (lens.dtype, lens.numel(), B)
        g, b, eps = ln
        if out is None:
            out = torch.empty(B, Lx, D, device=tokens.device, dtype=torch.bfloat16)
        src_mask = mel_lens = mel_mask = None
        T_mel = 0
        if masks is not None:
            src_mask, mel_lens, mel_mask = masks
            assert src_mask.dtype == torch.bool and tuple(src_mask.shape) == (B, Lx)
            if mel_mask is not None:
                assert mel_mask.dtype == torch.bool and mel_mask.shape[0] == B and mel_lens.dtype == torch.int64
                T_mel = mel_mask.shape[1]
        cd = None
        spk_out = emo_out = None
        if cond is not None:
            speakers, spk_table, emotions, arousals, valences, emo_table, aro_table, val_table, lin_w, lin_b = cond
            _gpu(speakers, spk_table, emotions, arousals, valences, emo_table, aro_table, val_table, lin_w, lin_b)
            cd = L.CondDesc()
            if spk_table is not None:
                spk_out = torch.empty(B, D, device=tokens.device)
                cd.speakers, cd.speaker_table, cd.n_speaker = _ptr(speakers), _ptr(spk_table), spk_table.shape[0]
                cd.spk_out = _ptr(spk_out)
            if emo_table is not None:
                emo_out = torch.empty(B, D, device=tokens.device)
                cd.emotions, cd.emo_table, cd.n_emo, cd.d_emo = _ptr(emotions), _ptr(emo_table), emo_table.shape[0], \
                    emo_table.shape[1]
                cd.arousals, cd.aro_table, cd.n_aro, cd.d_aro = _ptr(arousals), _ptr(aro_table), aro_table.shape[0], \
                    aro_table.shape[1]
                cd.valences, cd.val_table, cd.n_val, cd.d_val = _ptr(valences), _ptr(val_table), val_table.shape[0], \
                    val_table.shape[1]
                cd.lin_w, cd.lin_b, cd.emo_out = _ptr(lin_w), _ptr(lin_b), _ptr(emo_out)
        L.check(_lib.fs2_enc_embed_attn_block(
            _ptr(tokens), _ptr(table), table.shape[0], _ptr(pe), _ptr(bad_id_counter(tokens.device)), _ptr(lens), B, Lx,
            _ptr(wqkv_frag), _ptr(bqkv), _ptr(wfc_frag), _ptr(bfc), _ptr(g), _ptr(b), float(eps), n_head, d_k,
            float(temperature), _ptr(out), _ptr(src_mask), _ptr(mel_lens), T_mel, _ptr(mel_mask),
            ctypes.byref(cd) if cd is not None else None, *_enc_ws(tokens.device), _stream(tokens)),
            "fs2_enc_embed_attn_block")
        return (out, spk_out, emo_out) if cond is not None else out
    _gpu(x, lens, wqkv_frag, bqkv, wfc_frag, bfc)
    B, Lx, D = x.shape
    assert x.dtype == torch.bfloat16 and x.is_contiguous() and D == n_head * d_k, (x.dtype, tuple(x.shape))
    assert lens.dtype == torch.int64 and lens.numel() == B, (lens.dtype, lens.numel(), B)
    assert wqkv_frag.dtype == torch.bfloat16 and wqkv_frag.numel() == 3 * D * D and bqkv.numel() == 3 * D
    assert wfc_frag.dtype == torch.bfloat16 and wfc_frag.numel() == D * D and bfc.numel() == D
    g, b, eps = ln
    if out is None:
        out = torch.empty_like(x)
    L.check(_lib.fs2_enc_attn_block(_ptr(x), _ptr(lens), B, Lx, _ptr(wqkv_frag), _ptr(bqkv), _ptr(wfc_frag),
                                    _ptr(bfc), _ptr(g), _ptr(b), float(eps), n_head, d_k, float(temperature),
                                    _ptr(out), *_enc_ws(x.device), _stream(x)), "fs2_enc_attn_block")
    return out


def _enc_ws(device):
    """(pointer, bytes) of the split-K workspace for fs2_enc_attn_block's head-split form
    (FS2_ENC_HALF=1, A/B: measured no faster than one workgroup per utterance, profiles/r5y), or
    (None, 0): one workgroup per utterance (the default). FS2_ENC_TRACE=1 (trace builds): the
    workspace carries the phase stamps."""
    if os.environ.get("FS2_ENC_HALF", "0") != "1" and os.environ.get("FS2_ENC_TRACE", "0") != "1":
        return None, 0
    ws = splitk_workspace(device)
    return (None, 0) if ws is None else (ws.data_ptr(), ws.numel())


_bad_ids = {}


def bad_id_counter(device):
    """Per-device int32 count of out-of-vocabulary token ids seen by fs2_embed_pe (their rows
    are NaN). Allocated zeroed on first use outside graph capture."""
    if device.type != "cuda":
        return None
    c = _bad_ids.get(device.index)
    if c is None and not torch.cuda.is_current_stream_capturing():
        c = _bad_ids[device.index] = torch.zeros(1, dtype=torch.int32, device=device)
    return c


def raise_if_bad_ids(device):
    """IndexError (the reference's nn.Embedding error) if any forward on ``device`` met an
    out-of-vocabulary token id since the last check; one device->host read."""
    c = _bad_ids.get(device.index) if device.type == "cuda" else None
    if c is not None:
        n = int(c.item())
        if n:
            c.zero_()
            raise IndexError(f"fs2amd: {n} token id(s) outside the embedding table (their encoder rows are NaN)")


def attention_bwd(qkv, out, dout, lens, n_head, d_k, temperature, layout=None, lse=None):
    """Gradient of :func:`attention` (fs2_attention_bwd): dqkv f32 with qkv's shape. qkv / out in
    the forward's dtype (the MFMA operand type), dout f32."""
    _gpu(qkv, out, dout, lens)
    dout = dout.float().contiguous()
    if layout is not None:
        B, T = layout.B, layout.T
    else:
        B, T, _ = qkv.shape
    _check_attention_args(qkv, lens, B, n_head, d_k, layout)
    dqkv = torch.empty(qkv.shape, device=qkv.device, dtype=torch.float32)
    ws = torch.empty(2 * B * T * n_head, device=qkv.device, dtype=torch.float32)
    L.check(_lib.fs2_attention_bwd(_ptr(qkv), _dt(qkv), _rows(qkv, "qkv"), _ptr(out), _rows(out, "out"), _ptr(dout),
                                   _rows(dout, "dout"), _ptr(lens) if layout is None else None, B, T, n_head, d_k,
                                   float(temperature), _ptr(dqkv), _rows(dqkv, "dqkv"),
                                   _ptr(layout.cu) if layout is not None else None, _ptr(ws), ws.numel() * 4,
                                   _ptr(lse), _stream(qkv)), "fs2_attention_bwd")
    return dqkv


def embed_pe(tokens, table, pe, out_dtype):
    _gpu(tokens, table, pe)
    B, Lx = tokens.shape
    D = table.shape[1]
    out = torch.empty(B, Lx, D, device=tokens.device, dtype=torch_dtype(out_dtype))
    L.check(_lib.fs2_embed_pe(_ptr(tokens.contiguous()), _ptr(table), table.shape[0], _ptr(pe), B, Lx, D, _ptr(out),
                              out_dtype, _ptr(bad_id_counter(tokens.device)), _stream(tokens)), "fs2_embed_pe")
    return out


def cond_vectors(speakers, spk_table, emotions, arousals, valences, emo_table, aro_table, val_table, lin_w, lin_b, D):
    ref = speakers if speakers is not None else emotions
    _gpu(ref)
    B = ref.shape[0]
    spk_out = torch.empty(B, D, device=ref.device) if spk_table is not None else None
    emo_out = torch.empty(B, D, device=ref.device) if emo_table is not None else None
    d_emo = emo_table.shape[1] if emo_table is not None else 0
    d_aro = aro_table.shape[1] if aro_table is not None else 0
    d_val = val_table.shape[1] if val_table is not None else 0
    L.check(_lib.fs2_cond_vectors(
        _ptr(speakers), _ptr(spk_table), spk_table.shape[0] if spk_table is not None else 0,
        _ptr(emotions), _ptr(emo_table), emo_table.shape[0] if emo_table is not None else 0, d_emo,
        _ptr(arousals), _ptr(aro_table), aro_table.shape[0] if aro_table is not None else 0, d_aro,
        _ptr(valences), _ptr(val_table), val_table.shape[0] if val_table is not None else 0, d_val,
        _ptr(lin_w), _ptr(lin_b), B, D, _ptr(spk_out), _ptr(emo_out), _stream(ref)), "fs2_cond_vectors")
    return spk_out, emo_out


def cond_bwd(dy, speakers, spk_table, emotions, arousals, valences, emo_table, aro_table, val_table, lin_w, emo_out,
             d_spk=None, d_emo=None, d_aro=None, d_val=None, d_w=None, d_b=None):
    """Backward of y = x + spk_out[b] + emo_out[b] (fs2_cond_bwd): ACCUMULATES the speaker /
    emotion / arousal / valence table gradients and the emotion Linear's weight / bias gradients
    into the given tensors (None: skipped). dy [B, L, D] f32. The gradient of x is dy itself."""
    _gpu(dy, speakers, spk_table, emotions, emo_table, lin_w, emo_out)
    dy = dy.contiguous()
    assert dy.dtype == torch.float32 and dy.dim() == 3
    B, Lx, D = dy.shape
    cd = L.CondDesc()
    if spk_table is not None:
        cd.speakers, cd.speaker_table, cd.n_speaker = _ptr(speakers), _ptr(spk_table), spk_table.shape[0]
    if emo_table is not None:
        cd.emotions, cd.emo_table, cd.n_emo, cd.d_emo = _ptr(emotions), _ptr(emo_table), emo_table.shape[0], \
            emo_table.shape[1]
        cd.arousals, cd.aro_table, cd.n_aro, cd.d_aro = _ptr(arousals), _ptr(aro_table), aro_table.shape[0], \
            aro_table.shape[1]
        cd.valences, cd.val_table, cd.n_val, cd.d_val = _ptr(valences), _ptr(val_table), val_table.shape[0], \
            val_table.shape[1]
        cd.lin_w, cd.emo_out = _ptr(lin_w), _ptr(emo_out)
    gr = L.CondGrads()
    gr.d_speaker_table, gr.d_emo_table, gr.d_aro_table, gr.d_val_table, gr.d_lin_w, gr.d_lin_b = (
        _ptr(d_spk), _ptr(d_emo), _ptr(d_aro), _ptr(d_val), _ptr(d_w), _ptr(d_b))
    ws = torch.empty(max(1, _lib.fs2_cond_bwd_ws_bytes(B, D) // 4), device=dy.device, dtype=torch.float32)
    L.check(_lib.fs2_cond_bwd(_ptr(dy), B, Lx, D, ctypes.byref(cd), ctypes.byref(gr), _ptr(ws), ws.numel() * 4,
                              _stream(dy)), "fs2_cond_bwd")


def variance_embed(x, pred, target, control, bins, table):
    """In place: pred *= control (no target); x += table[bucketize(target or pred, bins)]."""
    _gpu(x, pred, target, bins, table)
    M = pred.numel()
    D = x.shape[-1]
    L.check(_lib.fs2_variance_embed(_ptr(x), _dt(x), _ptr(pred), _ptr(target), float(control), _ptr(bins),
                                    bins.numel() + 1, _ptr(table), M, D, _stream(x)), "fs2_variance_embed")


def vp_norm(y, gamma, beta, eps, out=None):
    """fs2_vp_norm: y f32 [rows, G*256] (relu(conv1) of G variance predictors) -> LayerNorm per
    group -> bf16 [rows, G*512]: group g's hi plane at g*512, lo plane at g*512 + 256."""
    _gpu(y, gamma, beta)
    G = gamma.numel() // 256
    rows = y.numel() // y.shape[-1]
    if out is None:
        out = torch.empty(*y.shape[:-1], G * 512, device=y.device, dtype=torch.bfloat16)
    L.check(_lib.fs2_vp_norm(_ptr(y), _rows(y, "y"), rows, G, 256, _ptr(gamma), _ptr(beta), float(eps), _ptr(out),
                             _rows(out, "out"), _stream(y)), "fs2_vp_norm")
    return out


def vp_head(y, gamma, beta, eps, lin_w, lin_b, lens, embed=None):
    """fs2_vp_head: y f32 [B, T, G*256] (relu(conv2)) -> per group LayerNorm, Linear(256->1), masked
    -> pred f32 [G, B, T]. embed = (g, x, target, control, bins, table): group g's value also does
    the pitch / energy embedding add into x in place (fs2_variance_embed semantics)."""
    _gpu(y, gamma, beta, lin_w, lin_b, lens)
    B, T, _ = y.shape
    G = gamma.numel() // 256
    assert lens.dtype == torch.int64 and lens.numel() == B
    pred = torch.empty(G, B, T, device=y.device, dtype=torch.float32)
    eg, x, target, control, bins, table = embed if embed is not None else (-1, None, None, 1.0, None, None)
    if x is not None:
        _gpu(x, target, bins, table)
        assert x.shape[:2] == (B, T) and table.shape[1] == x.shape[-1]
        if target is not None:
            assert target.dtype == torch.float32 and target.is_contiguous() and target.numel() == B * T
    L.check(_lib.fs2_vp_head(_ptr(y), _rows(y, "y"), B, T, G, 256, _ptr(gamma), _ptr(beta), float(eps), _ptr(lin_w),
                             _ptr(lin_b), _ptr(lens), _ptr(pred), int(eg), _ptr(x), _dt(x) if x is not None else 0,
                             _rows(x, "x") if x is not None else 0, x.shape[-1] if x is not None else 0,
                             _ptr(target), float(control), _ptr(bins),
                             bins.numel() + 1 if bins is not None else 0, _ptr(table), _stream(y)), "fs2_vp_head")
    return pred


def pack_vp_fused(convs):
    """The fs2_vp_fused weight buffer of G VariancePredictors: ``convs`` = [(conv1.weight,
    conv2.weight), ...] (nn.Conv1d [256, 256, 3] each). Per predictor and conv, K = (tap, channel)
    flattened, split into bf16 parts w = w_hi + w_lo, each in pack_frag_rows order; a wave's stream
    [2 convs][24 k-steps][hi, lo] is contiguous (include/fs2hip.h)."""
    out = []
    for pair in convs:
        per_conv = []
        for w in pair:
            w = w.detach().float()
            N, cin, ks = w.shape
            k = w.permute(0, 2, 1).reshape(N, ks * cin)
            hi = k.to(torch.bfloat16).float()
            lo = (k - hi).to(torch.bfloat16).float()
            parts = [pack_frag_rows(t).view(N // 64, ks * cin // 32, 2048) for t in (hi, lo)]
            per_conv.append(torch.stack(parts, 2))  # [N/64][K/32][2][2048]
        out.append(torch.stack(per_conv, 1).reshape(-1))  # [N/64][2 convs][K/32][2][2048]
    return torch.cat(out).contiguous()


def vp_fused(x, F, lens, embed=None):
    """fs2_vp_fused: F.G VariancePredictors (bf16x3) on bf16 rows x [B, L, 256] in one launch ->
    pred f32 [G, B, L]; embed = (g, target, control, bins, table): group g also writes
    x_out = x + table[bucketize(...)] (a new tensor; returned as the second value, else None)."""
    _gpu(x, F.w, F.vec, F.lin_b, lens)
    if x.dtype != torch.bfloat16 or x.shape[-1] != 256:
        raise TypeError("fs2amd.vp_fused: bf16 [B, L, 256] input only")
    B, Lx, _ = x.shape
    assert lens.dtype == torch.int64 and lens.numel() == B
    assert F.w.numel() == _lib.fs2_vp_fused_weight_elems(F.G)
    pred = torch.empty(F.G, B, Lx, device=x.device, dtype=torch.float32)
    d = L.VpFusedDesc()
    d.x, d.x_row_stride = x.data_ptr(), _rows(x, "x")
    d.w, d.vec, d.lin_b, d.ln_eps = F.w.data_ptr(), F.vec.data_ptr(), F.lin_b.data_ptr(), float(F.eps)
    d.B, d.L, d.G = B, Lx, F.G
    d.lens, d.pred, d.embed_group = lens.data_ptr(), pred.data_ptr(), -1
    x_out = None
    if embed is not None:
        g, target, control, bins, table = embed
        _gpu(target, bins, table)
        assert table.shape[1] == 256 and table.dtype == torch.float32 and bins.dtype == torch.float32
        if target is not None:
            assert target.dtype == torch.float32 and target.is_contiguous() and target.numel() == B * Lx
        x_out = torch.empty_like(x)
        d.embed_group = int(g)
        d.x_out, d.x_out_row_stride = x_out.data_ptr(), 256
        d.target, d.control = (target.data_ptr() if target is not None else None), float(control)
        d.bins, d.n_bins, d.table = bins.data_ptr(), bins.numel() + 1, table.data_ptr()
    L.check(_lib.fs2_vp_fused(ctypes.byref(d), _stream(x)), "fs2_vp_fused")
    return pred, x_out


def length_mask(lens, width):
    """get_mask_from_lengths (utils/tools.py:152-160) in one launch: bool [B, width], True = pad."""
    _gpu(lens)
    lens = lens.to(torch.int64).contiguous()
    B = lens.shape[0]
    mask = torch.empty(B, int(width), device=lens.device, dtype=torch.bool)
    L.check(_lib.fs2_length_masks(_ptr(lens), B, int(width), _ptr(mask), _stream(lens)), "fs2_length_masks")
    return mask


def _dur_kind(dur, logpred):
    if logpred:
        return L.DUR_LOGPRED
    if dur.dtype == torch.int64:
        return L.DUR_I64
    if dur.dtype == torch.float32:
        return L.DUR_F32
    raise TypeError(f"fs2amd: durations must be int64 or float32, got {dur.dtype}")


def pack_rows(lay, a, b=None):
    """Padded [B, T, C] rows -> packed [capacity, C] rows of SeqLayout ``lay`` (fs2_pack_rows); a
    second tensor ``b`` in the same launch. Rows past the layout's active rows are not written."""
    _gpu(a, b)
    outs = []
    for t in (a, b):
        if t is None:
            outs.append(None)
            continue
        assert t.is_contiguous() and t.shape[0] * t.shape[1] == lay.capacity, (tuple(t.shape), lay.capacity)
        outs.append(torch.empty(lay.capacity, t.shape[-1], device=t.device, dtype=t.dtype))
    rb = lambda t: t.shape[-1] * t.element_size()
    L.check(_lib.fs2_pack_rows(_ptr(a), rb(a), _ptr(outs[0]), _ptr(b), rb(b) if b is not None else 0, _ptr(outs[1]),
                               _ptr(lay.rowmap), lay.capacity, _stream(a)), "fs2_pack_rows")
    return outs[0], outs[1]


def postnet_assemble(y, lay, const_row, tail):
    """The PostNet valid-region output back to [B, T, C] f32 (fs2_postnet_assemble; each
    utterance's exact rows from the margin layout ``lay``)."""
    _gpu(y, const_row, tail)
    C = y.shape[-1]
    out = torch.empty(lay.B, lay.T, C, device=y.device, dtype=torch.float32)
    L.check(_lib.fs2_postnet_assemble(_ptr(y), _ptr(lay.rowmap), _ptr(lay.cu), lay.B, lay.T, C, _ptr(const_row),
                                      _ptr(tail), tail.shape[0], _ptr(out), _stream(y)), "fs2_postnet_assemble")
    return out


def len_stats(lens, bad=None):
    """int32 [max(lens), sum(lens), *bad or 0] on the device in one launch (fs2_len_stats)."""
    _gpu(lens, bad)
    lens = lens.to(torch.int64).contiguous()
    meta = torch.empty(3, device=lens.device, dtype=torch.int32)
    L.check(_lib.fs2_len_stats(_ptr(lens), lens.numel(), _ptr(bad), _ptr(meta), _stream(lens)), "fs2_len_stats")
    return meta


def lr_durations(dur, logpred=False, d_control=1.0):
    """Frame counts -> (cum int32 [B, L], mel_len int64 [B], d_rounded f32 [B, L] or None)."""
    _gpu(dur)
    dur = dur.contiguous()
    B, Lx = dur.shape
    cum = torch.empty(B, Lx, device=dur.device, dtype=torch.int32)
    mel_len = torch.empty(B, device=dur.device, dtype=torch.int64)
    d_rounded = torch.empty(B, Lx, device=dur.device, dtype=torch.float32) if logpred else None
    L.check(_lib.fs2_lr_durations(_ptr(dur), _dur_kind(dur, logpred), float(d_control), B, Lx, _ptr(cum),
                                  _ptr(mel_len), _ptr(d_rounded), _stream(dur)), "fs2_lr_durations")
    return cum, mel_len, d_rounded


def lr_expand(x, cum, mel_len, T_out, pe=None, out_dtype=None, index_map=False, out_layout=None, map_only=False):
    """Frame gather (+ PE). out_layout: write only the SeqLayout's frames, packed [B*T_out, D].
    map_only: return only the int32 [B, T_out] source-index map (no frames are moved)."""
    _gpu(x, cum, mel_len, pe)
    x = x.contiguous()
    B, Lx, D = x.shape
    od = _dt(x) if out_dtype is None else out_dtype
    if map_only:
        im = torch.empty(B, T_out, device=x.device, dtype=torch.int32)
        L.check(_lib.fs2_lr_expand(_ptr(x), _dt(x), _ptr(cum), _ptr(mel_len), B, Lx, D, T_out, None, None, od,
                                   _ptr(im), None, _stream(x)), "fs2_lr_expand")
        return im
    if out_layout is not None:
        assert out_layout.B == B and out_layout.T == T_out
        out = out_layout.empty(D, torch_dtype(od))
    else:
        out = torch.empty(B, T_out, D, device=x.device, dtype=torch_dtype(od))
    im = torch.empty(B, T_out, device=x.device, dtype=torch.int32) if index_map else None
    L.check(_lib.fs2_lr_expand(_ptr(x), _dt(x), _ptr(cum), _ptr(mel_len), B, Lx, D, T_out, _ptr(pe), _ptr(out), od,
                               _ptr(im), _ptr(out_layout.cu) if out_layout is not None else None, _stream(x)),
            "fs2_lr_expand")
    return (out, im) if index_map else out


def lr_backward(dy, cum, n_phonemes):
    """fs2_lr_backward: gradient of the LengthRegulator gather, dy f32 [B, T, D] -> dx f32
    [B, n_phonemes, D] (per phoneme the sum of dy over its frames [cum[i-1], cum[i]) below T, in
    frame order: deterministic)."""
    _gpu(dy, cum)
    dy = dy.float().contiguous()
    B, T, D = dy.shape
    if tuple(cum.shape) != (B, n_phonemes) or cum.dtype != torch.int32:
        raise ValueError(f"lr_backward: cum must be int32 [{B}, {n_phonemes}], got {cum.dtype} {tuple(cum.shape)}")
    dx = torch.empty(B, n_phonemes, D, device=dy.device, dtype=torch.float32)
    L.check(_lib.fs2_lr_backward(_ptr(dy), _ptr(cum.contiguous()), B, int(n_phonemes), D, T, _ptr(dx), _stream(dy)),
            "fs2_lr_backward")
    return dx


def variance_embed_ex(x, value, bins, table):
    """fs2_variance_embed_ex (training form, out of place): idx = bucketize(value, bins) (int64,
    torch.bucketize's right=False), out = x + table[idx]. Returns (out, idx)."""
    _gpu(x, value, bins, table)
    x = x.contiguous()
    value = value.detach().float().contiguous()
    M = value.numel()
    D = x.shape[-1]
    if x.numel() != M * D:
        raise ValueError(f"variance_embed_ex: x {tuple(x.shape)} vs {M} values")
    out = torch.empty_like(x)
    idx = torch.empty(value.shape, device=x.device, dtype=torch.int64)
    L.check(_lib.fs2_variance_embed_ex(_ptr(x), _dt(x), _ptr(value), _ptr(bins), bins.numel() + 1, _ptr(table), M, D,
                                       _ptr(out), _ptr(idx), _stream(x)), "fs2_variance_embed_ex")
    return out, idx


def lr_fused(x, lens, T_out, pe=None, out_dtype=None, dur=None, logpred=False, d_control=1.0, cum=None, mel_len=None,
             proj=None):
    """fs2_lr_fused: LengthRegulator gather (+ PE) into the packed decoder rows of the layout of
    ``lens`` over T_out, the layout built by the same launch. Durations scanned here (``dur``:
    returns (out, layout, cum, mel_len, d_rounded)) or from fs2_lr_durations (``cum``, ``mel_len``:
    returns (out, layout)). ``proj`` = (proj_src f32 [B*Lx, NP], proj_pe f32 [>= T_out, NP])
    (fs2_lr_fused_proj): the packed bf16 rows bf16(proj_src[src] + proj_pe[t]) come back as one
    more trailing result."""
    _gpu(x, lens, pe, dur, cum, mel_len)
    x = x.contiguous()
    B, Lx, D = x.shape
    dev = x.device
    od = _dt(x) if out_dtype is None else out_dtype
    lens = lens.to(torch.int64).contiguous()
    lay = SeqLayout.deferred(B, T_out, dev)
    out = lay.empty(D, torch_dtype(od))
    psrc = ppe = pout = None
    NP = 0
    if proj is not None:
        psrc, ppe = proj
        _gpu(psrc, ppe)
        NP = psrc.shape[-1]
        assert psrc.dtype == torch.float32 and ppe.dtype == torch.float32 and psrc.is_contiguous() \
            and ppe.is_contiguous() and psrc.numel() == B * Lx * NP and ppe.dim() == 2 and ppe.shape[1] == NP \
            and ppe.shape[0] >= T_out and NP % 8 == 0 and 8 <= NP <= 1536, (tuple(psrc.shape), tuple(ppe.shape), B, Lx, T_out)
        pout = lay.empty(NP, torch.bfloat16)
    if dur is not None:
        dur = dur.contiguous()
        cum = torch.empty(B, Lx, device=dev, dtype=torch.int32)
        mel_len = torch.empty(B, device=dev, dtype=torch.int64)
        d_rounded = torch.empty(B, Lx, device=dev, dtype=torch.float32) if logpred else None
        L.check(_lib.fs2_lr_fused_proj(_ptr(x), _dt(x), _ptr(dur), _dur_kind(dur, logpred), float(d_control), None,
                                       None, B, Lx, D, int(T_out), _ptr(pe), _ptr(lens), _ptr(lay.cu),
                                       _ptr(lay.row_pos), _ptr(lay.rowmap), _ptr(out), od, _ptr(cum), _ptr(mel_len),
                                       _ptr(d_rounded), _ptr(psrc), _ptr(ppe), NP, _ptr(pout), _stream(x)),
                "fs2_lr_fused_proj")
        res = (out, lay, cum, mel_len, d_rounded)
    else:
        L.check(_lib.fs2_lr_fused_proj(_ptr(x), _dt(x), None, 0, 1.0, _ptr(cum), _ptr(mel_len), B, Lx, D, int(T_out),
                                       _ptr(pe), _ptr(lens), _ptr(lay.cu), _ptr(lay.row_pos), _ptr(lay.rowmap),
                                       _ptr(out), od, None, None, None, _ptr(psrc), _ptr(ppe), NP, _ptr(pout),
                                       _stream(x)), "fs2_lr_fused_proj")
        res = (out, lay)
    return res + (pout,) if proj is not None else res


def length_regulate(x, duration, max_len=None, return_index_map=False):
    """Drop-in for the reference ``LengthRegulator.forward(x, duration, max_len)``
    (model/modules.py:192-194): returns (output [B, T, D], mel_len int64 [B]).

    T = max_len when given (and non-zero, like utils/tools.py:361), else max(mel_len) — the
    one device->host read this path needs. With max_len the whole op is ONE fs2_length_regulate
    launch (scan + gather + zero padding)."""
    if max_len:
        _gpu(x, duration)
        x, duration = x.contiguous(), duration.contiguous()
        B, Lx, D = x.shape
        T_out = int(max_len)
        cum = torch.empty(B, Lx, device=x.device, dtype=torch.int32)
        mel_len = torch.empty(B, device=x.device, dtype=torch.int64)
        out = torch.empty(B, T_out, D, device=x.device, dtype=x.dtype)
        im = torch.empty(B, T_out, device=x.device, dtype=torch.int32) if return_index_map else None
        L.check(_lib.fs2_length_regulate(_ptr(x), _dt(x), _ptr(duration), _dur_kind(duration, False), 1.0, B, Lx, D,
                                         T_out, None, _ptr(out), _dt(x), _ptr(cum), _ptr(mel_len), None, _ptr(im),
                                         _stream(x)), "fs2_length_regulate")
        return (out, mel_len, im) if return_index_map else (out, mel_len)
    cum, mel_len, _ = lr_durations(duration)
    T_out = int(mel_len.max().item()) if mel_len.numel() else 0
    res = lr_expand(x, cum, mel_len, T_out, index_map=return_index_map)
    if return_index_map:
        return res[0], mel_len, res[1]
    return res, mel_len


# ---- training-step kernels (train.hip) ------------------------------------------------------------
def res_ln_fwd(a, res, gamma, beta, eps, lens=None, p_drop=0.0, seed=None, salt=0, want_bf16=True):
    """y = masked_fill(LayerNorm(dropout(a) + res), t >= lens[b], 0) (fs2_res_ln_fwd): a f32
    [B, T, 256], res f32 / bf16. Returns (y f32, y bf16 or None, xhat f32, rstd f32 [B*T])."""
    _gpu(a, res, gamma, beta, lens, seed)
    B, T, D = a.shape
    assert a.dtype == torch.float32 and a.is_contiguous() and res.shape == a.shape and res.is_contiguous()
    y = torch.empty_like(a)
    yb = torch.empty(a.shape, device=a.device, dtype=torch.bfloat16) if want_bf16 else None
    xhat = torch.empty_like(a)
    rstd = torch.empty(B * T, device=a.device, dtype=torch.float32)
    L.check(_lib.fs2_res_ln_fwd(_ptr(a), _ptr(res), _dt(res), _ptr(gamma), _ptr(beta), _ptr(lens), B * T, T, D,
                                float(eps), float(p_drop), _ptr(seed), int(salt), _ptr(y), _ptr(yb), _ptr(xhat),
                                _ptr(rstd), _stream(a)), "fs2_res_ln_fwd")
    return y, yb, xhat, rstd


def _defer_add(defer, ws, **kw):
    """Queue one split-partial reduction for :func:`reduce_flush` (ws stays referenced until then)."""
    d = L.ReduceDesc()
    d.part = ws.data_ptr()
    for k, v in kw.items():
        if k == "outs":
            for j, t in enumerate(list(v) + [None] * (3 - len(v))):
                setattr(d, f"out{j}", t.data_ptr() if t is not None else None)
        else:
            setattr(d, k, v)
    defer.append((d, ws))


def reduce_flush(defer, like):
    """Run the queued reductions (fs2_reduce_batch_launch, <= 32 per launch) on ``like``'s stream."""
    for i in range(0, len(defer), L.REDUCE_BATCH_MAX):
        chunk = defer[i:i + L.REDUCE_BATCH_MAX]
        b = L.ReduceBatch()
        b.n = len(chunk)
        for j, (d, _) in enumerate(chunk):
            b.d[j] = d
        L.check(_lib.fs2_reduce_batch_launch(ctypes.byref(b), _stream(like)), "fs2_reduce_batch_launch")
    defer.clear()


def res_ln_bwd(dy, xhat, rstd, gamma, lens=None, p_drop=0.0, seed=None, salt=0, dgamma=None, dbeta=None, dbias=None,
               want_dbias=True, accumulate=False, defer=None):
    """Backward of :func:`res_ln_fwd` (fs2_res_ln_bwd): returns (dres f32, da bf16, dgamma, dbeta,
    dbias) — dbias is the bias gradient of the conv that produced a (None unless wanted / given);
    accumulate adds into the given dgamma / dbeta / dbias."""
    _gpu(dy, xhat, rstd, gamma, lens, seed)
    B, T, D = xhat.shape
    dy = dy.contiguous()
    dres = torch.empty_like(xhat)
    da = torch.empty(xhat.shape, device=xhat.device, dtype=torch.bfloat16)
    new = lambda: torch.empty(D, device=xhat.device, dtype=torch.float32)
    dgamma = new() if dgamma is None else dgamma
    dbeta = new() if dbeta is None else dbeta
    if dbias is None and want_dbias:
        dbias = new()
    ws = torch.empty(_lib.fs2_res_ln_bwd_ws_bytes(D) // 4, device=xhat.device, dtype=torch.float32)
    L.check(_lib.fs2_res_ln_bwd(_ptr(dy), _ptr(xhat), _ptr(rstd), _ptr(gamma), _ptr(lens), B * T, T, D,
                                float(p_drop), _ptr(seed), int(salt), _ptr(dres), _ptr(da), _ptr(dgamma), _ptr(dbeta),
                                _ptr(dbias), 1 if accumulate else 0, 1 if defer is not None else 0, _ptr(ws),
                                ws.numel() * 4, _stream(xhat)), "fs2_res_ln_bwd")
    if defer is not None:
        _defer_add(defer, ws, M=3 * D, S=_lib.fs2_ln_bwd_parts(B * T), kind=0, split=D,
                   accumulate=1 if accumulate else 0, outs=(dgamma, dbeta, dbias))
    return dres, da, dgamma, dbeta, dbias


def relu_ln_fwd(a, gamma, beta, eps, p_drop=0.0, seed=None, salt=0, want_bf16=True):
    """y = dropout(LayerNorm(relu(a))) over rows of 256 (fs2_relu_ln_fwd): returns (y f32, y bf16
    or None, xhat f32, rstd f32)."""
    _gpu(a, gamma, beta, seed)
    assert a.dtype == torch.float32 and a.is_contiguous() and a.shape[-1] == 256
    R = a.numel() // 256
    y = torch.empty_like(a)
    yb = torch.empty(a.shape, device=a.device, dtype=torch.bfloat16) if want_bf16 else None
    xhat = torch.empty_like(a)
    rstd = torch.empty(R, device=a.device, dtype=torch.float32)
    L.check(_lib.fs2_relu_ln_fwd(_ptr(a), _ptr(gamma), _ptr(beta), R, 256, float(eps), float(p_drop), _ptr(seed),
                                 int(salt), _ptr(y), _ptr(yb), _ptr(xhat), _ptr(rstd), _stream(a)), "fs2_relu_ln_fwd")
    return y, yb, xhat, rstd


def relu_ln_bwd(dy, a, xhat, rstd, gamma, p_drop=0.0, seed=None, salt=0, dgamma=None, dbeta=None, dbias=None,
                want_dbias=True, accumulate=False, defer=None):
    """Backward of :func:`relu_ln_fwd` (fs2_relu_ln_bwd): (da bf16, dgamma, dbeta, dbias)."""
    _gpu(dy, a, xhat, rstd, gamma, seed)
    dy = dy.contiguous()
    R = a.numel() // 256
    da = torch.empty(a.shape, device=a.device, dtype=torch.bfloat16)
    new = lambda: torch.empty(256, device=a.device, dtype=torch.float32)
    dgamma = new() if dgamma is None else dgamma
    dbeta = new() if dbeta is None else dbeta
    if dbias is None and want_dbias:
        dbias = new()
    ws = torch.empty(_lib.fs2_res_ln_bwd_ws_bytes(256) // 4, device=a.device, dtype=torch.float32)
    L.check(_lib.fs2_relu_ln_bwd(_ptr(dy), _ptr(a), _ptr(xhat), _ptr(rstd), _ptr(gamma), R, 256, float(p_drop),
                                 _ptr(seed), int(salt), _ptr(da), _ptr(dgamma), _ptr(dbeta), _ptr(dbias),
                                 1 if accumulate else 0, 1 if defer is not None else 0, _ptr(ws), ws.numel() * 4,
                                 _stream(a)), "fs2_relu_ln_bwd")
    if defer is not None:
        _defer_add(defer, ws, M=3 * 256, S=_lib.fs2_ln_bwd_parts(R), kind=0, split=256,
                   accumulate=1 if accumulate else 0, outs=(dgamma, dbeta, dbias))
    return da, dgamma, dbeta, dbias


def relu_ln_head_fwd(a, gamma, beta, eps, hw, hb, mask, p_drop=0.0, seed=None, salt=0):
    """The VariancePredictor's second layer and its head in one launch (fs2_relu_ln_head_fwd):
    out = masked_fill(dropout(LayerNorm(relu(a))) . hw + hb, mask, 0) over rows of 256 (a f32
    [..., 256], hw f32 [256], hb f32 [1], mask bool [...]). Returns (out f32 [...], xhat, rstd)."""
    _gpu(a, gamma, beta, hw, hb, mask, seed)
    assert a.dtype == torch.float32 and a.is_contiguous() and a.shape[-1] == 256
    assert hw.numel() == 256 and hb.numel() == 1 and hw.is_contiguous()
    R = a.numel() // 256
    if mask is not None:
        assert mask.dtype == torch.bool and mask.numel() == R
        mask = mask.contiguous()
    out = torch.empty(a.shape[:-1], device=a.device, dtype=torch.float32)
    xhat = torch.empty_like(a)
    rstd = torch.empty(R, device=a.device, dtype=torch.float32)
    L.check(_lib.fs2_relu_ln_head_fwd(_ptr(a), _ptr(gamma), _ptr(beta), R, 256, float(eps), float(p_drop), _ptr(seed),
                                      int(salt), None, _ptr(xhat), _ptr(rstd), _ptr(hw), _ptr(hb), _ptr(mask),
                                      _ptr(out), _stream(a)), "fs2_relu_ln_head_fwd")
    return out, xhat, rstd


def relu_ln_head_bwd(dout, mask, hw, beta, a, xhat, rstd, gamma, p_drop=0.0, seed=None, salt=0, dgamma=None,
                     dbeta=None, dbias=None, dhw=None, dhb=None, accumulate=False, defer=None):
    """Backward of :func:`relu_ln_head_fwd` (fs2_relu_ln_head_bwd): from dout (the predictor output's
    gradient) -> (da bf16, dgamma, dbeta, dbias, dhw, dhb)."""
    _gpu(dout, mask, hw, beta, a, xhat, rstd, gamma, seed)
    dout = dout.contiguous()
    R = a.numel() // 256
    assert dout.dtype == torch.float32 and dout.numel() == R
    da = torch.empty(a.shape, device=a.device, dtype=torch.bfloat16)
    new = lambda n: torch.empty(n, device=a.device, dtype=torch.float32)
    dgamma = new(256) if dgamma is None else dgamma
    dbeta = new(256) if dbeta is None else dbeta
    dbias = new(256) if dbias is None else dbias
    dhw = new(256) if dhw is None else dhw
    dhb = new(1) if dhb is None else dhb
    ws = torch.empty(_lib.fs2_relu_ln_head_bwd_ws_bytes(256) // 4, device=a.device, dtype=torch.float32)
    L.check(_lib.fs2_relu_ln_head_bwd(_ptr(dout), _ptr(mask.contiguous() if mask is not None else None), _ptr(hw),
                                      _ptr(beta), _ptr(a), _ptr(xhat), _ptr(rstd), _ptr(gamma), R, 256, float(p_drop),
                                      _ptr(seed), int(salt), _ptr(da), _ptr(dgamma), _ptr(dbeta), _ptr(dbias),
                                      _ptr(dhw), _ptr(dhb), 1 if accumulate else 0, 1 if defer is not None else 0,
                                      _ptr(ws), ws.numel() * 4, _stream(a)), "fs2_relu_ln_head_bwd")
    if defer is not None:
        S = _lib.fs2_ln_bwd_parts(R)
        acc = 1 if accumulate else 0
        _defer_add(defer, ws, M=3 * 256, S=S, kind=0, split=256, accumulate=acc, outs=(dgamma, dbeta, dbias))
        head = ws[(_lib.fs2_res_ln_bwd_ws_bytes(256) // 4):]
        _defer_add(defer, head, M=256 + 4, S=S, kind=2, split=256, accumulate=acc, outs=(dhw, dhb))
    return da, dgamma, dbeta, dbias, dhw, dhb


def embedding_bwd(tokens, dy, V, padding_idx=None, out=None, accumulate=False):
    """nn.Embedding weight gradient (fs2_embedding_bwd): tokens int64 [...], dy f32 [..., D] ->
    out f32 [V, D], deterministic; padding_idx row zero (or untouched when accumulating)."""
    _gpu(tokens, dy, out)
    D = dy.shape[-1]
    tok = tokens.reshape(-1).to(torch.int64).contiguous()
    d2 = dy.reshape(-1, D)
    if d2.dtype != torch.float32 or d2.stride(-1) != 1:
        d2 = d2.float().contiguous()
    if out is None:
        out = torch.empty(V, D, device=dy.device, dtype=torch.float32)
    L.check(_lib.fs2_embedding_bwd(_ptr(tok), tok.numel(), _ptr(d2), d2.stride(0), int(V), D,
                                   -1 if padding_idx is None else int(padding_idx), _ptr(out), 1 if accumulate else 0,
                                   _stream(dy)), "fs2_embedding_bwd")
    return out


def loss_fwd(mel, post, p, e, logd, mel_tgt, p_tgt, e_tgt, d_tgt, mv, pm, em, dm):
    """FastSpeech2Loss forward (fs2_loss_fwd): returns (losses f32 [6] = total, mel, postnet, pitch,
    energy, duration; stats [4]; the argument struct; the tensors it points at)."""
    _gpu(mel, post, p, e, logd, mel_tgt, p_tgt, e_tgt, d_tgt, mv, pm, em, dm)
    f = lambda t: t.detach().float().contiguous()
    u8 = lambda t: t.contiguous().to(torch.bool)
    keep = [f(mel), f(post), f(p), f(e), f(logd), mel_tgt.detach().float(), f(p_tgt), f(e_tgt),
            d_tgt.detach().to(torch.int64).contiguous(), u8(mv), u8(pm), u8(em), u8(dm)]
    mel_, post_, p_, e_, ld_, mt, pt, et, dt, mv_, pm_, em_, dm_ = keep
    if mt.stride(-1) != 1:
        mt = keep[5] = mt.contiguous()
    B, T, C = mel_.shape
    assert post_.shape == mel_.shape and mt.shape[0] == B and mt.shape[1] >= T and mt.shape[2] == C
    assert mv_.shape == (B, T) and p_.shape == pt.shape == pm_.shape and e_.shape == et.shape == em_.shape
    assert ld_.shape == dt.shape == dm_.shape
    a = L.LossArgs()
    a.mel, a.postnet, a.mel_tgt = mel_.data_ptr(), post_.data_ptr(), mt.data_ptr()
    a.tgt_bs, a.tgt_ts, a.mel_valid = mt.stride(0), mt.stride(1), mv_.data_ptr()
    a.B, a.T, a.n_mel = B, T, C
    a.p_pred, a.p_tgt, a.p_mask, a.n_p = p_.data_ptr(), pt.data_ptr(), pm_.data_ptr(), p_.numel()
    a.e_pred, a.e_tgt, a.e_mask, a.n_e = e_.data_ptr(), et.data_ptr(), em_.data_ptr(), e_.numel()
    a.logd_pred, a.d_tgt, a.d_mask, a.n_d = ld_.data_ptr(), dt.data_ptr(), dm_.data_ptr(), ld_.numel()
    out = torch.empty(6, device=mel.device, dtype=torch.float32)
    stats = torch.empty(4, device=mel.device, dtype=torch.float32)
    ws = torch.empty(_lib.fs2_loss_ws_bytes() // 4, device=mel.device, dtype=torch.float32)
    L.check(_lib.fs2_loss_fwd(ctypes.byref(a), _ptr(out), _ptr(stats), _ptr(ws), ws.numel() * 4, _stream(mel)),
            "fs2_loss_fwd")
    return out, stats, a, keep


def loss_bwd(args, keep, grad_out, stats, shapes):
    """FastSpeech2Loss backward (fs2_loss_bwd): gradients of (mel, postnet, pitch, energy, log_d)."""
    mel = keep[0]
    g = grad_out.float().contiguous()
    outs = [torch.empty(s, device=mel.device, dtype=torch.float32) for s in shapes]
    L.check(_lib.fs2_loss_bwd(ctypes.byref(args), _ptr(g), _ptr(stats), *[_ptr(t) for t in outs], _stream(mel)),
            "fs2_loss_bwd")
    return outs


def bn_train_fwd(z, gamma, beta, eps, momentum, running_mean=None, running_var=None, use_tanh=True, p_drop=0.0,
                 seed=None, salt=0, residual=None, want_bf16=True, want_f32=False):
    """PostNet BatchNorm (batch statistics) + tanh + dropout (+ residual) over z f32 [..., C]
    (fs2_bn_train_fwd): returns (y bf16 or None, y f32 or None, mean, rstd); running stats updated
    in place."""
    _gpu(z, gamma, beta, running_mean, running_var, seed, residual)
    C = z.shape[-1]
    R = z.numel() // C
    assert z.dtype == torch.float32 and z.is_contiguous()
    yb = torch.empty(z.shape, device=z.device, dtype=torch.bfloat16) if want_bf16 else None
    yf = torch.empty_like(z) if want_f32 else None
    mean = torch.empty(C, device=z.device, dtype=torch.float32)
    rstd = torch.empty(C, device=z.device, dtype=torch.float32)
    ws = torch.empty(_lib.fs2_bn_train_ws_bytes(C) // 4, device=z.device, dtype=torch.float32)
    if residual is not None:
        residual = residual.contiguous()
    L.check(_lib.fs2_bn_train_fwd(_ptr(z), R, C, _ptr(gamma), _ptr(beta), float(eps), float(momentum),
                                  _ptr(running_mean), _ptr(running_var), 1 if use_tanh else 0, float(p_drop),
                                  _ptr(seed), int(salt), _ptr(residual), _ptr(yb), _ptr(yf), _ptr(mean), _ptr(rstd),
                                  _ptr(ws), ws.numel() * 4, _stream(z)), "fs2_bn_train_fwd")
    return yb, yf, mean, rstd


def bn_train_bwd(dy, z, gamma, beta, mean, rstd, use_tanh=True, p_drop=0.0, seed=None, salt=0, dgamma=None,
                 dbeta=None, accumulate=False):
    """Backward of :func:`bn_train_fwd` (fs2_bn_train_bwd): (dz bf16, dgamma, dbeta)."""
    _gpu(dy, z, gamma, beta, mean, rstd, seed)
    C = z.shape[-1]
    R = z.numel() // C
    dy = dy.contiguous()
    dz = torch.empty(z.shape, device=z.device, dtype=torch.bfloat16)
    dgamma = torch.empty(C, device=z.device, dtype=torch.float32) if dgamma is None else dgamma
    dbeta = torch.empty(C, device=z.device, dtype=torch.float32) if dbeta is None else dbeta
    ws = torch.empty(_lib.fs2_bn_train_ws_bytes(C) // 4, device=z.device, dtype=torch.float32)
    L.check(_lib.fs2_bn_train_bwd(_ptr(dy), _ptr(z), R, C, _ptr(gamma), _ptr(beta), _ptr(mean), _ptr(rstd),
                                  1 if use_tanh else 0, float(p_drop), _ptr(seed), int(salt), _ptr(dz), _ptr(dgamma),
                                  _ptr(dbeta), 1 if accumulate else 0, _ptr(ws), ws.numel() * 4, _stream(z)),
            "fs2_bn_train_bwd")
    return dz, dgamma, dbeta


def colsum(x, out=None, accumulate=False):
    """out[n] (+)= sum over rows of x [..., N] (f32 / bf16), deterministic (fs2_colsum)."""
    _gpu(x, out)
    N = x.shape[-1]
    x2 = x.reshape(-1, N)
    if out is None:
        out = torch.empty(N, device=x.device, dtype=torch.float32)
    ws = torch.empty(_lib.fs2_colsum_ws_bytes(N) // 4, device=x.device, dtype=torch.float32)
    L.check(_lib.fs2_colsum(_ptr(x2), _dt(x2), x2.shape[0], N, _rows(x2, "x"), _ptr(out), 1 if accumulate else 0,
                            _ptr(ws), ws.numel() * 4, _stream(x)), "fs2_colsum")
    return out


def conv_wgrad(dy, x, ks, pad, dw=None, db=None, want_db=False, accumulate=False, parts=None, defer=None):
    """Conv1d weight gradient (fs2_conv_wgrad): dy [B, T, N] f32 / bf16, x [B, T, C] bf16 ->
    dw f32 [N, C, ks] (and db f32 [N] when want_db / db given); accumulate adds into dw / db.
    parts = ([dw_0, dw_1(, dw_2)], [db_0, ...] or None): N split into equal row parts written to
    separate tensors (Q / K / V); dw / db are then ignored."""
    _gpu(dy, x, dw, db)
    B, T, N = dy.shape
    C = x.shape[-1]
    assert x.shape[:2] == (B, T) and x.dtype == torch.bfloat16
    split, extra = 0, [None] * 4
    if parts is not None:
        dws, dbs = parts
        split = N // len(dws)
        for t in dws:
            assert t.is_contiguous() and t.numel() == split * C * ks and t.dtype == torch.float32
        dw = dws[0]
        db = dbs[0] if dbs is not None else None
        extra = [dws[1], dws[2] if len(dws) > 2 else None,
                 dbs[1] if dbs is not None else None, dbs[2] if dbs is not None and len(dbs) > 2 else None]
    else:
        if dw is None:
            dw = torch.empty(N, C, ks, device=dy.device, dtype=torch.float32)
        if db is None and want_db:
            db = torch.empty(N, device=dy.device, dtype=torch.float32)
        assert dw.is_contiguous() and dw.numel() == N * C * ks and dw.dtype == torch.float32
    ws = torch.empty(max(1, _lib.fs2_conv_wgrad_ws_bytes(B, T, N, C, ks) // 4), device=dy.device, dtype=torch.float32)
    L.check(_lib.fs2_conv_wgrad(_ptr(dy), _dt(dy), _rows(dy, "dy"), _ptr(x), _rows(x, "x"), B, T, N, C, ks, pad,
                                _ptr(dw), _ptr(db), 1 if accumulate else 0, split, *[_ptr(t) for t in extra],
                                1 if defer is not None else 0, _ptr(ws), ws.numel() * 4, _stream(dy)), "fs2_conv_wgrad")
    if defer is not None:
        S = _lib.fs2_conv_wgrad_splits(B, T, N, C, ks)
        sp = split if split else N
        dws = (dw, extra[0], extra[1]) if split else (dw,)
        dbs = (db, extra[2], extra[3]) if split else (db,)
        acc = 1 if accumulate else 0
        _defer_add(defer, ws, M=ks * N * C, S=S, kind=1, KS=ks, N=N, C=C, split=sp, accumulate=acc, outs=dws)
        if db is not None:
            _defer_add(defer, ws[S * ks * N * C:], M=N, S=S, kind=0, split=sp, accumulate=acc, outs=dbs)
    return dw, db
