"""FastSpeech2.forward on the fs2hip kernels — the launch sequence of the hot path.

Mirrors model/fastspeech2.py:73-148 step by step (eval semantics, reference quirks kept):

  src_masks / mel_masks                       utils/tools.py:152-160 (returned tensors)
  embed + PE                    fs2_embed_pe   transformer/Models.py:82-91
  4 x FFT block (encoder)       5 launches     transformer/Layers.py:21-30
     Q|K|V GEMM (N=768)  -> attention -> fc + res + LN + mask -> conv k9 + ReLU -> conv k1 + res + LN + mask
     (the last block's epilogue also adds the speaker and emotion vectors, fastspeech2.py:101-110)
  VarianceAdaptor                              model/modules.py:102-158
     duration + pitch VPs (bf16x3 column-split launches; the head adds the pitch embedding),
     energy VP (uses p_control, :124-125) + its embedding
     -> LengthRegulator scan (+ duration rounding :132-135) -> gather (+ decoder PE add)
  6 x FFT block (decoder)                      transformer/Models.py:139-171
  mel_linear, PostNet (BN folded) + residual   fastspeech2.py:134-136, transformer/Layers.py:129-137

Every arithmetic step is a HIP kernel launched on torch.cuda.current_stream(); torch only
allocates buffers and builds the two boolean mask tensors the 10-tuple returns. With
``max_mel_len`` given (teacher-forced / training-style batches) the path has no host sync;
without it, ONE device->host read (max(mel_len) and the out-of-vocabulary id count together,
:func:`host_meta`) sizes the decoder (the reference does B*L_max .item() syncs in
LengthRegulator.expand). fs2amd.graphs.SynthGraphs captures the two halves around that read.
"""
import os
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib as L
from . import ops
from .model import sinusoid_table


def _mask(lengths, width):
    """get_mask_from_lengths (utils/tools.py:152-160): True = padding (one fs2_length_masks launch)."""
    if lengths.is_cuda:
        return ops.length_mask(lengths, width)
    ids = torch.arange(0, width, device=lengths.device).unsqueeze(0).expand(lengths.shape[0], -1)
    return ids >= lengths.unsqueeze(1).expand(-1, width)


def _pe(P, which, n):
    tab = P.enc_pe if which == "enc" else P.dec_pe
    if n <= tab.shape[0]:
        return tab
    # eval with a sequence longer than max_seq_len: the reference recomputes the table for the
    # whole length (Models.py:82-87,145-152); its first rows equal the stored ones.
    key = f"_pe_{which}_{n}"
    if not hasattr(P, key):
        setattr(P, key, sinusoid_table(n, tab.shape[1]).to(tab.device))
    return getattr(P, key)


def _qkv_pe(P, n):
    """pe W^T + b of the decoder's first Q|K|V over >= n positions (packing.qkv_pe_rows), grown with
    the PE table for sequences past max_seq_len."""
    q = P.dec_qkv_pe
    if n <= q.table.shape[0]:
        return q.table
    key = f"_qkv_pe_{n}"
    if not hasattr(P, key):
        from .packing import qkv_pe_rows
        setattr(P, key, qkv_pe_rows(_pe(P, "dec", n)[:n], q.attn, q.compute))
    return getattr(P, key)


def lr_proj_ok(P, x):
    """The decoder's first Q|K|V projection folded into the LengthRegulator launch (bf16 packed
    decoder): the projection runs on the B*L phoneme rows (one fs2_conv1d, f32 out) and
    fs2_lr_fused_proj adds the per-position table while it gathers, instead of a GEMM over the
    ~7x more frames. FS2_LR_PROJ=0: the frame-level Q|K|V launch (A/B)."""
    if os.environ.get("FS2_LR_PROJ", "1") == "0" or getattr(P, "dec_qkv_pe", None) is None or CALIB is not None:
        return False
    lp = P.dec_layers[0]
    return x.dtype == torch.bfloat16 and (lp.fp8 is None or lp.fp8.wqkv is None) and lp.n_head * lp.d_k == x.shape[-1]


# Optional measurement hook: when a list, the forward's launches are bracketed by HIP events on
# the launch stream, (start, end, tag) appended in launch order (bench.py's live roofline timing:
# the decoder's fused FFN, every FFT-block GEMM launch, attention, the LengthRegulator). Decoder
# FFN tags: "fc+ffn[+qkv]" / "ffn[+qkv]" / "ffn8" / "conv9"; the other launches "<stack>:<op>" with
# stack "enc" / "dec" / "va" and op "qkv", "attn", "fc", "ffn", "conv1", "lr", "mel", "postnet".
TIMERS = None
_STACK = ["enc"]


def _record_event():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


class _Timed:
    """Context manager recording HIP events around the launches inside it when TIMERS is a list."""

    __slots__ = ("tag", "e0")

    def __init__(self, tag):
        self.tag = tag

    def __enter__(self):
        if TIMERS is not None:
            self.e0 = _record_event()
        return self

    def __exit__(self, *exc):
        if TIMERS is not None and exc[0] is None:
            TIMERS.append((self.e0, _record_event(), self.tag))
        return False


def _tm(op):
    return _Timed(f"{_STACK[0]}:{op}")
# fp8 calibration hook (FastSpeech2.calibrate_fp8): when a dict, every FFT block records
# (max|h|, max|f|) of its FFN inputs over the valid rows, keyed by the layer's key.
CALIB = None


def _fp8_like(x, layout, width):
    if layout is not None:
        return layout.empty(width, torch.float8_e4m3fn)
    return torch.empty(*x.shape[:-1], width, device=x.device, dtype=torch.float8_e4m3fn)


def fft_block(P, lp, x, lens, addvec1=None, addvec2=None, timed=False, layout=None, x8=None, next_s=None,
              qkv=None, nxt=None):
    """One FFT block (transformer/Layers.py:21-30) = 4 launches. With ``layout`` (ops.SeqLayout)
    x is packed [B*T, d_model]: only valid frames exist and no mask is applied (nothing to mask).
    fp8 (cfg5): ``x8`` is the fp8 copy of x for the Q|K|V GEMM; ``next_s`` asks for an fp8 copy
    of the block output at that scale (the next block's Q|K|V input). ``qkv``: this block's Q|K|V
    projection, already computed by the previous block's fused FFN; ``nxt``: the next block's
    packed layer, whose Q|K|V projection the fused FFN then computes in its epilogue.
    Returns (out, out8|None, next block's qkv|None)."""
    c = P.compute
    dt = P.act_dtype
    H, dk = lp.n_head, lp.d_k
    d_model = H * dk
    if layout is not None:
        lens = None
    q = lp.fp8
    if CALIB is not None and lp.key is not None:
        rows = int(layout.cu[-1]) if layout is not None else None
        xv = x[:rows] if rows is not None else x
        CALIB.setdefault(lp.key, {})["x"] = float(xv.float().abs().max()) if xv.numel() else 0.0
    if qkv is None and layout is None and lens is not None and enc_block_ok(P, lp, x):
        # Q|K|V + attention + fc + residual + LN + row mask as one launch per utterance (L <= 64)
        with _tm("qkv+attn+fc"):
            h = ops.enc_attn_block(x, lens, lp.wqf, lp.bqkv, lp.wfcf, lp.bfc, lp.ln1, H, dk, float(np.power(dk, 0.5)))
        return _ffn_tail(P, lp, x, h, lens, addvec1, addvec2, timed, layout, q, next_s, nxt)
    if qkv is not None:
        pass
    elif q is not None and q.wqkv is not None and x8 is not None:
        with _tm("qkv"):
            qkv = ops.conv1d(x8, q.wqkv, lp.bqkv, cin=d_model, ks=1, pad=0, compute=L.FS2_FP8, epilogue=L.EPI_BIAS,
                             out_dtype=dt, col_scale=q.cs_qkv, layout=layout)
    else:
        with _tm("qkv"):
            qkv = ops.conv1d(x, lp.wqkv, lp.bqkv, cin=d_model, ks=1, pad=0, compute=c, epilogue=L.EPI_BIAS,
                             out_dtype=dt, layout=layout)
    with _tm("attn"):
        att = ops.attention(qkv, lens, H, dk, float(np.power(dk, 0.5)), layout=layout)
    # cfg5: the fc+LN epilogue also writes the fp8 copy of h the e4m3 k=9 conv reads (one launch)
    h8 = None
    if q is None and getattr(lp, "wfcf", None) is not None and CALIB is None and ffn_pre_on() and \
            ffn_fused_ok(P, lp, x, layout) and ops.ffn_pre_ok(x, layout, lp.b1.numel(), lp.k1):
        # fc + residual + LN (SubLayers.py:54-55) in the fused FFN's prologue: no h round trip,
        # one launch less per block (the decoder's packed 112-row launches; the encoder's padded
        # split-hidden launches, each split recomputing its tile's h)
        fuse_qkv = nxt is not None and getattr(nxt, "wqf", None) is not None and \
            (nxt.fp8 is None or nxt.fp8.wqkv is None) and qkv_fused_on() and qkv_epilogue_ok(x, layout, lp)
        tag = "fc+ffn+qkv" if fuse_qkv else "fc+ffn"
        with _Timed(tag if timed else f"{_STACK[0]}:{tag}"):
            r = ops.ffn(x, lp.w12, lp.b1, lp.b2, ks=lp.k1, pad=lp.p1, ln=lp.ln2, lens=lens, addvec1=addvec1,
                        addvec2=addvec2, layout=layout, next_qkv=(nxt.wqf, nxt.bqkv) if fuse_qkv else None,
                        pre=(att, lp.wfcf, lp.bfc, lp.ln1))
        y, qn = r if fuse_qkv else (r, None)
        return y, None, qn
    if q is not None:
        h8 = (layout.empty(d_model, torch.float8_e4m3fn) if layout is not None
              else torch.empty(*x.shape[:-1], d_model, device=x.device, dtype=torch.float8_e4m3fn))
    with _tm("fc"):
        h = ops.conv1d(att, lp.wfc, lp.bfc, cin=d_model, ks=1, pad=0, compute=c, epilogue=L.EPI_RES_LN,
                       out_dtype=dt, residual=x, ln=lp.ln1, lens=lens, layout=layout, out2=h8,
                       out2_scale=1.0 / q.s_h if q is not None else 1.0)
    return _ffn_tail(P, lp, x, h, lens, addvec1, addvec2, timed, layout, q, next_s, nxt, h8=h8)


def _ffn_tail(P, lp, x, h, lens, addvec1, addvec2, timed, layout, q, next_s, nxt, h8=None):
    """The FFT block after its attention sub-layer: the PositionwiseFeedForward on h (fused or two
    launches, fp8 forms) -> (out, out8|None, next block's qkv|None)."""
    c = P.compute
    dt = P.act_dtype
    d_model = lp.n_head * lp.d_k
    if q is not None and layout is not None and getattr(q, "w12_8", None) is not None and ffn8_on() \
            and CALIB is None and lp.k1 == 9 and lp.p1 == 4:
        # cfg5: the whole FFN as ONE e4m3 launch (fs2_ffn8: hidden quantised on chip, never in HBM)
        y8 = _fp8_like(x, layout, d_model) if next_s is not None else None
        with _Timed("ffn8" if timed else f"{_STACK[0]}:ffn8"):
            y = ops.ffn8(h8, h, q.w12_8, q.cs1, lp.b1, 1.0 / q.s_f, q.cs2, lp.b2, ln=lp.ln2, layout=layout, out8=y8,
                         out8_scale=1.0 / next_s if next_s is not None else 1.0)
        return y, y8, None
    if q is not None:
        # cfg5: the FFN pair on e4m3 MFMA; the k=9 epilogue writes relu(.) directly as fp8 for w_2
        with _Timed("conv9" if timed else f"{_STACK[0]}:conv9"):
            f8 = ops.conv1d(h8, q.w1, lp.b1, cin=lp.c1, ks=lp.k1, pad=lp.p1, compute=L.FS2_FP8,
                            epilogue=L.EPI_BIAS_RELU, out_dtype=L.FS2_FP8, out_scale=1.0 / q.s_f, col_scale=q.cs1,
                            layout=layout)
        y8 = _fp8_like(x, layout, d_model) if next_s is not None else None
        with _tm("conv1"):
            y = ops.conv1d(f8, q.w2, lp.b2, cin=lp.c2, ks=lp.k2, pad=lp.p2, compute=L.FS2_FP8,
                           epilogue=L.EPI_RES_LN, out_dtype=dt, residual=h, ln=lp.ln2, lens=lens, addvec1=addvec1,
                           addvec2=addvec2, layout=layout, col_scale=q.cs2, out2=y8,
                           out2_scale=1.0 / next_s if next_s is not None else 1.0)
        return y, y8, None
    if ffn_wide_ok(P, lp, h, layout) and CALIB is None:
        # small row counts (the encoder's 4k phoneme rows): conv-k9 on 256-row x 64-column tiles
        # with the x tile LDS-resident, then the k=1 conv + LN (fs2_ffn_wide: two launches)
        with _Timed("ffn" if timed else f"{_STACK[0]}:ffn"):
            y = ops.ffn_wide(h, lp.w12, lp.b1, lp.b2, ks=lp.k1, pad=lp.p1, ln=lp.ln2, lens=lens, addvec1=addvec1,
                             addvec2=addvec2, layout=layout)
        return y, None, None
    if ffn_fused_ok(P, lp, h, layout) and CALIB is None:
        # the whole FFN (conv-k9 + ReLU + conv-k1 + residual + LN + mask) as one launch: the
        # [rows, 1024] hidden stays on chip
        fuse_qkv = nxt is not None and getattr(nxt, "wqf", None) is not None and \
            (nxt.fp8 is None or nxt.fp8.wqkv is None) and qkv_fused_on() and qkv_epilogue_ok(h, layout, lp)
        tag = "ffn+qkv" if fuse_qkv else "ffn"
        with _Timed(tag if timed else f"{_STACK[0]}:{tag}"):
            r = ops.ffn(h, lp.w12, lp.b1, lp.b2, ks=lp.k1, pad=lp.p1, ln=lp.ln2, lens=lens, addvec1=addvec1,
                        addvec2=addvec2, layout=layout, next_qkv=(nxt.wqf, nxt.bqkv) if fuse_qkv else None)
        y, qn = r if fuse_qkv else (r, None)
        return y, None, qn
    with _Timed("conv9" if timed else f"{_STACK[0]}:conv9"):
        f = ops.conv1d(h, lp.w1, lp.b1, cin=lp.c1, ks=lp.k1, pad=lp.p1, compute=c, epilogue=L.EPI_BIAS_RELU,
                       out_dtype=dt, layout=layout)
    if CALIB is not None and lp.key is not None:
        rows = int(layout.cu[-1]) if layout is not None else None
        hv, fv = (h[:rows], f[:rows]) if rows is not None else (h, f)
        CALIB[lp.key]["h"] = float(hv.float().abs().max()) if hv.numel() else 0.0
        CALIB[lp.key]["f"] = float(fv.float().abs().max()) if fv.numel() else 0.0
    with _tm("conv1"):
        y = ops.conv1d(f, lp.w2, lp.b2, cin=lp.c2, ks=lp.k2, pad=lp.p2, compute=c, epilogue=L.EPI_RES_LN,
                       out_dtype=dt, residual=h, ln=lp.ln2, lens=lens, addvec1=addvec1, addvec2=addvec2,
                       layout=layout)
    return y, None, None


def ffn_wide_ok(P, lp, h, layout):
    """fs2_ffn_wide for the padded encoder stack's FFN (no fused Q|K|V epilogue or fc prologue is
    asked there: the next block's one-launch attention sub-layer projects its own Q|K|V) when
    the rows are few (ops.ffn_wide_ok: the cfg2 encoder's 4,096; cfg4's 41k keep the fused
    112-row launch). Packed decoder launches keep fs2_ffn (its fc prologue and Q|K|V epilogue)."""
    if layout is not None or P.compute != L.FS2_BF16 or h.dtype != torch.bfloat16 or getattr(lp, "w12", None) is None:
        return False
    return (h.dim() == 3 and h.shape[-1] == 256 and lp.k2 == 1 and lp.p1 == (lp.k1 - 1) // 2
            and ops.ffn_wide_ok(h.shape[0] * h.shape[1], lp.b1.numel(), lp.k1))


FFN_FUSED_MIN_ROWS = 16384
FFN_SPLIT_MIN_WG = 128


def decoder_forms(P, rows):
    """The decoder launch choices a host-known active row count makes (packed stage 2 with
    ``rows_hint`` = rows): whether the FFN is the fused launch and its (tile rows, split) form --
    the only arithmetic the row bucket changes (grids and early exits aside). Two row buckets with
    equal forms give bit-identical decoder outputs (graphs.SynthGraphs' speculation relies on it)."""
    F = P.dec_layers[0].b1.numel() if P.dec_layers else 0
    tr, ns = ops.ffn_form(rows, F) if F else (0, 0)
    fused = os.environ.get("FS2_FFN_FUSED", "1") == "2" or rows >= FFN_FUSED_MIN_ROWS or -(-rows // tr) * ns >= FFN_SPLIT_MIN_WG
    return (fused, tr, ns)


def ffn8_on():
    """FS2_FFN8=0: the cfg5 FFN as the two e4m3 fs2_conv1d launches (A/B)."""
    return os.environ.get("FS2_FFN8", "1") != "0"


def ffn_pre_on():
    """FS2_FFN_PRE=0: the attention output projection + LN as its own fs2_conv1d launch (A/B)."""
    return os.environ.get("FS2_FFN_PRE", "1") != "0"


def qkv_fused_on():
    """The next block's Q|K|V projection in the fused FFN's epilogue (fs2_ffn wqkv). FS2_QKV_FUSED=0:
    separate Q|K|V launches (A/B)."""
    return os.environ.get("FS2_QKV_FUSED", "1") != "0"


def enc_block_on():
    """FS2_ENC_BLOCK=0: the encoder's attention sub-layer as three launches (A/B)."""
    return os.environ.get("FS2_ENC_BLOCK", "1") != "0"


def enc_block_ok(P, lp, x):
    """fs2_enc_attn_block applies: bf16 padded [B, L <= 64, 256] rows, 2 x 128-dim heads, the
    fragment-ordered Q|K|V / fc weights, a bf16 layer (not cfg5's fp8 ones), no calibration pass."""
    return (enc_block_on() and P.compute == L.FS2_BF16 and x.dtype == torch.bfloat16 and x.dim() == 3
            and x.shape[1] <= 64 and x.shape[2] == 256 and lp.n_head == 2 and lp.d_k == 128 and CALIB is None
            and getattr(lp, "wqf", None) is not None and getattr(lp, "wfcf", None) is not None
            and lp.fp8 is None)  # fp8 layers: their FFN reads the fp8 copy of h the fc epilogue writes


def embed_block_ok(P, Lx):
    """The first encoder block's launch also builds the encoder input (embedding + PE) and writes
    the forward's masks (fs2_enc_embed_attn_block). FS2_ENC_EMBED=0: fs2_embed_pe and the two
    fs2_length_masks launches (A/B)."""
    if os.environ.get("FS2_ENC_EMBED", "1") == "0" or not P.enc_layers or P.act_dtype != L.FS2_BF16:
        return False
    lp = P.enc_layers[0]
    return (enc_block_on() and P.compute == L.FS2_BF16 and 0 < Lx <= 64 and P.enc_emb.shape[1] == 256
            and lp.n_head == 2 and lp.d_k == 128 and CALIB is None and getattr(lp, "wqf", None) is not None
            and getattr(lp, "wfcf", None) is not None and lp.fp8 is None)


def qkv_epilogue_ok(x, layout, lp):
    """The Q|K|V epilogue only for unsplit FFN launches (the decoder's). In the split-hidden form
    (the encoder's 64-row tiles x 4 splits) only the last-arriving split of a tile runs the
    epilogue, so the projection ran on a quarter of the CUs, streaming all 393 KB of Q|K|V weights
    per tile: 21.8k of the launch's 79.7k cycles (profiles/r5e/enc_ffn_trace.txt), where the
    weight-resident projection over all CUs takes ~8 us. FS2_QKV_FUSED=2 keeps it everywhere (A/B)."""
    if os.environ.get("FS2_QKV_FUSED", "1") == "2":
        return True
    return ops.ffn_form(ops.ffn_launch_rows(x, layout), lp.b1.numel())[1] == 1


def ffn_fused_ok(P, lp, h, layout):
    """fs2_ffn covers bf16 FFNs with d_model 256, kernel-1 w_2 and a hidden width of whole 256-column
    chunks. Launches with enough 112-row tiles to fill the chip (the cfg2 decoder: 24.9k packed
    rows) run one workgroup per 112-row tile; smaller ones 64-row tiles and / or the split-hidden
    form (ops.ffn_form: 2-4 workgroups per tile, f32 partials summed by the last arriver) when that
    puts >= 128 workgroups
    on the chip. Graph-timed at the encoder shape (4k rows, 64-row tiles x 4 splits): 38.8 us vs
    45.5 us for the two fs2_conv1d launches; a free-running cfg2 decoder (11.1k rows, 64-row tiles):
    71 vs 105 us.
    FS2_FFN_FUSED=0: off (A/B), =2: on at every size (tests); default 1."""
    mode = os.environ.get("FS2_FFN_FUSED", "1")
    if mode == "0" or P.compute != L.FS2_BF16 or h.dtype != torch.bfloat16 or getattr(lp, "w12", None) is None:
        return False
    # rows: the active packed rows when the host knows them (free-running: from the one host read),
    # else the capacity. A launch is one round of 112-row tiles taking about one tile's time, so
    # below ~146 tiles the two fs2_conv1d launches (many more, smaller tiles) are faster.
    rows = h.shape[0] * h.shape[1] if layout is None else (getattr(layout, "rows_hint", None) or layout.capacity)
    if mode == "2" or rows >= FFN_FUSED_MIN_ROWS:
        return True
    # fewer rows: the split-hidden form (ops.ffn_form) puts 2-4 workgroups on each tile
    tr, ns = ops.ffn_form(rows, lp.b1.numel())
    return -(-rows // tr) * ns >= FFN_SPLIT_MIN_WG


def _stack(P, layers, x, lens, layout=None, timed=False, addvecs=(None, None), qkv0=None, tail_next=None):
    """FFT-block stack; in fp8 mode each block hands the next one an fp8 copy of its output.
    qkv0: the first block's Q|K|V projection, already computed (fs2_lr_fused_proj). tail_next: the
    block after the last one: its Q|K|V comes from the last block's fused epilogue and (x, qkv) is
    returned (SynthGraphs' split stage 2)."""
    _STACK[0] = "dec" if timed else "enc"
    x8 = None
    qkv = qkv0
    n = len(layers)
    if tail_next is not None and tail_next.fp8 is not None:
        raise NotImplementedError("_stack: tail_next with fp8 layers")
    for i, lp in enumerate(layers):
        nxt = layers[i + 1] if i + 1 < n else tail_next
        next_s = nxt.fp8.s_x if (nxt is not None and nxt.fp8 is not None and nxt.fp8.wqkv is not None) else None
        last = i == n - 1
        x, x8, qkv = fft_block(P, lp, x, lens, addvecs[0] if last else None, addvecs[1] if last else None,
                               timed=timed, layout=layout, x8=x8, next_s=next_s, qkv=qkv, nxt=nxt)
    return (x, qkv) if tail_next is not None else x


def packed_decoder_ok(P):
    """The packed decoder equals the reference's padded one when every padded frame an FFT block
    reads through a conv tap is zero there: h (input of w_1) is masked after the attention
    LayerNorm, and f = relu(w_1 h + b) (input of w_2) is not, so w_2 must be kernel-1
    (model.yaml conv_kernel_size [9, 1]). Attention only sees keys < len either way.
    FS2_PACKED_DECODER=0 forces the padded path."""
    import os
    if os.environ.get("FS2_PACKED_DECODER", "1") == "0":
        return False
    return all(lp.k2 == 1 and lp.p2 == 0 for lp in P.dec_layers)


def variance_predictor(vp, x, lens):
    """VariancePredictor (model/modules.py:209-250): 2 launches -> f32 [B, T] (f32, bf16 or bf16x3 MFMA)."""
    if vp.split:
        # bf16x3: logical inputs [x_hi | x_hi] (x is bf16: x_lo = 0) and [h_hi | h_hi | h_lo] read
        # through the channel-block map; conv1's LN epilogue writes h as two bf16 planes
        h2 = ops.conv1d(x, vp.w1, vp.b1, cin=2 * vp.c1, ks=vp.k1, pad=vp.p1, compute=L.FS2_BF16,
                        epilogue=L.EPI_RELU_LN, out_dtype=L.FS2_BF16, ln=vp.ln1, cin_block=vp.c1, cin_src=(0, 0),
                        out_split=True)
        return ops.conv1d(h2, vp.w2, vp.b2, cin=3 * vp.c2, ks=vp.k2, pad=vp.p2, compute=L.FS2_BF16,
                          epilogue=L.EPI_RELU_LN_DOT, ln=vp.ln2, lens=lens, dot=(vp.lin_w, vp.lin_b),
                          cin_block=vp.c2, cin_src=(0, 0, vp.c2))
    h = ops.conv1d(x, vp.w1, vp.b1, cin=vp.c1, ks=vp.k1, pad=vp.p1, compute=vp.compute, epilogue=L.EPI_RELU_LN,
                   out_dtype=vp.compute, ln=vp.ln1)
    return ops.conv1d(h, vp.w2, vp.b2, cin=vp.c2, ks=vp.k2, pad=vp.p2, compute=vp.compute,
                      epilogue=L.EPI_RELU_LN_DOT, ln=vp.ln2, lens=lens, dot=(vp.lin_w, vp.lin_b))


def vp_fused_on():
    """FS2_VP_FUSED=0: the column-split launches (round-2 form) instead of fs2_vp_fused (A/B)."""
    return os.environ.get("FS2_VP_FUSED", "1") != "0"


def vp_columns_on():
    """FS2_VP_COLUMNS=0: the bf16x3 predictors as LayerNorm-epilogue GEMMs (round-1 form, A/B)."""
    return os.environ.get("FS2_VP_COLUMNS", "1") != "0"


def variance_predictors(F, x, lens, embed=None):
    """G VariancePredictors on the same input x (model/modules.py:209-250), column-split bf16x3:
    conv1 (+ ReLU) as one launch over the G predictors' stacked columns, fs2_vp_norm (LayerNorm ->
    bf16 hi / lo planes), conv2 (+ ReLU) as one grouped launch (group g reads its own planes),
    fs2_vp_head (LayerNorm, Linear(256 -> 1), mask; optionally the pitch / energy embedding add of
    one group into x). Returns pred f32 [G, B, T]."""
    y1 = ops.conv1d(x, F.w1, F.b1, cin=2 * F.c, ks=F.k, pad=F.p, compute=L.FS2_BF16, epilogue=L.EPI_BIAS_RELU,
                    out_dtype=L.FS2_F32, cin_block=F.c, cin_src=(0, 0))
    h = ops.vp_norm(y1, F.g1, F.be1, F.eps)
    y2 = ops.conv1d(h, F.w2, F.b2, cin=3 * F.c, ks=F.k, pad=F.p, compute=L.FS2_BF16, epilogue=L.EPI_BIAS_RELU,
                    out_dtype=L.FS2_F32, cin_block=F.c, cin_src=(0, 0, F.c),
                    group=(F.c, 2 * F.c) if F.G > 1 else None)
    return ops.vp_head(y2, F.g2, F.be2, F.eps, F.lin_w, F.lin_b, lens, embed)


def _variance(P, kind, x, lens, target, control):
    pred = variance_predictor(P.vp[kind], x, lens)
    tgt = None
    if target is not None:
        tgt = target.to(device=x.device, dtype=torch.float32).contiguous()
    ops.variance_embed(x, pred, tgt, control, P.bins[kind], P.var_table[kind])
    return pred


def _device_ok(dev):
    return dev.type == "cuda"


def _streams_for(B):
    """Utterance groups run as parallel HIP streams (parallel branches of a captured graph): one
    group's partial last wave of workgroups and its launch ramps overlap the other group's work.
    FS2_STREAMS groups (default 1: measured no gain under graph replay in round 1), each at least 8
    utterances."""
    import os
    n = int(os.environ.get("FS2_STREAMS", "1"))
    return max(1, min(n, B // 8))


class _StreamSlot:
    """Group i: its side stream and its own split-K workspace (ops.splitk_slot)."""

    def __init__(self, stream, i):
        self.s, self.k = torch.cuda.stream(stream), ops.splitk_slot(i)

    def __enter__(self):
        self.s.__enter__()
        self.k.__enter__()

    def __exit__(self, *exc):
        self.k.__exit__(*exc)
        return self.s.__exit__(*exc)


class _ForkJoin:
    """n utterance groups on n side streams forked from / joined to the caller's stream (graph
    capture turns them into parallel branches). n == 1 runs inline and touches no stream API."""

    _cache = {}

    def __init__(self, dev, n):
        import contextlib

        self.n = n
        if n == 1:
            self.ctx = lambda i: contextlib.nullcontext()
            return
        key = (str(dev), n)
        if key not in self._cache:
            self._cache[key] = [torch.cuda.Stream(device=dev) for _ in range(n)]
        self.streams = self._cache[key]
        self.main = torch.cuda.current_stream(dev)
        self.ctx = lambda i: _StreamSlot(self.streams[i], i)

    def fork(self):
        if self.n > 1:
            for s in self.streams:
                s.wait_stream(self.main)

    def join(self, *tensors):
        """Main stream waits for every group; tensors made on side streams are marked as used by it."""
        if self.n > 1:
            for s in self.streams:
                self.main.wait_stream(s)
            for t in tensors:
                if t is not None:
                    t.record_stream(self.main)


def _stage1(P, va, g, p_control, d_control, defer_lr=False):
    """Encoder (+ conditioning), variance predictors, duration scan for one utterance group.
    defer_lr (teacher-forced durations, decoder length known): the duration scan is left to the
    one-launch LengthRegulator of stage 2 (fs2_lr_fused)."""
    fold = getattr(g, "mask_out", None) is not None
    if not fold:
        x = ops.embed_pe(g.texts, P.enc_emb, _pe(P, "enc", g.Lx), P.act_dtype)
    spk_vec = emo_vec = None
    has_cond = P.spk_table is not None or P.emo_table is not None
    # FS2_ENC_COND=1: the conditioning tiles on extra workgroups of the first block's launch (A/B:
    # 32.4 us for that launch against 16.8 + 9.2 for the block and fs2_cond_vectors, profiles/r5ck)
    cond_fold = fold and os.environ.get("FS2_ENC_COND", "0") == "1"
    if has_cond and not cond_fold:
        spk_vec, emo_vec = ops.cond_vectors(
            g.speakers if P.spk_table is not None else None, P.spk_table,
            g.emotions if P.emo_table is not None else None, g.arousals, g.valences, P.emo_table,
            getattr(P, "aro_table", None), getattr(P, "val_table", None), getattr(P, "emo_w", None),
            getattr(P, "emo_b", None), P.d_model)
    n_enc = len(P.enc_layers)
    if fold:
        # block 0's attention sub-layer with the embedding + PE and the masks in the same launch
        _STACK[0] = "enc"
        lp = P.enc_layers[0]
        cond = None
        if has_cond and cond_fold:  # the conditioning vectors on extra workgroups of the same launch
            cond = (g.speakers if P.spk_table is not None else None, P.spk_table,
                    g.emotions if P.emo_table is not None else None, g.arousals, g.valences, P.emo_table,
                    getattr(P, "aro_table", None), getattr(P, "val_table", None), getattr(P, "emo_w", None),
                    getattr(P, "emo_b", None))
        with _tm("qkv+attn+fc"):
            r = ops.enc_attn_block(None, g.lens_src, lp.wqf, lp.bqkv, lp.wfcf, lp.bfc, lp.ln1, lp.n_head, lp.d_k,
                                   float(np.power(lp.d_k, 0.5)), embed=(g.texts, P.enc_emb, _pe(P, "enc", g.Lx)),
                                   masks=g.mask_out, cond=cond)
        if cond is not None:
            h, spk_vec, emo_vec = r
        else:
            h = r
        last = n_enc == 1
        # a Q|K|V the FFN epilogue computes for block 1 is handed on (as the non-fold _stack does);
        # when block 1 runs the one-launch attention sub-layer, which projects its own, none is asked for
        nxt = P.enc_layers[1] if n_enc > 1 else None
        if nxt is not None and enc_block_ok(P, nxt, h):
            nxt = None
        x, _, qn = _ffn_tail(P, lp, h, h, g.lens_src, spk_vec if last else None, emo_vec if last else None, False,
                             None, None, None, nxt)
        if n_enc > 1:
            x = _stack(P, P.enc_layers[1:], x, g.lens_src, addvecs=(spk_vec, emo_vec), qkv0=qn)
    else:
        x = _stack(P, P.enc_layers, x, g.lens_src, addvecs=(spk_vec, emo_vec))
    if n_enc == 0 and (spk_vec is not None or emo_vec is not None):
        raise NotImplementedError("encoder_layer = 0")

    st = SimpleNamespace(x=x, p_pred=None, e_pred=None)
    st.phoneme_p = va.pitch_feature_level == "phoneme_level"
    st.phoneme_e = va.energy_feature_level == "phoneme_level"
    if getattr(P, "vpfused", None) is not None and st.phoneme_p and st.phoneme_e and x.dtype == torch.bfloat16 \
            and vp_fused_on():
        # duration + pitch as ONE launch (each a whole predictor per 32-row tile; the pitch group
        # writes x + pitch embedding to a new buffer), then energy on it (modules.py:110-126)
        V = P.vpfused
        with _Timed("va:vp"):
            dp, x = ops.vp_fused(x, V.dp, g.lens_src, embed=(1, g.p_targets, p_control, P.bins["pitch"],
                                                               P.var_table["pitch"]))
            st.log_d, st.p_pred = dp[0], dp[1]
            en, x = ops.vp_fused(x, V.energy, g.lens_src, embed=(0, g.e_targets, p_control, P.bins["energy"],
                                                                 P.var_table["energy"]))  # p_control: :124-125
        st.e_pred = en[0]
        st.x = x
    elif P.vpcols is not None and st.phoneme_p and st.phoneme_e and vp_columns_on():
        # duration + pitch in one set of launches (both read x; the pitch embedding is added to x
        # by the head), then energy on x + pitch embedding (modules.py:110-126)
        V = P.vpcols
        dp = variance_predictors(V.dp, x, g.lens_src,
                                 embed=(1, x, g.p_targets, p_control, P.bins["pitch"], P.var_table["pitch"]))
        st.log_d, st.p_pred = dp[0], dp[1]
        st.e_pred = variance_predictors(V.energy, x, g.lens_src, embed=(
            0, x, g.e_targets, p_control, P.bins["energy"], P.var_table["energy"]))[0]  # p_control: :124-125
    else:
        st.log_d = variance_predictor(P.vp["duration"], x, g.lens_src)
    if st.phoneme_p and st.p_pred is None:
        st.p_pred = _variance(P, "pitch", x, g.lens_src, g.p_targets, p_control)
    if st.phoneme_e and st.e_pred is None:
        st.e_pred = _variance(P, "energy", x, g.lens_src, g.e_targets, p_control)  # p_control: modules.py:124-125
    if g.d_targets is not None:
        st.d_rounded = None
        if defer_lr:
            st.cum = st.mel_len = None
            st.dur_pending = _dur_input(g.d_targets)
        else:
            st.cum, st.mel_len, _ = ops.lr_durations(_dur_input(g.d_targets))
    else:
        st.cum, st.mel_len, st.d_rounded = ops.lr_durations(st.log_d, logpred=True, d_control=d_control)
    return st


def _dur_input(d):
    return d if d.dtype in (torch.int64, torch.float32) else d.to(torch.int64)


def _ensure_lr(st):
    """The duration scan of a deferred stage 1, where stage 2 does not take fs2_lr_fused."""
    if st.cum is None:
        st.cum, st.mel_len, _ = ops.lr_durations(st.dur_pending)


def lr_fused_on():
    """FS2_LR_FUSED=0: the LengthRegulator as lr_durations + seq_layout + lr_expand (A/B)."""
    return os.environ.get("FS2_LR_FUSED", "1") != "0"


def lr_fused_ok(x):
    return lr_fused_on() and x.shape[1] <= 2048 and x.shape[0] <= 4096


def _stage2(P, g, st, T_out, T_dec, p_control, postnet_valid=False, rows_hint=None):
    """LengthRegulator gather, decoder, mel_linear, PostNet for one utterance group."""
    dec_lens = st.mel_len if g.d_targets is None else g.mel_lens
    frame_level = not (st.phoneme_p and st.phoneme_e)
    x = st.x
    if not frame_level and T_dec == T_out and packed_decoder_ok(P):
        # packed decoder: only the dec_lens frames of each utterance are computed
        # (cfg2: 24.9k of 27.5k rows, cfg4: 135k of 249k); mel_linear scatters back to [B, T, n_mel]
        x, lay = decode_packed(P, st, x, dec_lens, T_out, rows_hint)
        mel, pn = mel_postnet(P, x, lay, dec_lens, postnet_valid, rows_hint)
        return mel, pn, st
    # LR gather with the decoder's position encoding fused (frame-level variance needs the bare
    # expanded x first, so the PE add moves to a second pass in that configuration)
    _ensure_lr(st)
    if frame_level:
        x = ops.lr_expand(x, st.cum, st.mel_len, T_out, pe=None, out_dtype=P.act_dtype)
        if not st.phoneme_p:
            st.p_pred = _variance(P, "pitch", x, dec_lens, g.p_targets, p_control)
        if not st.phoneme_e:
            st.e_pred = _variance(P, "energy", x, dec_lens, g.e_targets, p_control)
        x = x[:, :T_dec].contiguous()
        x = _add_pe(x, _pe(P, "dec", T_dec))
    else:
        x = ops.lr_expand(x, st.cum, st.mel_len, T_out, pe=_pe(P, "dec", T_out), out_dtype=P.act_dtype)
        if T_dec != T_out:
            x = x[:, :T_dec].contiguous()
    if T_dec != T_out:
        dec_lens = torch.clamp(dec_lens, max=T_dec)
    x = _stack(P, P.dec_layers, x, dec_lens, timed=True)
    mel_bf = _mel_copy(P, x, x.shape[:2])
    mel = ops.conv1d(x, P.mel_w, P.mel_b, cin=P.d_model, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_BIAS,
                     out_dtype=L.FS2_F32, out2=mel_bf)
    return mel, _postnet(P, mel, mel_bf, dec_lens if postnet_valid else None, rows_hint), st


def decode_packed(P, st, x, dec_lens, T_lay, rows_hint=None):
    """LengthRegulator gather (+ PE) into the packed layout of dec_lens over T_lay frames and the
    decoder stack on those rows. The result does not depend on T_lay beyond T_lay >= max(dec_lens)
    (the packed rows, cu and row_pos are those of the valid frames; only the padded-row maps and
    the grids' early-exiting tails grow with it): fs2amd.graphs.SynthGraphs captures this part per
    T bucket. Returns (packed x [B*T_lay, d_model], layout)."""
    x, lay, qkv0 = _lr_packed(P, st, x, dec_lens, T_lay, rows_hint)
    return _stack(P, P.dec_layers, x, None, layout=lay, timed=True, qkv0=qkv0), lay


def decode_packed_head(P, st, x, dec_lens, T_lay, rows_hint=None):
    """decode_packed's LengthRegulator launch and first decoder block, whose fused epilogue also
    projects the second block's Q|K|V: returns (x1, layout, qkv1). With :func:`decode_packed_rest`
    the same launches in the same order (SynthGraphs captures the two as separate graphs: the
    small first one starts the GPU sooner after the host read)."""
    x, lay, qkv0 = _lr_packed(P, st, x, dec_lens, T_lay, rows_hint)
    x1, qkv1 = _stack(P, P.dec_layers[:1], x, None, layout=lay, timed=True, qkv0=qkv0, tail_next=P.dec_layers[1])
    return x1, lay, qkv1


def decode_packed_rest(P, x1, lay, qkv1):
    return _stack(P, P.dec_layers[1:], x1, None, layout=lay, timed=True, qkv0=qkv1)


def _lr_packed(P, st, x, dec_lens, T_lay, rows_hint=None):
    """The LengthRegulator part of decode_packed: (packed x, layout, first block's Q|K|V or None)."""
    qkv0 = None
    if lr_fused_ok(x):
        proj = None
        if lr_proj_ok(P, x):
            xw = getattr(st, "xw", None)  # SynthGraphs: already run at the end of stage 1
            if xw is None:
                xw = phoneme_qkv0(P, x)
            proj = (xw.view(-1, xw.shape[-1]), _qkv_pe(P, T_lay))
        # scan (teacher-forced) + packed layout + gather (+ PE) (+ the first Q|K|V) in one launch
        with _Timed("va:lr"):
            if st.cum is None:
                r = ops.lr_fused(x, dec_lens, T_lay, pe=_pe(P, "dec", T_lay), out_dtype=P.act_dtype,
                                 dur=st.dur_pending, proj=proj)
                x, lay, st.cum, st.mel_len = r[:4]
            else:
                r = ops.lr_fused(x, dec_lens, T_lay, pe=_pe(P, "dec", T_lay), out_dtype=P.act_dtype,
                                 cum=st.cum, mel_len=st.mel_len, proj=proj)
                x, lay = r[:2]
            qkv0 = r[-1] if proj is not None else None
    else:
        _ensure_lr(st)
        lay = ops.SeqLayout(dec_lens, T_lay)
        x = ops.lr_expand(x, st.cum, st.mel_len, T_lay, pe=_pe(P, "dec", T_lay), out_dtype=P.act_dtype,
                          out_layout=lay)
    # active rows when known on the host (free-running), rounded up (ops.rows_bucket) so that
    # a captured stage-2 graph serves every batch of the bucket
    lay.rows_hint = None if rows_hint is None else ops.rows_bucket(rows_hint, lay.capacity)
    return x, lay, qkv0


def phoneme_qkv0(P, x):
    """x W^T of the decoder's first Q|K|V on the phoneme rows (Models.py:145-152 input; the LR
    launch adds the per-position pe W^T + b by linearity), f32."""
    lp = P.dec_layers[0]
    with _Timed("dec:qkv0"):
        return ops.conv1d(x, lp.wqkv, None, cin=x.shape[-1], ks=1, pad=0, compute=P.compute, epilogue=L.EPI_BIAS,
                          out_dtype=L.FS2_F32)


def split_stage2_ok(P):
    """SynthGraphs' stage 2 as two graphs (the first block, then the rest), opt-in
    (FS2_SYNTH_SPLIT=1): measured 1.351 ms per free-running call against 1.299 ms as one graph
    (profiles/r5s1) -- the gap after the host read is not the graph's size, and the second
    launch adds its own."""
    return (os.environ.get("FS2_SYNTH_SPLIT", "0") == "1" and len(P.dec_layers) >= 2
            and all(lp.fp8 is None for lp in P.dec_layers))


def mel_postnet(P, x, lay, dec_lens, postnet_valid=False, rows_hint=None):
    """mel_linear from the packed decoder rows into the padded [B, lay.T, n_mel] contract (padded
    frames get the bias, as the reference's masked decoder output gives) and the PostNet +
    residual with the reference's padded semantics over lay.T frames."""
    mel_bf = _mel_copy(P, x, (lay.B, lay.T))
    with _Timed("dec:mel"):
        mel = ops.conv1d(x, P.mel_w, P.mel_b, cin=P.d_model, ks=1, pad=0, compute=P.compute, epilogue=L.EPI_BIAS,
                         out_dtype=L.FS2_F32, src_layout=lay, out2=mel_bf)
    with _Timed("dec:postnet"):
        pn = _postnet(P, mel, mel_bf, dec_lens if postnet_valid else None, rows_hint)
    return mel, pn


def packed_stage2_ok(P, st, x):
    """The packed decoder path of _stage2 applies (phoneme-level variance, kernel-1 w_2, lr_fused)."""
    return st.phoneme_p and st.phoneme_e and packed_decoder_ok(P) and lr_fused_ok(x)


def run_forward(model, speakers, emotions, arousals, valences, texts, src_lens, max_src_len, mels, mel_lens,
                max_mel_len, p_targets, e_targets, d_targets, p_control, e_control, d_control):
    dev = texts.device
    if not _device_ok(dev):
        raise RuntimeError("fs2amd: FastSpeech2.forward runs on the HIP kernels only; move the model and the batch "
                           "to a ROCm device (no CPU fallback)")
    P = model.packed(dev)
    va = model.variance_adaptor
    ids = lambda t: None if t is None else torch.as_tensor(t).to(device=dev, dtype=torch.int64).contiguous()
    f32 = lambda t: None if t is None else t.to(device=dev, dtype=torch.float32).contiguous()
    B = texts.shape[0]
    Lx = int(max_src_len)
    if texts.shape[1] != Lx:
        raise RuntimeError(f"texts has {texts.shape[1]} positions but max_src_len is {Lx}")
    src_lens = src_lens.to(dev)
    n = _streams_for(B)
    mel_w = None if mel_lens is None else (max_mel_len if max_mel_len is not None else int(mel_lens.max().item()))
    mask_out = None
    if n == 1 and embed_block_ok(P, Lx):
        # the first encoder block's launch builds its input and writes both masks (fs2_enc_embed_attn_block)
        src_masks = torch.empty(B, Lx, device=dev, dtype=torch.bool)
        mel_masks = None if mel_lens is None else torch.empty(B, int(mel_w), device=dev, dtype=torch.bool)
        mask_out = (src_masks, None if mel_lens is None else mel_lens.to(dev).to(torch.int64).contiguous(), mel_masks)
    else:
        src_masks = _mask(src_lens, Lx)
        mel_masks = _mask(mel_lens, mel_w) if mel_lens is not None else None
    full = SimpleNamespace(
        speakers=ids(speakers), emotions=ids(emotions), arousals=ids(arousals), valences=ids(valences),
        texts=ids(texts), lens_src=src_lens.to(torch.int64).contiguous(), Lx=Lx,
        p_targets=f32(p_targets), e_targets=f32(e_targets),
        d_targets=None if d_targets is None else d_targets.to(dev),
        mel_lens=None if mel_lens is None else mel_lens.to(dev).to(torch.int64).contiguous(), mask_out=mask_out)

    # utterance groups (contiguous ranges of b; same padded L / T as the whole batch, so every
    # group's outputs are bit-identical to the one-group run)
    bounds = [(B * i // n, B * (i + 1) // n) for i in range(n)]

    def part(b0, b1):
        sl = lambda t: None if t is None else t[b0:b1]
        return SimpleNamespace(**{k: (sl(v) if torch.is_tensor(v) else v) for k, v in vars(full).items()})

    groups = [part(b0, b1) for b0, b1 in bounds] if n > 1 else [full]
    fj = _ForkJoin(dev, n)
    fj.fork()
    sts = []
    # teacher-forced with the decoder length given: the duration scan joins the LengthRegulator's
    # one launch in stage 2
    defer = d_targets is not None and bool(max_mel_len)
    for i, g in enumerate(groups):
        with fj.ctx(i):
            sts.append(_stage1(P, va, g, p_control, d_control, defer_lr=defer))

    mel_len = sts[0].mel_len if n == 1 else None
    if not max_mel_len or d_targets is None:
        # free-running: the decoder length is max(mel_len) over ALL groups (one host read)
        if n > 1:
            fj.join(*[st.mel_len for st in sts])
            mel_len = torch.cat([st.mel_len for st in sts])
            fj.fork()
    if d_targets is None or not max_mel_len:
        # the ONE host read of the free-running path: max(mel_len) and the out-of-vocabulary id
        # count in one device->host copy
        max_len, sum_len = host_meta(mel_len, dev)
        T_out = int(max_mel_len) if max_mel_len else max_len
    else:
        T_out = int(max_mel_len)
    if d_targets is None:
        mel_masks = _mask(mel_len, max_len)  # get_mask_from_lengths(mel_len): width max(mel_len)
    if mel_masks is None or mel_masks.shape[1] != T_out:
        raise RuntimeError(f"decoder mask width {None if mel_masks is None else mel_masks.shape[1]} != length-"
                           f"regulated length {T_out} (the reference fails here too: Models.py:157)")
    # free-running batches padded to one long utterance: the PostNet's valid-region form
    pn_valid = d_targets is None and T_out == max_len and postnet_valid_rows(B, T_out, sum_len)
    if pn_valid:
        # the valid-region PostNet's constant row / tail block (cached per weight pack) made on the
        # caller's stream before the groups' streams are released again: no group reads them
        # before they are written
        _postnet_consts(P, _mel_copy_on(P))
        fj.fork()
    T_dec = min(T_out, P.max_seq_len) if model.training else T_out
    if T_dec != T_out:
        mel_masks = mel_masks[:, :T_dec]

    res = []
    for i, (g, st) in enumerate(zip(groups, sts)):
        with fj.ctx(i):
            res.append(_stage2(P, g, st, T_out, T_dec, p_control, pn_valid,
                               sum_len if (d_targets is None and n == 1) else None))
    if n == 1:
        mel, postnet_mel, st = res[0]
        out = (mel, postnet_mel, st.p_pred, st.e_pred, st.log_d, st.d_rounded, st.mel_len)
    else:
        fj.join(*[t for r in res for t in (r[0], r[1], r[2].p_pred, r[2].e_pred, r[2].log_d, r[2].d_rounded,
                                           r[2].mel_len)])
        cat = lambda ts: None if ts[0] is None else torch.cat(ts)
        out = (cat([r[0] for r in res]), cat([r[1] for r in res]), cat([r[2].p_pred for r in res]),
               cat([r[2].e_pred for r in res]), cat([r[2].log_d for r in res]),
               cat([r[2].d_rounded for r in res]), cat([r[2].mel_len for r in res]))
    mel, postnet_mel, p_pred, e_pred, log_d, d_rounded, mel_len = out
    if d_targets is not None:
        d_rounded = d_targets
    return (mel, postnet_mel, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_len)


HOST_READS = [0]  # device->host reads made by the forward path (tests assert one per free-running call)


def meta_vector(mel_len, dev):
    """[max(mel_len), sum(mel_len), out-of-vocabulary count] as int32 on the device (one copy)."""
    return ops.len_stats(mel_len, ops.bad_id_counter(dev))


def check_meta(meta, dev):
    """Host side of the one read: IndexError (the reference's nn.Embedding error) when the
    out-of-vocabulary counter is set; returns (max(mel_len), sum(mel_len))."""
    if int(meta[2]):
        ops.bad_id_counter(dev).zero_()
        raise IndexError(f"fs2amd: {int(meta[2])} token id(s) outside the embedding table (their encoder rows are NaN)")
    return int(meta[0]), int(meta[1])


_META_HOST = {}


def host_meta(mel_len, dev):
    """The free-running path's ONE device->host read: max(mel_len), sum(mel_len) and the
    out-of-vocabulary counter in one copy, into pinned memory the host polls (a blocking
    synchronize parks the thread: a wake-up of tens of us per call)."""
    from .graphs import _spin_until_landed

    meta = meta_vector(mel_len, dev)
    if meta.device.type != "cuda":  # host-side dry runs (tests/test_host.py)
        HOST_READS[0] += 1
        return check_meta(meta.cpu(), dev)
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)  # per stream: reentrant across threads
    ent = _META_HOST.get(key)
    if ent is None or ent[0].shape != meta.shape:
        host = torch.empty(meta.shape, dtype=meta.dtype, pin_memory=True)
        ent = _META_HOST[key] = (host, host.numpy())  # numpy view: cheap element reads while polling
    host, host_np = ent
    host_np[0] = -1
    host.copy_(meta, non_blocking=True)
    _spin_until_landed(host_np)
    torch.cuda.current_stream(dev).synchronize()
    HOST_READS[0] += 1
    return check_meta(host_np.copy(), dev)


def postnet_valid_rows(B, T, sum_len):
    """Use the PostNet's valid-region form when the padded batch is mostly padding (free-running
    synthesis: one long utterance sets T for all): its rows <= sum(len) + 20 B against B * T."""
    return postnet_valid_region_on() and B > 0 and sum_len + POSTNET_MARGIN * B < 0.5 * B * T


def _mel_copy_on(P):
    return P.compute == L.FS2_BF16 and os.environ.get("FS2_MEL_BF16", "1") != "0"


def _mel_copy(P, x, bt):
    """bf16 copy of mel_linear's output, written by the same epilogue (fs2_conv_desc.out2): PostNet's
    first conv then reads bf16 through LDS-DMA instead of converting f32 in registers. The bf16
    GEMM rounds its f32 input to bf16 the same way, so the conv's operands are unchanged."""
    if not _mel_copy_on(P):
        return None
    return torch.empty(*bt, P.mel_w.shape[0], device=x.device, dtype=torch.bfloat16)


# PostNet = 5 Conv1d(k=5, pad=2): an output frame depends on input frames within +-10.
POSTNET_REACH = 10
POSTNET_MARGIN = 2 * POSTNET_REACH


def wconv_on():
    return os.environ.get("FS2_WCONV", "1") != "0"


def pn_head_on():
    """FS2_PN_HEAD=0: the PostNet's first two convs as two fs2_wconv launches (A/B)."""
    return os.environ.get("FS2_PN_HEAD", "1") != "0"


def pn_tail_fused_on():
    """FS2_PN_TAIL_FUSED=0: the PostNet's last conv + residual as its own fs2_wconv launch (A/B)."""
    return os.environ.get("FS2_PN_TAIL_FUSED", "1") != "0"


def postnet_valid_region_on():
    return os.environ.get("FS2_POSTNET_VALID", "1") != "0"


def _postnet_consts(P, bf16_input):
    """The PostNet output wherever its input is all padding: every padded mel frame is mel_linear's
    bias (the decoder output there is masked to 0), so away from the valid frames the output is
    one constant row c, and its last POSTNET_REACH frames before T (zero padding beyond T) are one
    fixed block. Both come from one [1, 40, n_mel] run of the same kernels on bias-valued frames
    (row 20 and rows 30..39), cached per weight pack; computed outside any graph capture."""
    ent = getattr(P, "_postnet_consts", None)
    if ent is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("PostNet constants must be computed before graph capture (run the forward once)")
        b = P.mel_b.float().reshape(1, 1, -1).expand(1, 2 * POSTNET_MARGIN, -1).contiguous()
        y = _postnet(P, b, b.to(torch.bfloat16) if bf16_input else None)
        ent = (y[0, POSTNET_MARGIN].clone(), y[0, 2 * POSTNET_MARGIN - POSTNET_REACH:].clone())
        P._postnet_consts = ent
    return ent


def _postnet(P, mel, mel_bf=None, mel_len=None, sum_len=None):
    """PostNet (BN folded, transformer/Layers.py:92-137) + residual (fastspeech2.py:136) with the
    reference's padded [B, T, n_mel] semantics: padded frames (bias values) feed the k5 taps and
    get outputs too. mel_bf: optional bf16 copy of mel, the first conv's input (the residual stays
    f32).

    mel_len given: the convs run on packed rows over each utterance's valid frames + 20 (the rest
    of an utterance more than 40 frames shorter than T is constant input): its outputs are exact
    on the first len + 10 frames; frames from len + 10 to T - 10 are the constant row and the last
    10 the fixed block (_postnet_consts). An utterance within 40 frames of T runs whole. Free-
    running cfg2 (T = 959 for 11.1k valid frames) computes 12.4k rows instead of 61.4k."""
    if mel_len is not None and postnet_valid_region_on() and mel.shape[0] > 0:
        return _postnet_valid(P, mel, mel_bf, mel_len, sum_len)
    y = mel if mel_bf is None else mel_bf
    return _postnet_convs(P, y, mel)


def _postnet_convs(P, y, res, layout=None):
    """The PostNet's convs (BN folded) on y (mel's bf16 copy, or the f32 mel) + the residual res
    (f32 mel); padded [B, T, C] rows, or packed rows of ``layout`` (the valid-region form). Both
    forms take the same kernels: fs2_wconv for layers 0 + 1 (one launch), 2, 3 and the last conv +
    residual (its N = 80 form); fs2_conv1d where those shapes do not apply."""
    n_pn = len(P.postnet)
    first = 0
    if n_pn > 2 and y.dtype == torch.bfloat16 and wconv_on() and pn_head_on() and \
            getattr(P.postnet[0], "wfr", None) is not None and getattr(P.postnet[1], "wfr", None) is not None and \
            P.postnet[0].cin == 80 and P.postnet[0].k == 5 and P.postnet[0].p == 2 and P.postnet[1].p == 2:
        # layers 0 and 1 (80 -> 512 -> 512) in one launch: the first conv's output stays on chip
        l0, l1 = P.postnet[0], P.postnet[1]
        y = ops.wconv(y, l0.wfr, l0.b, ks=l0.k, pad=l0.p, second=(l1.wfr, l1.b), layout=layout)
        first = 2
    last = P.postnet[-1]
    for i, lp in enumerate(P.postnet):
        if i < first:
            continue
        if i == n_pn - 2 and n_pn > 2 and getattr(lp, "wfr", None) is not None and lp.cin == 512 and lp.k == 5 \
                and lp.p == 2 and getattr(last, "wtail", None) is not None and last.cin == 512 and last.k == 5 \
                and last.p == 2 and wconv_on() and pn_tail_fused_on() \
                and y.dtype == torch.bfloat16 and res.dtype == torch.float32:
            # layers 3 and 4 (512 -> 512 tanh, 512 -> 80 + residual) in one launch: the 512-channel
            # output stays on chip
            return ops.wconv(y, lp.wfr, lp.b, ks=lp.k, pad=lp.p, layout=layout,
                             tail=(last.wtail, last.b, res.contiguous()))
        if i < n_pn - 1 and getattr(lp, "wfr", None) is not None and wconv_on() and y.dtype == torch.bfloat16:
            # 512 -> 512 convs: the weight-streamed kernel (fs2_wconv)
            y = ops.wconv(y, lp.wfr, lp.b, ks=lp.k, pad=lp.p, layout=layout)
        elif i < n_pn - 1:
            y = ops.conv1d(y, lp.w, lp.b, cin=lp.cin, ks=lp.k, pad=lp.p, compute=P.compute,
                           epilogue=L.EPI_BIAS_TANH, out_dtype=P.act_dtype, layout=layout)
        elif getattr(lp, "wtail", None) is not None and wconv_on() and y.dtype == torch.bfloat16 \
                and res.dtype == torch.float32:
            # 512 -> 80 + residual: all 80 columns per wave, weights through an LDS ring
            y = ops.wconv_tail(y, lp.wtail, lp.b, res.contiguous(), ks=lp.k, pad=lp.p, layout=layout)
        else:
            y = ops.conv1d(y, lp.w, lp.b, cin=lp.cin, ks=lp.k, pad=lp.p, compute=P.compute, epilogue=L.EPI_BIAS_RES,
                           out_dtype=L.FS2_F32, residual=res, layout=layout)
    return y


def _postnet_valid(P, mel, mel_bf, mel_len, sum_len=None):
    B, T, C = mel.shape
    c, tail = _postnet_consts(P, mel_bf is not None)
    # each utterance's frames + POSTNET_MARGIN, or all T when within 2 margins of it
    lay = ops.SeqLayout(mel_len, T, margin=POSTNET_MARGIN)
    # the host's bound on the packed rows (free-running: sum(mel_len) from the one host read),
    # bucketed so a captured graph serves every batch of the bucket: sizes the wconv grids
    # (a function of the decoder's row bucket only, as the stage-2 graph key: rows <= sum + 20 B)
    lay.rows_hint = None if sum_len is None else \
        min(ops.rows_bucket(sum_len, B * T) + POSTNET_MARGIN * B, lay.capacity)
    # the f32 mel (the residual) and its bf16 copy (the first conv's input) packed in one launch
    res, y = ops.pack_rows(lay, mel.contiguous(), None if mel_bf is None else mel_bf.contiguous())
    if y is None:
        y = res
    y = _postnet_convs(P, y, res, layout=lay)
    # [B, T, C]: computed rows where exact, else the constant row / the tail block
    return ops.postnet_assemble(y, lay, c.contiguous(), tail.contiguous())


def _add_pe(x, pe):
    """x[b, t] += pe[t] via the LR gather with identity durations (every frame its own source)."""
    B, T, D = x.shape
    ones = torch.ones(B, T, dtype=torch.int64, device=x.device)
    cum, ml, _ = ops.lr_durations(ones)
    return ops.lr_expand(x, cum, ml, T, pe=pe, out_dtype=ops._dt(x))
