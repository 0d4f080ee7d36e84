"""The HIP hot path as ``torch.library`` custom ops ("registered as torch.library ops
(fs2::length_regulate, ...) so autograd and DDP work").

Each op wraps the C-ABI launch of :mod:`fs2amd.ops` (no CPU fallback: CPU tensors raise, as every
entry point does) and carries a fake (meta) implementation, so ``torch.compile`` / ``torch.export``
trace through it with ``fullgraph=True`` instead of breaking the graph at a ctypes call:

* ``fs2::length_regulate(x, duration, max_len) -> (out, mel_len)`` —
  ``LengthRegulator.forward`` (model/modules.py:161-194 + utils/tools.py:360-378); ``max_len <= 0``
  means max(mel_len) (a data-dependent size: an unbacked symbol under tracing).
* ``fs2::attention(qkv, lens, n_head, d_k, temperature) -> out`` — ``ScaledDotProductAttention`` with
  the key-padding mask and the head split / merge (transformer/Modules.py:14-25,
  transformer/SubLayers.py:36-52) over the fused [B, T, 3·H·dk] projection; differentiable
  (backward: ``fs2::attention_bwd``, the flash-style recompute of fs2_attention_bwd).
* ``fs2::attention_bwd(qkv, out, dout, lens, n_head, d_k, temperature) -> dqkv`` (f32).
* ``fs2::ffn(x, w_packed, b1, b2, ln_gamma, ln_beta, ln_eps, lens, ks, pad) -> y`` — the FFT block's
  ``PositionwiseFeedForward`` + residual + LayerNorm + padding mask (transformer/SubLayers.py:85-93,
  transformer/Layers.py:28) as one fs2_ffn launch (inference; weights from ops.pack_ffn_weights).
* ``fs2::conv1d(x, w_packed, bias, cin, ks, pad, compute, epilogue, out_dtype) -> y`` — fs2_conv1d
  with a plain (bias / activation) epilogue.

Importing this module (``import fs2amd.library``, or the ``model`` drop-in package) registers the ops;
the C library itself is loaded at the first launch.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import ops


@torch.library.custom_op("fs2::length_regulate", mutates_args=())
def length_regulate(x: Tensor, duration: Tensor, max_len: int) -> Tuple[Tensor, Tensor]:
    out, mel_len = ops.length_regulate(x, duration, max_len if max_len > 0 else None)
    return out, mel_len


@length_regulate.register_fake
def _length_regulate_fake(x, duration, max_len):
    B, _, D = x.shape
    T = max_len if max_len > 0 else torch.library.get_ctx().new_dynamic_size()
    return x.new_empty(B, T, D), duration.new_empty(B, dtype=torch.int64)


@torch.library.custom_op("fs2::attention", mutates_args=())
def attention(qkv: Tensor, lens: Tensor, n_head: int, d_k: int, temperature: float) -> Tensor:
    return ops.attention(qkv, lens, n_head, d_k, temperature)


@attention.register_fake
def _attention_fake(qkv, lens, n_head, d_k, temperature):
    B, T, _ = qkv.shape
    return qkv.new_empty(B, T, n_head * d_k)


@torch.library.custom_op("fs2::attention_bwd", mutates_args=())
def attention_bwd(qkv: Tensor, out: Tensor, dout: Tensor, lens: Tensor, n_head: int, d_k: int,
                  temperature: float) -> Tensor:
    return ops.attention_bwd(qkv, out, dout, lens, n_head, d_k, temperature)


@attention_bwd.register_fake
def _attention_bwd_fake(qkv, out, dout, lens, n_head, d_k, temperature):
    return qkv.new_empty(qkv.shape, dtype=torch.float32)


def _attention_setup(ctx, inputs, output):
    qkv, lens, n_head, d_k, temperature = inputs
    ctx.save_for_backward(qkv, lens, output)
    ctx.meta = (n_head, d_k, temperature)


def _attention_backward(ctx, grad):
    qkv, lens, out = ctx.saved_tensors
    dqkv = torch.ops.fs2.attention_bwd(qkv, out, grad, lens, *ctx.meta)
    return dqkv.to(qkv.dtype), None, None, None, None


torch.library.register_autograd("fs2::attention", _attention_backward, setup_context=_attention_setup)


@torch.library.custom_op("fs2::ffn", mutates_args=())
def ffn(x: Tensor, w_packed: Tensor, b1: Tensor, b2: Tensor, ln_gamma: Tensor, ln_beta: Tensor, ln_eps: float,
        lens: Optional[Tensor], ks: int, pad: int) -> Tensor:
    return ops.ffn(x, w_packed, b1, b2, ks=ks, pad=pad, ln=(ln_gamma, ln_beta, ln_eps), lens=lens)


@ffn.register_fake
def _ffn_fake(x, w_packed, b1, b2, ln_gamma, ln_beta, ln_eps, lens, ks, pad):
    return torch.empty_like(x)


@torch.library.custom_op("fs2::conv1d", mutates_args=())
def conv1d(x: Tensor, w_packed: Tensor, bias: Optional[Tensor], cin: int, ks: int, pad: int, compute: int,
           epilogue: int, out_dtype: int) -> Tensor:
    """fs2_conv1d with a plain epilogue (bias / bias + ReLU / bias + tanh / bias + leaky ReLU):
    ``nn.Conv1d`` / ``nn.Linear`` over [B, T, C] rows (the VariancePredictor / PostNet / mel_linear
    convolutions, model/modules.py:253-296, transformer/Layers.py:33-137, model/fastspeech2.py:134);
    w_packed from ops.pack_conv_weight (N = w_packed.shape[0] output channels)."""
    from . import _lib as L
    if epilogue not in (L.EPI_BIAS, L.EPI_BIAS_RELU, L.EPI_BIAS_TANH, L.EPI_BIAS_LRELU):
        raise ValueError("fs2::conv1d: plain epilogues only (residual / LayerNorm forms go through fs2amd.ops)")
    return ops.conv1d(x, w_packed, bias, cin=cin, ks=ks, pad=pad, compute=compute, epilogue=epilogue,
                      out_dtype=out_dtype)


@conv1d.register_fake
def _conv1d_fake(x, w_packed, bias, cin, ks, pad, compute, epilogue, out_dtype):
    B, T, _ = x.shape
    return x.new_empty(B, T, w_packed.shape[0], dtype=ops.torch_dtype(out_dtype))


OPS = ("length_regulate", "attention", "attention_bwd", "ffn", "conv1d")
