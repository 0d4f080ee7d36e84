"""CPU stand-ins for libfs2hip.so used by the dry-run tests (no GPU): they let the Python
plumbing of the forward / training step run on CPU tensors so argument, shape and autograd
errors surface before GPU time. The numbers they produce are NOT parity data."""
import ctypes

import torch


class RecordingLib:
    """Stands in for libfs2hip.so: records every launch entry point call, returns FS2_OK.
    Host-only helpers (cin_pad, version strings) go to the real library."""

    HOST = {"fs2_conv_cin_pad", "fs2_status_string", "fs2_version"}

    def __init__(self, real):
        self.real, self.calls = real, []

    def __getattr__(self, name):
        if name in self.HOST:
            return getattr(self.real, name)

        def call(*args):
            self.calls.append(name)
            return 0

        return call


class ZeroingLib(RecordingLib):
    """Recording stub that also zero-fills the outputs of conv / attention launches."""

    def __getattr__(self, name):
        if name in self.HOST:
            return getattr(self.real, name)

        def call(*args):
            self.calls.append(name)
            if name == "fs2_conv1d":
                d = args[0]._obj
                es = 2 if d.out_dtype == 1 else 4
                ctypes.memset(d.out, 0, d.B * d.T * (d.out_row_stride if d.epilogue != 6 else 1) * es)
            elif name in ("fs2_attention", "fs2_attention_ex"):
                B, T, out, os_ = args[4], args[5], args[9], args[10]
                ctypes.memset(out, 0, B * T * os_ * (2 if args[1] == 1 else 4))
            elif name == "fs2_attention_bwd":  # dqkv f32 [B*T, >= 3*H*dk] (else uninitialised memory)
                B, T, dqkv, rs = args[8], args[9], args[13], args[14]
                ctypes.memset(dqkv, 0, B * T * rs * 4)
            return 0

        return call


def lr_durations(dur, logpred=False, d_control=1.0):
    f = torch.clamp(dur.long(), min=0)
    return torch.cumsum(f, 1).int(), f.sum(1), None


def _index_map(cum, mel_len, T):
    t = torch.arange(T)[None, :, None]
    src = (cum[:, None, :].long() <= t).sum(-1)
    return torch.where(t[..., 0] < mel_len[:, None], src, torch.full_like(src, -1)).int()


def lr_expand(x, cum, mel_len, T, pe=None, out_dtype=None, index_map=False, out_layout=None, map_only=False):
    im = _index_map(cum, mel_len, T)
    if map_only:
        return im
    B, L, D = x.shape
    xz = torch.cat([x.float(), x.new_zeros(B, 1, D, dtype=torch.float32)], 1)
    idx = torch.where(im < 0, torch.full_like(im, L), im).long()
    out = torch.gather(xz, 1, idx.unsqueeze(-1).expand(-1, -1, D))
    if pe is not None:
        out = out + pe[:T]
    return (out, im) if index_map else out


def lr_backward(dy, cum, n):
    B, T, D = dy.shape
    im = _index_map(cum, cum[:, -1].long() if cum.shape[1] else torch.zeros(B, dtype=torch.long), T).long()
    dx = torch.zeros(B, n + 1, D)
    return dx.scatter_add_(1, torch.where(im < 0, n, im).unsqueeze(-1).expand(-1, -1, D), dy.float())[:, :n]


def variance_embed_ex(x, value, bins, table):
    idx = torch.bucketize(value.float(), bins)
    return x + table[idx], idx


def embedding_bwd(tokens, dy, V, padding_idx=None, out=None, accumulate=False):
    D = dy.shape[-1]
    g = torch.zeros(V, D).index_add_(0, tokens.reshape(-1).long(), dy.reshape(-1, D).float())
    if padding_idx is not None:
        g[padding_idx] = 0
    if out is None:
        return g
    if accumulate:
        out.add_(g)
    else:
        out.copy_(g)
    return out


def install_training_stubs(setattr_fn):
    """Zero-filling kernels, CPU LR scan / gather / its gradient, bucketize + embedding, masks,
    device check off, for fs2amd.training."""
    from fs2amd import _lib, ops, training

    lib = ZeroingLib(_lib.load())
    setattr_fn(ops, "_lib", lib)
    setattr_fn(ops, "_gpu", lambda *a: None)
    setattr_fn(ops, "_stream", lambda *a: None)
    setattr_fn(training, "_device_ok", lambda dev: True)
    setattr_fn(training, "_mask", lambda l, w: torch.arange(int(w))[None, :] >= l[:, None])
    setattr_fn(ops, "lr_durations", lr_durations)
    setattr_fn(ops, "lr_expand", lr_expand)
    setattr_fn(ops, "lr_backward", lr_backward)
    setattr_fn(ops, "variance_embed_ex", variance_embed_ex)
    setattr_fn(ops, "embedding_bwd", embedding_bwd)
    return lib
