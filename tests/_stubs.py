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
            elif name == "fs2_attention":
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


def lr_expand(x, cum, mel_len, T, pe=None, out_dtype=None, index_map=False, out_layout=None, map_only=False):
    t = torch.arange(T)[None, :, None]
    src = (cum[:, None, :].long() <= t).sum(-1)
    im = torch.where(t[..., 0] < mel_len[:, None], src, torch.full_like(src, -1)).int()
    if map_only:
        return im
    return torch.zeros(x.shape[0], T, x.shape[2]), im


def install_training_stubs(setattr_fn):
    """Zero-filling kernels, CPU LR scan / masks, device check off, for fs2amd.training."""
    from fs2amd import _lib, ops, training

    lib = ZeroingLib(_lib.load())
    setattr_fn(ops, "_lib", lib)
    setattr_fn(ops, "_gpu", lambda *a: None)
    setattr_fn(ops, "_stream", lambda *a: None)
    setattr_fn(training, "_device_ok", lambda dev: True)
    setattr_fn(training, "_mask", lambda l, w: torch.arange(int(w))[None, :] >= l[:, None])
    setattr_fn(ops, "lr_durations", lr_durations)
    setattr_fn(ops, "lr_expand", lr_expand)
    return lib
