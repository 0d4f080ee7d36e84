"""fs2amd.library: the hot-path ops registered with torch.library (SURVEY §8b boundary), CPU side.

* every op exists under ``torch.ops.fs2`` after ``import fs2amd.library``;
* the fake (meta) implementations give the reference's output shapes / dtypes with no device
  (``FakeTensorMode`` over ROCm-device fakes), including the data-dependent frame count of the
  LengthRegulator when ``max_len`` is not given (an unbacked symbol);
* the real implementations refuse CPU tensors (no CPU fallback), like every entry point.
"""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode
from torch.fx.experimental.symbolic_shapes import ShapeEnv


@pytest.fixture(scope="module")
def lib():
    import fs2amd.library as lib

    return lib


def test_ops_registered(lib):
    for name in lib.OPS:
        assert hasattr(torch.ops.fs2, name), name


def test_fake_shapes(lib):
    with FakeTensorMode(shape_env=ShapeEnv()):
        qkv = torch.empty(3, 70, 768, device="cuda", dtype=torch.bfloat16)
        lens = torch.empty(3, device="cuda", dtype=torch.int64)
        o = torch.ops.fs2.attention(qkv, lens, 2, 128, 128 ** 0.5)
        assert o.shape == (3, 70, 256) and o.dtype == torch.bfloat16
        d = torch.ops.fs2.attention_bwd(qkv, o, o.float(), lens, 2, 128, 128 ** 0.5)
        assert d.shape == qkv.shape and d.dtype == torch.float32
        x = torch.empty(3, 11, 256, device="cuda", dtype=torch.bfloat16)
        dur = torch.empty(3, 11, device="cuda", dtype=torch.int64)
        y, ml = torch.ops.fs2.length_regulate(x, dur, 40)
        assert y.shape == (3, 40, 256) and y.dtype == torch.bfloat16 and ml.shape == (3,) and ml.dtype == torch.int64
        y, _ = torch.ops.fs2.length_regulate(x, dur, 0)  # max(mel_len): data-dependent
        assert y.shape[0] == 3 and y.shape[2] == 256 and not isinstance(y.shape[1], int)
        f = torch.ops.fs2.ffn(x, torch.empty(10, device="cuda", dtype=torch.bfloat16), torch.empty(1024, device="cuda"),
                              torch.empty(256, device="cuda"), torch.empty(256, device="cuda"),
                              torch.empty(256, device="cuda"), 1e-5, lens, 9, 4)
        assert f.shape == x.shape and f.dtype == x.dtype
        from fs2amd import _lib as L
        c = torch.ops.fs2.conv1d(x, torch.empty(80, 256, device="cuda", dtype=torch.bfloat16), None, 256, 1, 0,
                                 L.FS2_BF16, L.EPI_BIAS, L.FS2_F32)
        assert c.shape == (3, 11, 80) and c.dtype == torch.float32


def test_cpu_tensors_refused(lib):
    qkv = torch.zeros(1, 4, 768, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        torch.ops.fs2.attention(qkv, torch.full((1,), 4), 2, 128, 128 ** 0.5)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        torch.ops.fs2.length_regulate(torch.zeros(1, 3, 256), torch.ones(1, 3, dtype=torch.int64), 0)
