"""Host-side logic on CPU: the C-ABI library loads and exports every declared symbol, the
drop-in module has the reference's constructor / state_dict contract, packing is right."""
import ctypes
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _common import configs, manifest, oracle_state_dict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    from fs2amd import _lib

    lib = _lib.load()
    declared = _lib.header_symbols(os.path.join(REPO, "include", "fs2hip.h"))
    assert len(declared) == len(_lib.SIGNATURES) == 71
    for name in declared:
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} not bound in fs2amd/_lib.py"
    assert b"gfx950" in lib.fs2_version()
    # provenance: the loaded library was compiled from exactly these sources
    assert lib.fs2_build_id().decode() == _lib.source_build_id()
    assert lib.fs2_status_string(1) == b"invalid argument"
    assert lib.fs2_conv_cin_pad(80, _lib.FS2_BF16) == 128 and lib.fs2_conv_cin_pad(80, _lib.FS2_F32) == 96


def test_conv_desc_layout_matches_header():
    """ctypes mirror of fs2_conv_desc has the C layout (offsets computed by the compiler)."""
    import subprocess
    import tempfile

    from fs2amd import _lib

    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "fs2hip.h"
#define P(f) printf("%s %zu\n", #f, offsetof(fs2_conv_desc, f));
int main(void){ P(x) P(x_row_stride) P(w) P(B) P(compute) P(residual) P(res_row_stride) P(ln_gamma) P(ln_eps)
 P(lens) P(dot_w) P(dot_b) P(out) P(out_dtype) P(out_row_stride) P(out_div) P(group_n) P(group_cin) printf("size %zu\n", sizeof(fs2_conv_desc)); }
'''
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "t.c"), "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), os.path.join(d, "t.c"), "-o", os.path.join(d, "t")],
                   check=True)
    out = subprocess.run([os.path.join(d, "t")], capture_output=True, text=True, check=True).stdout.split("\n")
    for line in out:
        if not line:
            continue
        name, off = line.split()
        if name == "size":
            assert int(off) == ctypes.sizeof(_lib.ConvDesc)
        else:
            assert getattr(_lib.ConvDesc, name).offset == int(off), name


@pytest.mark.parametrize("cname,pyname", [("fs2_ffn_desc", "FfnDesc"), ("fs2_wconv_desc", "WconvDesc"),
                                          ("fs2_vp_fused_desc", "VpFusedDesc"), ("fs2_ffn8_desc", "Ffn8Desc"),
                                          ("fs2_pack_desc", "PackDesc"), ("fs2_loss_args", "LossArgs"),
                                          ("fs2_adam_param", "AdamParam"), ("fs2_reduce_desc", "ReduceDesc"),
                                          ("fs2_reduce_batch", "ReduceBatch"), ("fs2_cond_desc", "CondDesc"),
                                          ("fs2_cond_grads", "CondGrads")])
def test_ffn_desc_layout_matches_header(cname, pyname):
    """ctypes mirrors of fs2_ffn_desc / fs2_wconv_desc have the C layout (every field's offset, and
    the size)."""
    import subprocess
    import tempfile

    from fs2amd import _lib

    cls = getattr(_lib, pyname)
    names = [f[0] for f in cls._fields_]
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"fs2hip.h\"\nint main(void){" + "".join(
        f'printf("{n} %zu\\n", offsetof({cname}, {n}));' for n in names) + \
        f'printf("size %zu\\n", sizeof({cname})); }}\n'
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "t.c"), "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), os.path.join(d, "t.c"), "-o", os.path.join(d, "t")],
                   check=True)
    out = subprocess.run([os.path.join(d, "t")], capture_output=True, text=True, check=True).stdout.split("\n")
    seen = 0
    for line in out:
        if not line:
            continue
        name, off = line.split()
        if name == "size":
            assert int(off) == ctypes.sizeof(cls)
        else:
            assert getattr(cls, name).offset == int(off), name
            seen += 1
    assert seen == len(names)


def test_invalid_arguments_are_rejected_without_a_gpu():
    from fs2amd import _lib

    lib = _lib.load()
    d = _lib.ConvDesc()  # all-null descriptor
    assert lib.fs2_conv1d(ctypes.byref(d), None) == _lib.FS2_EINVAL
    fd = _lib.FfnDesc()  # all-null descriptor; then shapes the fused FFN does not cover
    assert lib.fs2_ffn(ctypes.byref(fd), None) == _lib.FS2_EINVAL
    for k in ("x", "w", "b1", "b2", "ln_gamma", "ln_beta", "out"):
        setattr(fd, k, 256)
    fd.x, fd.out = 512, 1024
    fd.B, fd.T, fd.D, fd.F, fd.KS, fd.pad, fd.x_row_stride, fd.out_row_stride = 2, 8, 256, 1024, 9, 4, 256, 256
    fd.D = 512
    assert lib.fs2_ffn(ctypes.byref(fd), None) == _lib.FS2_EUNSUPPORTED
    fd.D, fd.F = 256, 1000
    assert lib.fs2_ffn(ctypes.byref(fd), None) == _lib.FS2_EUNSUPPORTED
    fd.F, fd.KS = 1024, 11
    assert lib.fs2_ffn(ctypes.byref(fd), None) == _lib.FS2_EUNSUPPORTED
    fd.KS, fd.out = 9, fd.x  # out aliasing x
    assert lib.fs2_ffn(ctypes.byref(fd), None) == _lib.FS2_EINVAL
    assert lib.fs2_ffn_weight_elems(9, 1024) == 1024 * 9 * 256 + 256 * 1024
    assert lib.fs2_ffn_weight_elems(3, 512) == 512 * 3 * 256 + 256 * 512
    wd = _lib.WconvDesc()
    assert lib.fs2_wconv(ctypes.byref(wd), None) == _lib.FS2_EINVAL
    wd.x, wd.w, wd.bias, wd.out = 512, 256, 256, 1024
    wd.B, wd.T, wd.Cin, wd.N, wd.KS, wd.pad, wd.x_row_stride, wd.out_row_stride = 2, 8, 512, 512, 5, 2, 512, 512
    wd.epilogue = _lib.EPI_BIAS_RELU
    assert lib.fs2_wconv(ctypes.byref(wd), None) == _lib.FS2_EUNSUPPORTED
    wd.epilogue, wd.KS = _lib.EPI_BIAS_TANH, 3
    assert lib.fs2_wconv(ctypes.byref(wd), None) == _lib.FS2_EUNSUPPORTED
    wd.KS, wd.out = 5, wd.x
    assert lib.fs2_wconv(ctypes.byref(wd), None) == _lib.FS2_EINVAL
    assert lib.fs2_wconv_weight_elems(5, 512, 512) == 512 * 5 * 512

    assert lib.fs2_attention(None, 0, 768, None, 1, 1, 2, 128, 11.3, None, 256, None, None, None) == _lib.FS2_EINVAL
    assert lib.fs2_lr_durations(None, 0, 1.0, 1, 1, None, None, None, None) == _lib.FS2_EINVAL
    assert lib.fs2_lr_expand(None, 0, None, None, 1, 1, 8, 1, None, None, 0, None, None, None) == _lib.FS2_EINVAL
    assert lib.fs2_vp_norm(None, 512, 1, 2, 256, None, None, 1e-5, None, 1024, None) == _lib.FS2_EINVAL
    assert lib.fs2_vp_head(None, 512, 1, 1, 2, 256, None, None, 1e-5, None, None, None, None, -1, None, 0, 256, 256,
                           None, 1.0, None, 256, None, None) == _lib.FS2_EINVAL
    assert lib.fs2_seq_layout(None, 1, 1, None, None, None, None) == _lib.FS2_EINVAL
    vd = _lib.VpFusedDesc()
    assert lib.fs2_vp_fused(ctypes.byref(vd), None) == _lib.FS2_EINVAL
    for k in ("x", "w", "vec", "lin_b", "lens", "pred"):
        setattr(vd, k, 256)
    vd.x, vd.B, vd.L, vd.G, vd.x_row_stride, vd.embed_group = 512, 2, 8, 3, 256, -1
    assert lib.fs2_vp_fused(ctypes.byref(vd), None) == _lib.FS2_EINVAL  # G = 3
    vd.G, vd.embed_group = 2, 1
    assert lib.fs2_vp_fused(ctypes.byref(vd), None) == _lib.FS2_EINVAL  # embedding without x_out / bins / table
    vd.x_out, vd.bins, vd.table, vd.n_bins, vd.x_out_row_stride = vd.x, 256, 256, 256, 256
    assert lib.fs2_vp_fused(ctypes.byref(vd), None) == _lib.FS2_EINVAL  # x_out aliasing x
    assert lib.fs2_vp_fused_weight_elems(2) == 2 * 4 * 2 * 24 * 2 * 2048


def _model():
    from fs2amd.model import FastSpeech2

    pc, mc, _ = configs()
    return FastSpeech2(pc, mc)


def test_state_dict_contract_matches_reference():
    m = _model()
    sd = m.state_dict()
    man = manifest()["keys"]
    assert list(sd.keys()) == list(man.keys()) or set(sd.keys()) == set(man.keys())
    assert len(sd) == 240
    for k, v in sd.items():
        assert list(v.shape) == man[k]["shape"], k
    # constructor-computed tensors are identical to the reference's (PE tables, bins)
    for k in ("encoder.position_enc", "decoder.position_enc", "variance_adaptor.pitch_bins",
              "variance_adaptor.energy_bins"):
        import hashlib
        assert hashlib.sha256(sd[k].numpy().tobytes()).hexdigest() == man[k]["sha256"], k
    n_train = sum(p.numel() for p in m.parameters() if p.requires_grad)
    assert n_train == 34_659_075


def test_load_reference_state_dict_strict():
    m = _model()
    m.load_state_dict(oracle_state_dict(), strict=True)


def test_packing_batchnorm_fold_and_layouts():
    """Packed operands reproduce the reference ops in plain torch (CPU)."""
    from fs2amd import _lib as L
    from fs2amd.packing import pack_model

    m = _model()
    m.load_state_dict(oracle_state_dict())
    m.eval()
    P = pack_model(m, "cpu", "fp32")
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 31, 512, generator=g)
    seq = m.postnet.convolutions[1]
    with torch.no_grad():
        ref = seq[1](seq[0].conv(x.transpose(1, 2))).transpose(1, 2)
    lp = P.postnet[1]
    w = lp.w[:, :, :512].permute(0, 2, 1)
    got = F.conv1d(x.transpose(1, 2), w, lp.b, padding=2).transpose(1, 2)
    assert float((got - ref).abs().max()) < 1e-4
    lay = P.enc_layers[0]
    a = m.encoder.layer_stack[0].slf_attn
    assert torch.equal(lay.wqkv[:256, 0, :], a.w_qs.weight) and torch.equal(lay.wqkv[512:, 0, :], a.w_vs.weight)
    assert lay.w1.shape == (1024, 9, 256) and torch.equal(lay.w1[:, 3, :], m.encoder.layer_stack[0].pos_ffn.w_1.weight[:, :, 3])
    Pb = pack_model(m, "cpu", "bf16")
    assert Pb.enc_layers[0].w1.dtype == torch.bfloat16 and Pb.vp["pitch"].w1.dtype == torch.float32
    assert Pb.postnet[0].w.shape == (512, 5, 128)


def test_forward_refuses_cpu_tensors_eval_and_train():
    from fs2amd.data import synth_batch

    m = _model().eval()
    with pytest.raises(RuntimeError, match="HIP"):
        with torch.no_grad():
            m(**synth_batch(1, 8, seed=3))
    m.train()
    with pytest.raises(RuntimeError, match="HIP"):
        m(**synth_batch(1, 8, seed=3, with_mels=True, pe_targets=True))


def test_drop_in_import_path():
    """`from model import FastSpeech2, FastSpeech2Loss, ScheduledOptim` like the reference callers."""
    import importlib
    import sys

    pkg_root = os.path.join(REPO, "expressive-fastspeech2-mandarin_amd")
    sys.path.insert(0, pkg_root)
    mod = importlib.import_module("model")
    assert mod.__file__.startswith(pkg_root)
    from fs2amd.model import FastSpeech2
    assert mod.FastSpeech2 is FastSpeech2
    assert hasattr(mod, "FastSpeech2Loss") and hasattr(mod, "ScheduledOptim")


from _stubs import RecordingLib as _RecordingLib  # noqa: E402


class _FakeForkJoin:
    def __init__(self, dev, n):
        import contextlib

        self.n = n
        self.ctx = lambda i: contextlib.nullcontext()

    def fork(self):
        pass

    def join(self, *t):
        pass


def stub_seq_layout(monkeypatch, ops):
    """With the kernels stubbed fs2_seq_layout writes nothing: fill cu / rowmap on the host (the
    PostNet's valid-region path indexes with the row map in torch); likewise the free-running host
    read's [max, sum, bad ids] (fs2_len_stats) from torch."""
    real_layout_init = ops.SeqLayout.__init__
    real_lr_fused = ops.lr_fused

    def fill(self, lens, T, margin=0):
        ln = lens.to(torch.int64)
        if margin:
            ln = torch.where(ln + 2 * margin > T, torch.full_like(ln, T), ln + margin)
        ln = ln.clamp(0, T)
        cu = torch.cat([ln.new_zeros(1), ln.cumsum(0)])
        t = torch.arange(T)
        rm = torch.where(t[None, :] < ln[:, None], cu[:-1, None] + t[None, :], torch.full((1,), -1))
        self.rowmap.copy_(rm.reshape(-1).to(torch.int32))
        self.cu.copy_(cu.to(torch.int32))

    def layout_init(self, lens, T, margin=0):
        real_layout_init(self, lens, T, margin)
        fill(self, lens, T, margin)

    def lr_fused(x, lens, T_out, **kw):  # the one-launch LR builds its layout on the device
        r = real_lr_fused(x, lens, T_out, **kw)
        fill(r[1], lens, T_out)
        return r

    monkeypatch.setattr(ops.SeqLayout, "__init__", layout_init)
    monkeypatch.setattr(ops, "lr_fused", lr_fused)
    monkeypatch.setattr(ops, "len_stats", lambda lens, bad=None: torch.stack(
        [lens.max(), lens.sum(), torch.zeros((), dtype=lens.dtype)]).to(torch.int32))


@pytest.mark.parametrize("packed", ["1", "0"])
@pytest.mark.parametrize("teacher", [True, False])
@pytest.mark.parametrize("streams", ["1", "2"])
def test_forward_launch_sequence_dry_run(monkeypatch, packed, teacher, streams):
    """The forward's Python plumbing (shapes, strides, descriptors, layouts) on CPU with the
    kernels stubbed: no GPU needed, catches argument errors before any GPU time is spent."""
    from fs2amd import ops, runtime, _lib
    from fs2amd.data import synth_batch

    rec = _RecordingLib(_lib.load())
    monkeypatch.setattr(ops, "_lib", rec)
    monkeypatch.setattr(ops, "_gpu", lambda *a: None)
    monkeypatch.setattr(ops, "_stream", lambda *a: None)
    monkeypatch.setattr(runtime, "_device_ok", lambda dev: True)
    monkeypatch.setenv("FS2_PACKED_DECODER", packed)
    monkeypatch.setenv("FS2_STREAMS", streams)
    monkeypatch.setattr(runtime, "_ForkJoin", _FakeForkJoin)
    stub_seq_layout(monkeypatch, ops)
    m = _model().eval()
    args = synth_batch(17, 6, 11, seed=2, teacher=teacher)
    if not teacher:
        # the stubbed duration kernel writes nothing: give mel_len a defined size
        real_lr = ops.lr_durations

        def lr_durations(dur, logpred=False, d_control=1.0):
            cum, ml, dr = real_lr(dur, logpred, d_control)
            ml.fill_(7)
            return cum, ml, dr

        monkeypatch.setattr(ops, "lr_durations", lr_durations)
    with torch.no_grad():
        out = m(**args)
    assert len(out) == 10 and out[0].shape[-1] == 80 and out[1].shape == out[0].shape
    assert out[0].shape[0] == 17 and out[9].shape == (17,)
    n_conv = rec.calls.count("fs2_conv1d")
    k = int(streams)
    # per group: 10 FFT blocks x 4 GEMMs + 3 VPs x 2 + mel_linear + 5 PostNet convs (these batches
    # are not mostly padding: the padded PostNet form)
    assert n_conv == k * (10 * 4 + 6 + 1 + 5), rec.calls
    assert rec.calls.count("fs2_attention_ex") == k * 10
    # the packed decoder's layout: built by the one-launch LengthRegulator (fs2_lr_fused)
    assert any(c.startswith("fs2_lr_fused") for c in rec.calls) == (packed == "1")
    assert ("fs2_lr_expand" in rec.calls) == (packed == "0")


def test_training_step_dry_run(monkeypatch):
    """train.py's step (forward, FastSpeech2Loss, backward) through fs2amd.training on CPU with the
    kernels stubbed (zeros) and the LR scan / masks done by the test: checks the autograd graph
    reaches exactly the parameters the reference's own step gives gradients to."""
    import numpy as np
    from fs2amd.data import loss_inputs, synth_batch
    from fs2amd.loss import FastSpeech2Loss
    from _common import GOLDEN
    from _stubs import install_training_stubs

    lib = install_training_stubs(monkeypatch.setattr)
    pc, mc, _ = configs()
    m = _model().train()
    args = synth_batch(3, 5, 9, seed=4, with_mels=True, pe_targets=True)
    out = m(**args)
    assert out[0].shape == (3, int(args["max_mel_len"]), 80)
    losses = FastSpeech2Loss(pc, mc)(loss_inputs(args), out)
    losses[0].backward()
    got = {k for k, p in m.named_parameters() if p.grad is not None}
    ref = {str(k) for k in np.load(f"{GOLDEN}/train_grads.npz")["grad_keys"]}
    assert got == ref, got ^ ref
    assert "fs2_conv1d" in lib.calls and "fs2_attention_ex" in lib.calls


def test_loss_matches_oracle_masked_select_form():
    """fs2amd.loss (mask-weighted sums, no host sync) vs the oracle's restatement of
    model/loss.py (masked_select + mean), with gradients."""
    from oracle import fs2_oracle as O
    from fs2amd.loss import FastSpeech2Loss

    pc, mc, _ = configs()
    g = torch.Generator().manual_seed(0)
    B, L, T = 3, 9, 31
    src_lens, mel_lens = torch.tensor([9, 5, 1]), torch.tensor([31, 17, 4])
    src_masks = torch.arange(L)[None, :] >= src_lens[:, None]
    mel_masks = torch.arange(T)[None, :] >= mel_lens[:, None]
    preds = [torch.randn(B, T, 80, generator=g, requires_grad=True), torch.randn(B, T, 80, generator=g, requires_grad=True),
             torch.randn(B, L, generator=g, requires_grad=True), torch.randn(B, L, generator=g, requires_grad=True),
             torch.randn(B, L, generator=g, requires_grad=True)]
    out = (*preds, None, src_masks, mel_masks, src_lens, mel_lens)
    mels, pt, et = torch.randn(B, T + 2, 80, generator=g), torch.randn(B, L, generator=g), torch.randn(B, L, generator=g)
    dur = torch.randint(0, 7, (B, L), generator=g)
    ours = FastSpeech2Loss(pc, mc)((None,) * 9 + (mels, mel_lens, T, pt, et, dur), out)
    ref = O.loss(pc, mels, pt, et, dur, out)
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    ga = torch.autograd.grad(ours[0], preds)
    gb = torch.autograd.grad(ref[0], preds)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("compute", [0, 1])
@pytest.mark.parametrize("cin", [80, 256])
def test_pack_conv_weight_layout(compute, cin):
    """packed[n, k, c] == w[n, c, k] (zero channel padding), contiguous, compute dtype."""
    from fs2amd import ops

    w = torch.randn(12, cin, 5)
    p = ops.pack_conv_weight(w, compute)
    assert p.is_contiguous() and p.dtype == ops.torch_dtype(compute)
    assert p.shape == (12, 5, ops.cin_pad(cin, compute))
    torch.testing.assert_close(p[:, :, :cin].float(), w.permute(0, 2, 1).to(p.dtype).float())
    assert not p[:, :, cin:].float().abs().sum()


def test_checkpoint_resume_round_trip(tmp_path):
    """train.py:151-161 save -> utils/model.py:11-34 restore: the 240-key model state, Adam's
    moments and the Noam step counter (model/optimizer.py:19) come back, and one more step from
    the restored pair equals one more step of the original (CPU, gradients injected)."""
    import types
    from fs2amd import config as C
    from fs2amd.checkpoint import checkpoint_path, get_model, load_checkpoint, save_checkpoint
    from fs2amd.optimizer import ScheduledOptim

    pc, mc, _ = configs()
    tc = dict(C.ESD_TRAIN_CONFIG, path={"ckpt_path": str(tmp_path)})
    m = _model()
    opt = ScheduledOptim(m, tc, mc, 0)
    g = torch.Generator().manual_seed(0)
    grads = [[torch.randn(p.shape, generator=g) * 1e-2 for p in m.parameters()] for _ in range(3)]

    def step(model, o, gs):
        for p, gr in zip(model.parameters(), gs):
            p.grad = gr.clone() if p.requires_grad else None
        o.step_and_update_lr()
        o.zero_grad()

    step(m, opt, grads[0])
    step(m, opt, grads[1])
    save_checkpoint(checkpoint_path(tc, 2), m, opt)
    ck = load_checkpoint(checkpoint_path(tc, 2))
    assert set(ck) == {"model", "optimizer"} and len(ck["model"]) == 240
    m2, opt2 = get_model(types.SimpleNamespace(restore_step=2), (pc, mc, tc), "cpu", train=True)
    assert opt2.current_step == 2 and m2.training
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k
    step(m, opt, grads[2])
    step(m2, opt2, grads[2])
    assert opt.current_step == opt2.current_step == 3
    assert opt._optimizer.param_groups[0]["lr"] == opt2._optimizer.param_groups[0]["lr"]
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k
    ev = get_model(types.SimpleNamespace(restore_step=2), (pc, mc, tc), "cpu")
    assert not ev.training


def test_pack_ffn_weights_layout():
    """fs2_ffn's weight buffer: w_1 then w_2 in MFMA fragment order (include/fs2hip.h, fs2_ffn)."""
    from fs2amd import ops

    g = torch.Generator().manual_seed(0)
    for F, ks in ((1024, 9), (1024, 3), (512, 3)):
        w1, w2 = torch.randn(F, 256, ks, generator=g), torch.randn(256, F, 1, generator=g)
        p = ops.pack_ffn_weights(w1, w2)
        assert p.shape == (F * ks * 256 + 256 * F,) and p.dtype == torch.bfloat16
        a = p[:F * ks * 256].view(F // 64, ks, 8, 4, 4, 16, 8)
        b = p[F * ks * 256:].view(4, F // 32, 4, 4, 16, 8)
        for q, k, s_, bb, h, r, e in ((0, 0, 0, 0, 0, 0, 0), (3, ks - 1, 5, 2, 3, 11, 6), (F // 64 - 1, 1, 7, 3, 1, 15, 7)):
            assert a[q, k, s_, bb, h, r, e] == w1[64 * q + 16 * bb + r, 32 * s_ + 8 * h + e, k].to(torch.bfloat16)
        for q, s_, bb, h, r, e in ((0, 0, 0, 0, 0, 0), (2, F // 32 - 1, 1, 2, 9, 4), (3, 3, 3, 3, 15, 7)):
            assert b[q, s_, bb, h, r, e] == w2[64 * q + 16 * bb + r, 32 * s_ + 8 * h + e, 0].to(torch.bfloat16)
        # a permutation: every weight exactly once
        assert torch.equal(p.float().sort().values, torch.cat([w1.reshape(-1), w2.reshape(-1)]).to(torch.bfloat16).float().sort().values)


def test_pack_train_plan_on_host():
    """fs2_pack_train_plan (host-only): workgroups per descriptor = 32 x 32 (n, c) tiles, 256
    elements per f32 copy; invalid descriptors rejected."""
    from fs2amd import _lib

    lib = _lib.load()
    arr = (_lib.PackDesc * 3)()
    for d in arr:
        d.src, d.fwd = 4096, 8192
    arr[0].N, arr[0].C, arr[0].KS, arr[0].N_tot = 1024, 256, 9, 1024
    arr[1].N, arr[1].C, arr[1].KS, arr[1].N_tot, arr[1].n_off = 256, 1024, 1, 512, 256
    arr[2].N, arr[2].f32_copy = 768, 1
    nb = ctypes.c_int(0)
    assert lib.fs2_pack_train_plan(arr, 3, ctypes.byref(nb)) == _lib.FS2_OK
    assert (arr[0].blk0, arr[1].blk0, arr[2].blk0) == (0, 256, 512) and nb.value == 515
    arr[1].n_off = 300  # past N_tot
    assert lib.fs2_pack_train_plan(arr, 3, ctypes.byref(nb)) == _lib.FS2_EINVAL
