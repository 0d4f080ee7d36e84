"""fs2amd.graphs.SynthGraphs — free-running synthesis as two HIP graphs around ONE host read.

* outputs bit-identical to the eager forward (same kernels, same order) in fp32 and bf16, on the
  committed cfg2 free-running reference inputs, on a second batch of the same shape (static
  input refill) and on a batch with another T_out (a new stage-2 graph);
* exactly one device->host read per call, eager and graphed: runtime.HOST_READS, and torch's
  synchronizing-operation detector (set_sync_debug_mode) sees at most that one;
* out-of-vocabulary ids raise IndexError at that read, as nn.Embedding does in the reference.
"""
import warnings

import numpy as np
import pytest
import torch

from _common import configs, load_case, oracle_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from fs2amd.model import FastSpeech2

    pc, mc, _ = configs()
    m = FastSpeech2(pc, mc)
    m.load_state_dict(oracle_state_dict())
    return m.to(DEV).eval()


def _dev(args):
    from fs2amd.data import to_device

    return to_device({k: v for k, v in args.items() if k not in ("mels", "mel_lens", "max_mel_len", "d_targets")}, DEV)


def _same(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x is None or y is None:
            assert x is None and y is None, i
            continue
        assert x.shape == y.shape and torch.equal(x, y), i


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_graphs_equal_eager(model, prec):
    from fs2amd.data import synth_batch
    from fs2amd.graphs import SynthGraphs

    model.set_precision(prec)
    args, _, _, _ = load_case("cfg2_free")
    b1 = _dev(args)
    synth = SynthGraphs(model)
    with torch.no_grad():
        _same(synth(**b1), model(**b1))
        # same shapes, other values: the static inputs refill (and T_out may move)
        b2 = _dev(synth_batch(64, 64, seed=77, teacher=False))
        b2 = dict(b2, max_src_len=b1["max_src_len"], texts=torch.nn.functional.pad(
            b2["texts"], (0, b1["max_src_len"] - b2["texts"].shape[1])))
        _same(synth(**b2), model(**b2))
        _same(synth(**b1), model(**b1))
        # controls are part of the stage-1 key; a d_control change moves T_out (new stage-2 graph)
        _same(synth(**b1, d_control=1.2), model(**b1, d_control=1.2))
    assert synth.captures >= 3


def test_one_host_read_per_call(model):
    from fs2amd import runtime as R
    from fs2amd.graphs import SynthGraphs

    model.set_precision("bf16")
    args, _, _, _ = load_case("cfg2_free")
    b = _dev(args)
    synth = SynthGraphs(model)
    with torch.no_grad():
        synth(**b)  # captures
        model(**b)
        torch.cuda.synchronize()
        for fn in (lambda: model(**b), lambda: synth(**b)):
            n0 = R.HOST_READS[0]
            torch.cuda.set_sync_debug_mode("warn")
            try:
                with warnings.catch_warnings(record=True) as w:
                    warnings.simplefilter("always")
                    fn()
            finally:
                torch.cuda.set_sync_debug_mode(0)
            syncs = [x for x in w if "synchroniz" in str(x.message)]
            assert R.HOST_READS[0] - n0 == 1
            assert len(syncs) <= 1, [str(x.message) for x in syncs]


def test_bad_ids_raise(model):
    from fs2amd.graphs import SynthGraphs

    model.set_precision("bf16")
    args, _, _, _ = load_case("cfg2_free")
    b = _dev(args)
    bad = dict(b, texts=b["texts"].clone())
    bad["texts"][3, 0] = 10_000
    synth = SynthGraphs(model)
    with torch.no_grad():
        with pytest.raises(IndexError):
            model(**bad)
        with pytest.raises(IndexError):
            synth(**bad)
        # the counter was reset: a clean batch runs
        out = synth(**b)
    assert np.isfinite(out[1].float().cpu().numpy()).all()


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_weight_change_recaptures_both_stages(model, prec):
    """A parameter changed in place between two calls (a training step, a checkpoint load) builds a
    new weight pack: the stage-1 graph AND the stage-2 graphs captured on its outputs must be
    dropped and recaptured (a replayed stale stage-2 graph would read the old pack and the freed
    stage-1 buffers). Both calls must equal the eager forward on the weights of the time."""
    from fs2amd.graphs import SynthGraphs

    model.set_precision(prec)
    args, _, _, _ = load_case("cfg2_free")
    b = _dev(args)
    synth = SynthGraphs(model)
    w = model.decoder.layer_stack[0].pos_ffn.w_1.weight
    saved = w.detach().clone()
    try:
        with torch.no_grad():
            _same(synth(**b), model(**b))
            n = synth.captures
            w.mul_(1.25)  # decoder-only change: T_out and the stage-2 key stay the same
            _same(synth(**b), model(**b))
            # every graph of the first call recaptured (stage 1 + stage 2's one or two graphs)
            assert synth.captures == 2 * n, (synth.captures, n)
    finally:
        with torch.no_grad():
            w.copy_(saved)
    synth.close()


def test_stage1_lru_bound(model):
    """Stage-1 graphs are an LRU too (a serving loop with many batch shapes / controls must not grow
    GPU memory without bound); evicting one drops the stage-2 graphs that read its outputs."""
    from fs2amd.graphs import SynthGraphs

    model.set_precision("bf16")
    args, _, _, _ = load_case("cfg2_free")
    b = _dev(args)
    synth = SynthGraphs(model, max_stage1=2)
    with torch.no_grad():
        for d in (1.0, 1.1, 1.2):
            _same(synth(**b, d_control=d), model(**b, d_control=d))
    assert len(synth._g1) == 2
    keys1 = list(synth._g1)
    assert all(any(k[:len(k1)] == k1 for k1 in keys1) for k in synth._g2)
    synth.close()
