"""Host input pipeline on the GPU: the packed pinned H2D (one copy per batch) gives exactly the
reference's to_device tensors, the Prefetcher delivers every batch in order, and the model
called positionally with the reference's tuples equals the keyword call."""
import os

import numpy as np
import pytest
import torch

from _common import GOLDEN, configs, oracle_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from fs2amd.pipeline import write_synthetic_corpus

    return write_synthetic_corpus(str(tmp_path_factory.mktemp("corpus")), 24, seed=0, long_every=11, max_seq_len=2000)


def _cfg(corpus):
    from fs2amd import config as C

    pc, mc, _ = configs()
    return dict(pc, path={"preprocessed_path": corpus}), mc, C.ESD_TRAIN_CONFIG


def test_packed_h2d_matches_reference_to_device(corpus):
    from fs2amd.pipeline import Dataset, to_device

    ref = np.load(os.path.join(GOLDEN, "pipeline_batches.npz"))
    pc, mc, tc = _cfg(corpus)
    ds = Dataset("train.txt", pc, mc, tc, sort=True)
    batches = ds.collate_fn([ds[i] for i in range(len(ds))])
    outs = [to_device(b, DEV) for b in batches]  # back-to-back: exercises the double-buffered slots
    torch.cuda.synchronize()
    for j, b in enumerate(outs):
        for k, v in enumerate(b):
            if torch.is_tensor(v):
                assert v.is_cuda and str(v.dtype) == str(ref[f"train_sorted__{j}__{k}__dtype"])
                np.testing.assert_array_equal(v.cpu().numpy(), ref[f"train_sorted__{j}__{k}"])


def test_prefetcher_order_and_content(corpus):
    from fs2amd.pipeline import Dataset, Prefetcher, to_device

    pc, mc, tc = _cfg(corpus)
    ds = Dataset("train.txt", pc, mc, tc, sort=True)
    loader = torch.utils.data.DataLoader(ds, batch_size=8, shuffle=False, collate_fn=ds.collate_fn)
    expect = [to_device(b, "cpu") for item in loader for b in item]
    got = list(Prefetcher(loader, DEV, depth=2))
    assert len(got) == len(expect)
    for g, e in zip(got, expect):
        assert g[0] == e[0]
        for a, b in zip(g, e):
            if torch.is_tensor(a):
                assert torch.equal(a.cpu(), b)


def test_positional_equals_keyword_call(corpus):
    from fs2amd.model import FastSpeech2
    from fs2amd.pipeline import Dataset, TextDataset, to_device

    pc, mc, tc = _cfg(corpus)
    m = FastSpeech2(pc, mc)
    m.load_state_dict(oracle_state_dict())
    m = m.to(DEV).eval().set_precision("fp32")
    ds = Dataset("val.txt", pc, mc, tc, sort=True)
    b = to_device(ds.collate_fn([ds[i] for i in range(len(ds))])[0], DEV)
    names = ["speakers", "emotions", "arousals", "valences", "texts", "src_lens", "max_src_len", "mels", "mel_lens",
             "max_mel_len", "p_targets", "e_targets", "d_targets"]
    with torch.no_grad():
        pos = m(*(b[2:]))  # train.py:82 / evaluate.py:43 form (13 positional)
        kw = m(**dict(zip(names, b[2:])))
    for a, c in zip(pos, kw):
        if torch.is_tensor(a):
            assert torch.equal(a, c)
    td = TextDataset(os.path.join(corpus, "val.txt"), pc, mc)
    tb = to_device(td.collate_fn([td[i] for i in range(len(td))]), DEV)
    with torch.no_grad():
        out = m(*(tb[2:]), p_control=1.0, e_control=1.0, d_control=1.0)  # synthesize_chinese_pinyin.py:140-145
    assert out[0].shape[0] == len(td) and out[0].shape[1] == int(out[9].max())
