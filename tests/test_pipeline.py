"""Host input pipeline (fs2amd.pipeline) against the reference's own batch assembly.

tests/golden/pipeline_batches.npz holds what the reference's dataset_chinese.Dataset /
TextDataset collate_fn + utils.tools.to_device produced (CPU) over the deterministic synthetic
corpus write_synthetic_corpus(dir, 24, seed=0, long_every=11): every array of every tuple must be
EQUAL (values, shapes, dtypes) — this is integer / copy work, so bit-exact.
"""
import os

import numpy as np
import pytest
import torch

from _common import GOLDEN, configs


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    from fs2amd.pipeline import write_synthetic_corpus

    return write_synthetic_corpus(str(tmp_path_factory.mktemp("corpus")), 24, seed=0, long_every=11, max_seq_len=2000)


@pytest.fixture(scope="module")
def ref():
    return np.load(os.path.join(GOLDEN, "pipeline_batches.npz"))


def _cfg(corpus):
    from fs2amd import config as C

    pc, mc, tc = configs()
    pc = dict(pc, path={"preprocessed_path": corpus})
    return pc, mc, C.ESD_TRAIN_CONFIG


def _check(tag, got, ref):
    for k, v in enumerate(got):
        r = ref[f"{tag}__{k}"]
        if torch.is_tensor(v):
            assert str(v.dtype) == str(ref[f"{tag}__{k}__dtype"]), (tag, k)
            v = v.cpu().numpy()
        v = np.asarray(v)
        assert v.shape == r.shape, (tag, k, v.shape, r.shape)
        np.testing.assert_array_equal(v, r, err_msg=f"{tag} field {k}")


@pytest.mark.parametrize("tag,fname,sort,drop", [("train_sorted", "train.txt", True, False),
                                                 ("train_drop", "train.txt", True, True),
                                                 ("val_plain", "val.txt", False, False)])
def test_dataset_collate_matches_reference(corpus, ref, tag, fname, sort, drop):
    from fs2amd.pipeline import Dataset, to_device

    pc, mc, tc = _cfg(corpus)
    ds = Dataset(fname, pc, mc, tc, sort=sort, drop_last=drop)
    batches = ds.collate_fn([ds[i] for i in range(len(ds))])
    assert len(batches) == int(ref[f"{tag}__n"])
    for j, b in enumerate(batches):
        assert len(b) == 15
        _check(f"{tag}__{j}", to_device(b, "cpu"), ref)


def test_text_dataset_collate_matches_reference(corpus, ref):
    from fs2amd.pipeline import TextDataset, to_device

    pc, mc, _ = _cfg(corpus)
    td = TextDataset(os.path.join(corpus, "val.txt"), pc, mc)
    b = to_device(td.collate_fn([td[i] for i in range(len(td))]), "cpu")
    assert len(b) == 9
    _check("text", b, ref)


def test_long_utterances_are_dropped(corpus):
    """process_meta drops mels longer than max_seq_len (long_every=11 made utt0010 / utt0021)."""
    from fs2amd.pipeline import Dataset

    pc, mc, tc = _cfg(corpus)
    ds = Dataset("train.txt", pc, mc, tc)
    assert "utt0010" not in ds.basename and len(ds) == 17


def test_symbol_table():
    """text/symbols_pinyin.py: 108 symbols; phonemes spelled like letters take the later id."""
    from fs2amd.pipeline import SYMBOLS, SYMBOL_TO_ID, phones_to_ids

    assert len(SYMBOLS) == 108 and SYMBOL_TO_ID["_"] == 0 and SYMBOL_TO_ID["a"] == 64
    assert SYMBOL_TO_ID["zh"] == 107 and SYMBOL_TO_ID["A"] == 12 and SYMBOL_TO_ID["v"] == 59
    np.testing.assert_array_equal(phones_to_ids("{b ie xx z o ng}"), [67, 80, 106, 88, 87])
    assert phones_to_ids("{}").shape == (0,)


@pytest.mark.parametrize("py,phones", [
    ("zhang", ["zh", "a", "ng"]), ("shi", ["sh", "i"]), ("xue", ["x", "ue"]), ("lv", ["l", "y"]),
    ("lve", ["l", "ue"]), ("yuan", ["y", "ua", "n"]), ("er", ["er"]), ("a", ["a"]),
    ("duo", ["d", "u", "o"]),  # final 'uo' not in the table: spelled per character
    ("jiong", ["j", "io", "ng"]), ("ng", ["n", "g"]), ("hm", ["h", "m"]), ("chuang", ["ch", "ua", "ng"]),
    ("wen", ["w", "e", "n"]), ("qvn", ["q", "y", "n"]), ("", [])])
def test_pinyin_rules(py, phones):
    """synthesize_chinese_pinyin.py:34-96, expected lists derived by hand from its rule table
    (the script imports pypinyin at module level, which this image lacks, so it is not run)."""
    from fs2amd.pipeline import pinyin_to_phonemes

    assert pinyin_to_phonemes(py) == phones


def test_preprocess_chinese_text():
    """synthesize_chinese_pinyin.py:106-130: '{...}' phoneme strings, unknown phonemes -> '_' (0),
    character text through lazy_pinyin (parity-unpinned: pypinyin absent; a stub stands in)."""
    from fs2amd.pipeline import SYMBOL_TO_ID as S, preprocess_chinese_text

    np.testing.assert_array_equal(preprocess_chinese_text("{b ie xx z o ng}"), [67, 80, 0, 106, 88, 87])
    assert preprocess_chinese_text("{}").shape == (0,)
    # only a string wrapped on both sides is a phoneme string
    got = preprocess_chinese_text("{b a", lazy_pinyin=lambda t: ["ba"])
    np.testing.assert_array_equal(got, [S["b"], S["a"]])
    got = preprocess_chinese_text("你好", lazy_pinyin=lambda t: ["ni", "hao", "xx1"])
    np.testing.assert_array_equal(got, [S["n"], S["i"], S["h"], S["ao"], S["x"], S["x"], 0])
    try:
        import pypinyin  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            preprocess_chinese_text("你好")


def test_pad_helpers():
    from fs2amd.pipeline import pad_1D, pad_2D

    a = pad_1D([np.array([1, 2, 3]), np.array([4])])
    np.testing.assert_array_equal(a, [[1, 2, 3], [4, 0, 0]])
    b = pad_2D([np.ones((2, 3)), np.ones((4, 3))], maxlen=5)
    assert b.shape == (2, 5, 3) and b[0, 2:].sum() == 0
    with pytest.raises(ValueError):
        pad_2D([np.ones((6, 3))], maxlen=5)


def test_positional_call_dry_run(corpus, monkeypatch):
    """The reference's callers hand the model batch[2:] positionally (train.py:82: 13 args;
    synthesize_chinese_pinyin.py:140-145: 7 args): the drop-in forward takes both tuple forms
    (kernels stubbed, CPU)."""
    from fs2amd import ops, runtime, _lib
    from fs2amd.model import FastSpeech2
    from fs2amd.pipeline import Dataset, TextDataset, to_device
    from test_host import _FakeForkJoin, _RecordingLib, stub_seq_layout
    from _common import oracle_state_dict

    stub_seq_layout(monkeypatch, ops)
    rec = _RecordingLib(_lib.load())
    monkeypatch.setattr(ops, "_lib", rec)
    monkeypatch.setattr(ops, "_gpu", lambda *a: None)
    monkeypatch.setattr(ops, "_stream", lambda *a: None)
    monkeypatch.setattr(runtime, "_device_ok", lambda dev: True)
    monkeypatch.setattr(runtime, "_ForkJoin", _FakeForkJoin)
    pc, mc, tc = _cfg(corpus)
    m = FastSpeech2(pc, mc)
    m.load_state_dict(oracle_state_dict())
    m.eval()
    ds = Dataset("val.txt", pc, mc, tc, sort=True)
    b = to_device(ds.collate_fn([ds[i] for i in range(len(ds))])[0], "cpu")
    with torch.no_grad():
        out = m(*(b[2:]))
    assert len(out) == 10 and out[0].shape[:2] == (b[2].shape[0], int(b[11]))
    td = TextDataset(os.path.join(corpus, "val.txt"), pc, mc)
    tb = to_device(td.collate_fn([td[i] for i in range(3)]), "cpu")

    real_lr = ops.lr_durations

    def lr_durations(dur, logpred=False, d_control=1.0):  # the stub kernel writes nothing: size mel_len
        cum, ml, dr = real_lr(dur, logpred, d_control)
        ml.fill_(5)
        return cum, ml, dr

    monkeypatch.setattr(ops, "lr_durations", lr_durations)
    with torch.no_grad():
        out = m(*(tb[2:]), p_control=1.0, e_control=1.0, d_control=1.0)
    assert len(out) == 10 and out[0].shape[0] == 3
