"""Synthetic ESD-shaped phoneme batches in the reference's batch layout.

The reference's callers hand the model ``batch[2:]`` of the 9-tuple text batch
(``synthesize_chinese_pinyin.py:300``: ids, raw_texts, speakers, emotions, arousals,
valences, texts, text_lens, max_text_len) or of the 15-tuple training batch
(``dataset_chinese.py:171-190``, ``train.py:82``). :func:`synth_batch` produces the model
arguments of either form from a seeded ``torch.Generator`` (draw order fixed below):

* src_lens ~ U{L_min..L_max}; texts ~ U{64..107} (pinyin ids, ``text/symbols_pinyin.py``), 0 beyond length
* speakers U{0..9}, emotions U{0..4}, arousals U{0..3}, valences U{0..4}
* durations ~ U{d_lo..d_hi}, 0 beyond length; mel_lens = row sums
* optional pitch/energy targets ~ N(0,1), 0 beyond length; optional mels ~ N(0,1)
"""
import torch


def synth_batch(B, L_min, L_max=None, seed=1, d_range=(2, 10), teacher=True, pe_targets=False,
                with_mels=False, n_mels=80):
    L_max = L_min if L_max is None else L_max
    g = torch.Generator().manual_seed(seed)
    src_lens = torch.randint(L_min, L_max + 1, (B,), generator=g, dtype=torch.int64)
    max_src_len = int(src_lens.max())
    pos = torch.arange(max_src_len).unsqueeze(0)
    valid = pos < src_lens.unsqueeze(1)
    texts = torch.randint(64, 108, (B, max_src_len), generator=g, dtype=torch.int64) * valid
    speakers = torch.randint(0, 10, (B,), generator=g, dtype=torch.int64)
    emotions = torch.randint(0, 5, (B,), generator=g, dtype=torch.int64)
    arousals = torch.randint(0, 4, (B,), generator=g, dtype=torch.int64)
    valences = torch.randint(0, 5, (B,), generator=g, dtype=torch.int64)
    durations = torch.randint(d_range[0], d_range[1] + 1, (B, max_src_len), generator=g, dtype=torch.int64) * valid
    p_t = torch.randn(B, max_src_len, generator=g) * valid
    e_t = torch.randn(B, max_src_len, generator=g) * valid
    mel_lens = durations.sum(1)
    max_mel_len = int(mel_lens.max())
    mels = torch.randn(B, max_mel_len, n_mels, generator=g) if with_mels else None
    args = dict(speakers=speakers, emotions=emotions, arousals=arousals, valences=valences, texts=texts,
                src_lens=src_lens, max_src_len=max_src_len)
    if teacher:
        args.update(mels=mels, mel_lens=mel_lens, max_mel_len=max_mel_len, d_targets=durations)
        if pe_targets:
            args.update(p_targets=p_t, e_targets=e_t)
    return args


def loss_inputs(args):
    """The reference batch tuple as FastSpeech2Loss indexes it (``inputs[9:]`` = mels, mel_lens,
    max_mel_len, pitches, energies, durations; dataset_chinese.py collate order)."""
    return (None,) * 9 + (args["mels"], args["mel_lens"], args["max_mel_len"], args["p_targets"],
                          args["e_targets"], args["d_targets"])


def to_device(args, device):
    return {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in args.items()}


def shard(args, rank, world):
    """Contiguous split of a batch along B for one-process-per-GPU inference.

    Each shard is re-padded to its own maxima (max_src_len / max_mel_len), which is what
    the reference would see if called per shard (padding classes)."""
    B = args["texts"].shape[0]
    per = (B + world - 1) // world
    lo, hi = min(rank * per, B), min((rank + 1) * per, B)
    out = {}
    for k, v in args.items():
        out[k] = v[lo:hi] if torch.is_tensor(v) and v.dim() >= 1 and v.shape[0] == B else v
    if hi > lo:
        L = int(out["src_lens"].max())
        out["max_src_len"] = L
        for k in ("texts", "d_targets", "p_targets", "e_targets"):
            if out.get(k) is not None:
                out[k] = out[k][:, :L]
        if out.get("mel_lens") is not None:
            T = int(out["mel_lens"].max())
            out["max_mel_len"] = T
            if out.get("mels") is not None:
                out["mels"] = out["mels"][:, :T]
    return out
