"""Host input pipeline: the reference's batch assembly and H2D hand-off, built to keep GPUs fed.

Drop-in for (same names, arguments, tuple layouts and error behaviour):

* ``Dataset`` — ``dataset_chinese.py:14-190``: metadata ``train.txt`` / ``val.txt`` lines
  ``name|speaker|{phones}|raw_text|...|emotion|arousal|valence``, per-utterance
  ``<preprocessed_path>/{mel,pitch,energy,duration}/<speaker>-<kind>-<name>.npy``, utterances
  longer than ``max_seq_len`` frames dropped, ``collate_fn`` (optionally length-sorted groups of
  ``batch_size``, tail kept unless ``drop_last``) -> list of 15-tuples (``reprocess``,
  ``:127-169``);
* ``TextDataset`` — ``dataset_chinese.py:193-276``: the 9-tuple synthesis batch;
* ``pad_1D`` / ``pad_2D`` — ``utils/tools.py:323-357``;
* ``to_device`` — ``utils/tools.py:18-127``: the 6-, 9-, 12- and 15-tuple forms, same dtypes.

What is MI355X-native about it: ``to_device`` to a ROCm device packs every array of the batch into
ONE pinned host staging buffer and issues ONE asynchronous host->device copy (the reference issues
a pageable, synchronous ``.to(device)`` per array: 6-11 small DMAs per batch); the device tensors
are typed views of one device buffer. :class:`Prefetcher` runs the collate + pack + copy of the
next batches on a worker thread and a side copy stream (double-buffered pinned slots, HIP events),
so the host pipeline and the H2D copy overlap the model's kernels.

The phoneme vocabulary is the reference's pinyin symbol table (``text/symbols_pinyin.py:1-27``):
pad, '-', 10 punctuation marks, 52 ASCII letters, 44 pinyin phonemes; where a phoneme spells the
same string as a letter the later (phoneme) id wins, exactly as the reference's dict comprehension
resolves it (``'a' -> 64``).
"""
import json
import os
import string
import threading
import queue

import numpy as np
import torch

PINYIN_PHONEMES = ("a ai ao b c ch d e ei er f g h i ia iao ie iu j k l m n ng o ou p q r s sh spn t u ua uai ue "
                   "ui uo w x y z zh").split()
SYMBOLS = ["_", "-"] + list("!'(),.:;? ") + list(string.ascii_uppercase + string.ascii_lowercase) + PINYIN_PHONEMES
SYMBOL_TO_ID = {}
for _i, _s in enumerate(SYMBOLS):  # later entries overwrite earlier ones (dict comprehension semantics)
    SYMBOL_TO_ID[_s] = _i


def phones_to_ids(text):
    """``{b ie z o ng}`` -> int64 ids; symbols missing from the table are skipped (ref :49-57)."""
    body = text.strip("{}")
    if not body.strip():
        return np.array([])
    return np.array([SYMBOL_TO_ID[p] for p in body.split() if p in SYMBOL_TO_ID])


# ------------------------------------------------------------------ synthesis text front-end
# synthesize_chinese_pinyin.py:24-130. Initials are tried two-letter first (zh ch sh), then one
# letter, in the reference's order; every initial maps to itself. Finals map to 1-2 phonemes; a
# final outside the table is spelled character by character, each character through the same
# table when it is a one-letter final and kept as-is otherwise.
_INITIALS_2 = ("zh", "ch", "sh")
_INITIALS_1 = tuple("bpmfdtnlgkhjqxrzcsyw")
_FINALS = {
    "v": "y", "ve": "ue", "vn": "y n",
    "an": "a n", "en": "e n", "in": "i n", "un": "u n",
    "ang": "a ng", "eng": "e ng", "ing": "i ng", "ong": "o ng",
    "ian": "ia n", "iang": "ia ng", "iong": "io ng", "uan": "ua n", "uang": "ua ng",
}
for _f in ("a", "o", "e", "i", "u", "ai", "ei", "ui", "ao", "ou", "iu", "ie", "ue", "er", "iao", "uai"):
    _FINALS[_f] = _f


def pinyin_to_phonemes(py):
    """One toneless pinyin syllable -> phoneme list (synthesize_chinese_pinyin.py:34-96)."""
    initial = next((i for i in _INITIALS_2 if py.startswith(i)), "") or \
        next((i for i in _INITIALS_1 if py.startswith(i)), "")
    final = py[len(initial):]
    out = [initial] if initial else []
    if final in _FINALS:
        out += _FINALS[final].split()
    else:
        for ch in final:
            out += _FINALS[ch].split() if ch in _FINALS else [ch]
    return out


def chinese_to_pinyin_phonemes(text, lazy_pinyin=None):
    """Chinese characters -> phonemes (synthesize_chinese_pinyin.py:24-104). The syllables come from
    ``pypinyin.lazy_pinyin(text, style=Style.NORMAL)`` (:29); pypinyin is not part of this image,
    so pass ``lazy_pinyin`` (text -> list of toneless syllables) or install pypinyin. That one call
    is parity-unpinned here; the syllable -> phoneme rules are tested."""
    if lazy_pinyin is None:
        try:
            import pypinyin
        except ImportError as e:
            raise ImportError("chinese_to_pinyin_phonemes needs pypinyin (or a lazy_pinyin callable) "
                              "for character text; pass phonemes as '{...}' instead") from e
        syllables = pypinyin.lazy_pinyin(text, style=pypinyin.Style.NORMAL)
    else:
        syllables = lazy_pinyin(text)
    return [p for py in syllables for p in pinyin_to_phonemes(py)]


def preprocess_chinese_text(text, preprocess_config=None, lazy_pinyin=None):
    """synthesize_chinese_pinyin.py:106-130: ``{...}`` is a phoneme string (split on whitespace),
    anything else goes through the pinyin rules; a phoneme missing from the symbol table becomes
    the pad id ``'_'`` (0) — unlike ``Dataset``, which drops it (dataset_chinese.py:55)."""
    if text.startswith("{") and text.endswith("}"):
        phonemes = text[1:-1].split()
    else:
        phonemes = chinese_to_pinyin_phonemes(text, lazy_pinyin)
    return np.array([SYMBOL_TO_ID.get(p, SYMBOL_TO_ID["_"]) for p in phonemes])


# ------------------------------------------------------------------ padding (utils/tools.py:323-357)
def pad_1D(inputs, PAD=0):
    """Stack 1-D arrays zero-padded (or PAD-padded) to the longest one."""
    max_len = max(len(x) for x in inputs)
    dtype = np.result_type(*[np.asarray(x).dtype for x in inputs])
    out = np.full((len(inputs), max_len), PAD, dtype=dtype)
    for i, x in enumerate(inputs):
        out[i, :len(x)] = x
    return out


def pad_2D(inputs, maxlen=None):
    """Stack [T_i, C] arrays zero-padded along T to ``maxlen`` (default: the longest); a longer
    input raises ValueError("not max_len") like the reference."""
    max_len = maxlen if maxlen else max(np.shape(x)[0] for x in inputs)
    C = np.shape(inputs[0])[1]
    dtype = np.result_type(*[np.asarray(x).dtype for x in inputs])
    out = np.zeros((len(inputs), max_len, C), dtype=dtype)
    for i, x in enumerate(inputs):
        if np.shape(x)[0] > max_len:
            raise ValueError("not max_len")
        out[i, :np.shape(x)[0]] = x
    return out


# ------------------------------------------------------------------ datasets
def _read_meta(path, preprocessed_path, max_seq_len):
    """process_meta (dataset_chinese.py:104-125 / :237-258): keep utterances whose mel has at most
    max_seq_len frames (the mel header is read through a memory map, not the whole array)."""
    name, speaker, text, raw_text, aux = [], [], [], [], []
    with open(path, "r", encoding="utf-8") as f:
        for line in f.readlines():
            parts = line.strip("\n").split("|")
            n, s, t, r = parts[:4]
            mel = np.load(os.path.join(preprocessed_path, "mel", f"{s}-mel-{n}.npy"), mmap_mode="r")
            if mel.shape[0] > max_seq_len:
                continue
            name.append(n)
            speaker.append(s)
            text.append(t)
            raw_text.append(r)
            aux.append("|".join(parts[4:]))
    return name, speaker, text, raw_text, aux


class _Maps:
    def _load_maps(self, preprocessed_path):
        with open(os.path.join(preprocessed_path, "speakers.json")) as f:
            self.speaker_map = json.load(f)
        with open(os.path.join(preprocessed_path, "emotions.json")) as f:
            raw = json.load(f)
        self.emotion_map, self.arousal_map, self.valence_map = raw["emotion_dict"], raw["arousal_dict"], raw["valence_dict"]

    def _labels(self, idx):
        aux = self.aux_data[idx].split("|")
        return (self.speaker_map[self.speaker[idx]], self.emotion_map[aux[-3]], self.arousal_map[aux[-2]],
                self.valence_map[aux[-1]])


class Dataset(torch.utils.data.Dataset, _Maps):
    """dataset_chinese.py:14-190 (training / validation batches, 15-tuples)."""

    def __init__(self, filename, preprocess_config, model_config, train_config, sort=False, drop_last=False):
        self.dataset_name = preprocess_config["dataset"]
        self.preprocessed_path = preprocess_config["path"]["preprocessed_path"]
        self.cleaners = preprocess_config["preprocessing"]["text"]["text_cleaners"]
        self.max_seq_len = model_config["max_seq_len"]
        self.batch_size = train_config["optimizer"]["batch_size"]
        self.basename, self.speaker, self.text, self.raw_text, self.aux_data = _read_meta(
            os.path.join(self.preprocessed_path, filename), self.preprocessed_path, self.max_seq_len)
        self._load_maps(self.preprocessed_path)
        self.sort = sort
        self.drop_last = drop_last

    def __len__(self):
        return len(self.text)

    def _npy(self, kind, idx):
        s, n = self.speaker[idx], self.basename[idx]
        return np.load(os.path.join(self.preprocessed_path, kind, f"{s}-{kind}-{n}.npy"))

    def __getitem__(self, idx):
        spk, emo, aro, val = self._labels(idx)
        return {"id": self.basename[idx], "speaker": spk, "emotion": emo, "arousal": aro, "valence": val,
                "text": phones_to_ids(self.text[idx]), "raw_text": self.raw_text[idx], "mel": self._npy("mel", idx),
                "pitch": self._npy("pitch", idx), "energy": self._npy("energy", idx),
                "duration": self._npy("duration", idx)}

    def reprocess(self, data, idxs):
        """One 15-tuple (dataset_chinese.py:127-169)."""
        d = [data[i] for i in idxs]
        text_lens = np.array([x["text"].shape[0] for x in d])
        mel_lens = np.array([x["mel"].shape[0] for x in d])
        return ([x["id"] for x in d], [x["raw_text"] for x in d], np.array([x["speaker"] for x in d]),
                np.array([x["emotion"] for x in d]), np.array([x["arousal"] for x in d]),
                np.array([x["valence"] for x in d]), pad_1D([x["text"] for x in d]), text_lens, max(text_lens),
                pad_2D([x["mel"] for x in d]), mel_lens, max(mel_lens), pad_1D([x["pitch"] for x in d]),
                pad_1D([x["energy"] for x in d]), pad_1D([x["duration"] for x in d]))

    def collate_fn(self, data):
        """Groups of batch_size (by descending phoneme count when sort), tail group kept unless
        drop_last (dataset_chinese.py:171-190)."""
        n = len(data)
        if self.sort:
            order = np.argsort(-np.array([x["text"].shape[0] for x in data]))
        else:
            order = np.arange(n)
        cut = n - n % self.batch_size
        groups = order[:cut].reshape((-1, self.batch_size)).tolist()
        if not self.drop_last and n > cut:
            groups.append(order[cut:].tolist())
        return [self.reprocess(data, g) for g in groups]


class TextDataset(torch.utils.data.Dataset, _Maps):
    """dataset_chinese.py:193-276 (synthesis batches, 9-tuples)."""

    def __init__(self, filepath, preprocess_config, model_config):
        self.cleaners = preprocess_config["preprocessing"]["text"]["text_cleaners"]
        self.preprocessed_path = preprocess_config["path"]["preprocessed_path"]
        self.max_seq_len = model_config["max_seq_len"]
        self.basename, self.speaker, self.text, self.raw_text, self.aux_data = _read_meta(
            filepath, self.preprocessed_path, self.max_seq_len)
        self._load_maps(self.preprocessed_path)

    def __len__(self):
        return len(self.text)

    def __getitem__(self, idx):
        spk, emo, aro, val = self._labels(idx)
        return (self.basename[idx], spk, emo, aro, val, phones_to_ids(self.text[idx]), self.raw_text[idx])

    def collate_fn(self, data):
        texts = [d[5] for d in data]
        text_lens = np.array([t.shape[0] for t in texts])
        return ([d[0] for d in data], [d[6] for d in data], np.array([d[1] for d in data]),
                np.array([d[2] for d in data]), np.array([d[3] for d in data]), np.array([d[4] for d in data]),
                pad_1D(texts), text_lens, max(text_lens))


# ------------------------------------------------------------------ H2D (utils/tools.py:18-127)
# Per tuple form: the positions that become tensors and the dtype the reference casts each to
# (None = keep the numpy dtype: torch.from_numpy without a cast).
_L, _F = torch.int64, torch.float32
_LAYOUT = {
    15: {2: _L, 3: _L, 4: _L, 5: _L, 6: _L, 7: None, 9: _F, 10: None, 12: _F, 13: None, 14: _L},
    12: {2: _L, 3: _L, 4: None, 6: _F, 7: None, 9: _F, 10: None, 11: _L},
    9: {2: _L, 3: _L, 4: _L, 5: _L, 6: _L, 7: None},
    6: {2: _L, 3: _L, 4: None},
}
_NP = {torch.int64: np.int64, torch.float32: np.float32}


def _cast(a, dt):
    a = np.asarray(a)
    return a if dt is None else a.astype(_NP[dt], copy=False)


class _Staging:
    """Pinned host slots (grown on demand); slot i is reused only after its last copy finished."""

    def __init__(self, n_slots=2):
        self.bufs = [None] * n_slots
        self.events = [None] * n_slots
        self.i = 0

    def take(self, nbytes):
        i = self.i
        self.i = (self.i + 1) % len(self.bufs)
        if self.events[i] is not None:
            self.events[i].synchronize()
        if self.bufs[i] is None or self.bufs[i].numel() < nbytes:
            self.bufs[i] = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, pin_memory=True)
        return i, self.bufs[i]


_staging = {}
_staging_lock = threading.Lock()


def to_device(data, device):
    """utils/tools.py:18-127 for the 15-, 12-, 9- and 6-tuple batches (anything else: None, like
    the reference). On a ROCm device: one pinned staging buffer, one async H2D copy on the
    current stream, typed views of one device buffer."""
    layout = _LAYOUT.get(len(data))
    if layout is None:
        return None
    device = torch.device(device)
    arrays = {i: _cast(data[i], dt) for i, dt in layout.items()}
    out = list(data)
    if device.type != "cuda":
        for i, a in arrays.items():
            out[i] = torch.from_numpy(np.ascontiguousarray(a)).to(device)
        return tuple(out)
    offs, total = {}, 0
    for i, a in arrays.items():
        offs[i] = total
        total += (a.nbytes + 255) // 256 * 256  # 256 B aligned views
    with _staging_lock:
        st = _staging.setdefault(device.index, _Staging())
        slot, host = st.take(total)
        hv = host.numpy()
        for i, a in arrays.items():
            hv[offs[i]:offs[i] + a.nbytes] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
        dev = torch.empty(max(total, 1), dtype=torch.uint8, device=device)
        dev.copy_(host[:total], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        st.events[slot] = ev
    for i, a in arrays.items():
        t = torch.from_numpy(np.empty(0, dtype=a.dtype)).dtype
        out[i] = dev[offs[i]:offs[i] + a.nbytes].view(t).view(a.shape)
    return tuple(out)


class Prefetcher:
    """Iterate ``loader`` (a DataLoader whose collate_fn returns a batch or a list of batches) on a
    worker thread: each batch is collated, packed and copied to ``device`` on a side copy stream
    up to ``depth`` batches ahead; iteration yields device batches whose copies the consumer's
    current stream has already been made to wait for (no host sync)."""

    _END = object()

    def __init__(self, loader, device, depth=2):
        self.loader, self.device, self.depth = loader, torch.device(device), depth

    def __iter__(self):
        q = queue.Queue(maxsize=self.depth)
        dev = self.device
        stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None

        def work():
            try:
                for item in self.loader:
                    for b in (item if isinstance(item, list) else [item]):
                        if stream is None:
                            q.put((to_device(b, dev), None))
                            continue
                        with torch.cuda.stream(stream):
                            db = to_device(b, dev)
                            ev = torch.cuda.Event()
                            ev.record(stream)
                        q.put((db, ev))
            except BaseException as e:  # surfaced in the consumer
                q.put((e, "error"))
            q.put((self._END, None))

        th = threading.Thread(target=work, daemon=True)
        th.start()
        while True:
            b, ev = q.get()
            if b is self._END:
                break
            if ev == "error":
                raise b
            if ev is not None:
                torch.cuda.current_stream(dev).wait_event(ev)
                for t in b:
                    if torch.is_tensor(t):
                        t.record_stream(torch.cuda.current_stream(dev))
            yield b
        th.join()


def write_synthetic_corpus(directory, n_utts=24, seed=0, L_range=(3, 40), d_range=(1, 12), long_every=0,
                           max_seq_len=2000):
    """A deterministic ESD-shaped preprocessed corpus (test / bench input, same file layout as
    preprocessor/preprocessor.py:183-205,300-317 writes): side files, train.txt / val.txt and
    per-utterance mel [T, 80] f32, phoneme-level pitch / energy [L] f32 and duration [L] int64
    (sum = T). ``long_every`` > 0 makes every n-th utterance longer than max_seq_len frames."""
    from .config import SYNTH_EMOTIONS, SYNTH_SPEAKERS, write_side_files

    write_side_files(directory)
    rng = np.random.default_rng(seed)
    for kind in ("mel", "pitch", "energy", "duration"):
        os.makedirs(os.path.join(directory, kind), exist_ok=True)
    speakers = list(SYNTH_SPEAKERS)
    emos, aros, vals = (list(SYNTH_EMOTIONS[k]) for k in ("emotion_dict", "arousal_dict", "valence_dict"))
    lines = []
    for u in range(n_utts):
        L = int(rng.integers(L_range[0], L_range[1] + 1))
        phones = [PINYIN_PHONEMES[j] for j in rng.integers(0, len(PINYIN_PHONEMES), L)]
        if u % 7 == 3:
            phones.insert(1, "xx")  # a symbol outside the table: skipped by the id mapping
        dur = rng.integers(d_range[0], d_range[1] + 1, len([p for p in phones if p in SYMBOL_TO_ID])).astype(np.int64)
        if long_every and u % long_every == long_every - 1:
            dur[0] += max_seq_len
        T = int(dur.sum())
        spk, name = speakers[u % len(speakers)], f"utt{u:04d}"
        np.save(os.path.join(directory, "mel", f"{spk}-mel-{name}.npy"), rng.standard_normal((T, 80)).astype(np.float32))
        np.save(os.path.join(directory, "pitch", f"{spk}-pitch-{name}.npy"),
                rng.standard_normal(len(dur)).astype(np.float32))
        np.save(os.path.join(directory, "energy", f"{spk}-energy-{name}.npy"),
                rng.standard_normal(len(dur)).astype(np.float32))
        np.save(os.path.join(directory, "duration", f"{spk}-duration-{name}.npy"), dur)
        lines.append(f"{name}|{spk}|{{{' '.join(phones)}}}|raw {u}|{emos[u % 5]}|{aros[u % 4]}|{vals[(u * 3) % 5]}")
    with open(os.path.join(directory, "train.txt"), "w", encoding="utf-8") as f:
        f.write("\n".join(lines[: n_utts * 3 // 4]) + "\n")
    with open(os.path.join(directory, "val.txt"), "w", encoding="utf-8") as f:
        f.write("\n".join(lines[n_utts * 3 // 4:]) + "\n")
    return directory
