"""Drop-in ``FastSpeech2`` whose forward runs on the fs2hip kernels (MI355X / gfx950).

Same constructor ``FastSpeech2(preprocess_config, model_config)`` (reads
``<preprocessed_path>/{stats,speakers,emotions}.json``), same ``forward`` signature and
10-tuple return, same 240-key ``state_dict`` as the reference (model/fastspeech2.py:13-148),
so ``synthesize_chinese_pinyin.py:140-145`` / ``evaluate.py:43`` call it unchanged and
reference checkpoints load with ``load_state_dict``. The ``nn`` sub-modules below only
HOLD the parameters under the reference's names; the forward never calls them.

Precision: ``model_config["hip"]["dtype"]`` (or env ``FS2_HIP_DTYPE``, or
:meth:`FastSpeech2.set_precision`) selects
* ``"fp32"`` — every GEMM on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32), f32 activations;
  the parity mode (matches the reference CPU path to ~1e-5).
* ``"bf16"`` — FFT blocks, attention, mel_linear and PostNet on bf16 MFMA with f32
  accumulation/LayerNorm. The VariancePredictors default to split-precision ``"bf16x3"``
  (x_hi·w_hi + x_hi·w_lo + x_lo·w_hi on bf16 MFMA, f32 accumulation: their outputs feed discrete
  decisions, duration rounding and pitch/energy buckets, SURVEY.md §0 trap 2);
  ``vp_dtype="fp32"`` selects exact f32, ``"bf16"`` plain bf16.
* ``"fp8"`` — cfg5: bf16 mode with the FFN Conv1d pair (and Q|K|V of blocks 1..n) on e4m3
  MFMA; VariancePredictors as in bf16 mode.
"""
import json
import os
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from .config import N_SRC_VOCAB


def sinusoid_table(n_position, d_hid):
    """Sinusoid position table (numpy fp64 -> f32), transformer/Models.py:10-30."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    hid = np.arange(d_hid)
    tab = pos / np.power(10000, 2 * (hid // 2) / d_hid)
    tab[:, 0::2] = np.sin(tab[:, 0::2])
    tab[:, 1::2] = np.cos(tab[:, 1::2])
    return torch.from_numpy(tab.astype(np.float32))


# ------------------------------------------------------------------ parameter holders
class _MultiHeadAttention(nn.Module):
    def __init__(self, n_head, d_model):
        super().__init__()
        self.n_head, self.d_k = n_head, d_model // n_head
        self.w_qs = nn.Linear(d_model, d_model)
        self.w_ks = nn.Linear(d_model, d_model)
        self.w_vs = nn.Linear(d_model, d_model)
        self.layer_norm = nn.LayerNorm(d_model)
        self.fc = nn.Linear(d_model, d_model)


class _PositionwiseFeedForward(nn.Module):
    def __init__(self, d_in, d_hid, kernel_size):
        super().__init__()
        self.kernel_size = tuple(kernel_size)
        self.w_1 = nn.Conv1d(d_in, d_hid, kernel_size[0], padding=(kernel_size[0] - 1) // 2)
        self.w_2 = nn.Conv1d(d_hid, d_in, kernel_size[1], padding=(kernel_size[1] - 1) // 2)
        self.layer_norm = nn.LayerNorm(d_in)


class _FFTBlock(nn.Module):
    def __init__(self, d_model, n_head, d_inner, kernel_size):
        super().__init__()
        self.slf_attn = _MultiHeadAttention(n_head, d_model)
        self.pos_ffn = _PositionwiseFeedForward(d_model, d_inner, kernel_size)


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        tr = cfg["transformer"]
        d = tr["encoder_hidden"]
        self.max_seq_len, self.d_model, self.n_head = cfg["max_seq_len"], d, tr["encoder_head"]
        self.src_word_emb = nn.Embedding(N_SRC_VOCAB, d, padding_idx=0)
        self.position_enc = nn.Parameter(sinusoid_table(cfg["max_seq_len"] + 1, d).unsqueeze(0), requires_grad=False)
        self.layer_stack = nn.ModuleList(
            [_FFTBlock(d, tr["encoder_head"], tr["conv_filter_size"], tr["conv_kernel_size"])
             for _ in range(tr["encoder_layer"])])


class _Decoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        tr = cfg["transformer"]
        d = tr["decoder_hidden"]
        self.max_seq_len, self.d_model, self.n_head = cfg["max_seq_len"], d, tr["decoder_head"]
        self.position_enc = nn.Parameter(sinusoid_table(cfg["max_seq_len"] + 1, d).unsqueeze(0), requires_grad=False)
        self.layer_stack = nn.ModuleList(
            [_FFTBlock(d, tr["decoder_head"], tr["conv_filter_size"], tr["conv_kernel_size"])
             for _ in range(tr["decoder_layer"])])


class _Conv(nn.Module):
    def __init__(self, cin, cout, kernel_size, padding):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, kernel_size, padding=padding)


class _VariancePredictor(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d_in = cfg["transformer"]["encoder_hidden"]
        f = cfg["variance_predictor"]["filter_size"]
        k = cfg["variance_predictor"]["kernel_size"]
        p = cfg["variance_predictor"]["dropout"]
        self.kernel = k
        self.conv_layer = nn.Sequential(OrderedDict([
            ("conv1d_1", _Conv(d_in, f, k, (k - 1) // 2)), ("relu_1", nn.ReLU()),
            ("layer_norm_1", nn.LayerNorm(f)), ("dropout_1", nn.Dropout(p)),
            ("conv1d_2", _Conv(f, f, k, 1)), ("relu_2", nn.ReLU()),  # padding=1 hard-coded (modules.py:230)
            ("layer_norm_2", nn.LayerNorm(f)), ("dropout_2", nn.Dropout(p)),
        ]))
        self.linear_layer = nn.Linear(f, 1)


class LengthRegulator(nn.Module):
    """Drop-in for the reference ``model.modules.LengthRegulator`` (modules.py:161-194):
    ``forward(x, duration, max_len) -> (output, mel_len)`` on the fs2hip scan + gather kernels."""

    def forward(self, x, duration, max_len):
        from .ops import length_regulate

        return length_regulate(x, duration, max_len)


class _VarianceAdaptor(nn.Module):
    def __init__(self, pcfg, cfg):
        super().__init__()
        self.duration_predictor = _VariancePredictor(cfg)
        self.length_regulator = LengthRegulator()
        self.pitch_predictor = _VariancePredictor(cfg)
        self.energy_predictor = _VariancePredictor(cfg)
        self.pitch_feature_level = pcfg["preprocessing"]["pitch"]["feature"]
        self.energy_feature_level = pcfg["preprocessing"]["energy"]["feature"]
        assert self.pitch_feature_level in ["phoneme_level", "frame_level"]
        assert self.energy_feature_level in ["phoneme_level", "frame_level"]
        ve = cfg["variance_embedding"]
        assert ve["pitch_quantization"] in ["linear", "log"]
        assert ve["energy_quantization"] in ["linear", "log"]
        n_bins = ve["n_bins"]
        with open(os.path.join(pcfg["path"]["preprocessed_path"], "stats.json")) as f:
            stats = json.load(f)
        for kind in ("pitch", "energy"):
            lo, hi = stats[kind][:2]
            if ve[f"{kind}_quantization"] == "log":
                bins = torch.exp(torch.linspace(np.log(lo), np.log(hi), n_bins - 1))
            else:
                bins = torch.linspace(lo, hi, n_bins - 1)
            setattr(self, f"{kind}_bins", nn.Parameter(bins, requires_grad=False))
        d = cfg["transformer"]["encoder_hidden"]
        self.pitch_embedding = nn.Embedding(n_bins, d)
        self.energy_embedding = nn.Embedding(n_bins, d)


class _ConvNorm(nn.Module):
    def __init__(self, cin, cout, k):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, k, padding=(k - 1) // 2)


class _PostNet(nn.Module):
    def __init__(self, n_mel=80, dim=512, k=5, n=5):
        super().__init__()
        chans = [n_mel] + [dim] * (n - 1) + [n_mel]
        self.kernel = k
        self.convolutions = nn.ModuleList(
            [nn.Sequential(_ConvNorm(chans[i], chans[i + 1], k), nn.BatchNorm1d(chans[i + 1])) for i in range(n)])


# ------------------------------------------------------------------ the model
class FastSpeech2(nn.Module):
    """FastSpeech2 (mel-synthesis forward on fs2hip kernels). See module docstring."""

    def __init__(self, preprocess_config, model_config):
        super().__init__()
        self.model_config = model_config
        self.preprocess_config = preprocess_config
        tr = model_config["transformer"]
        self.encoder = _Encoder(model_config)
        self.variance_adaptor = _VarianceAdaptor(preprocess_config, model_config)
        self.decoder = _Decoder(model_config)
        n_mel = preprocess_config["preprocessing"]["mel"]["n_mel_channels"]
        self.mel_linear = nn.Linear(tr["decoder_hidden"], n_mel)
        self.postnet = _PostNet(n_mel=n_mel)
        pp = preprocess_config["path"]["preprocessed_path"]
        self.speaker_emb = None
        if model_config["multi_speaker"]:
            with open(os.path.join(pp, "speakers.json")) as f:
                n_speaker = len(json.load(f))
            self.speaker_emb = nn.Embedding(n_speaker, tr["encoder_hidden"])
        self.emotion_emb = None
        if model_config["multi_emotion"]:
            with open(os.path.join(pp, "emotions.json")) as f:
                raw = json.load(f)
            d = tr["encoder_hidden"]
            self.emotion_emb = nn.Embedding(len(raw["emotion_dict"]), d // 2)
            self.arousal_emb = nn.Embedding(len(raw["arousal_dict"]), d // 4)
            self.valence_emb = nn.Embedding(len(raw["valence_dict"]), d // 4)
            self.emotion_linear = nn.Sequential(nn.Linear(d, d), nn.ReLU())
        hip = model_config.get("hip", {}) if isinstance(model_config, dict) else {}
        self._precision = hip.get("dtype", os.environ.get("FS2_HIP_DTYPE", "fp32"))
        # VariancePredictors in bf16 / fp8 mode: split-precision bf16x3 (same discrete decisions as
        # exact f32 on the cfg2 flip-rate sample, tools/flip_rate.py); "fp32" / "bf16" selectable
        self._vp_precision = hip.get("vp_dtype", os.environ.get("FS2_HIP_VP_DTYPE", "bf16x3"))
        self._packs = {}
        self.train_dropout = True  # False: train-mode semantics without dropout (parity tests)
        self._fp8_scales = None    # {("enc"|"dec", layer): {"x": amax block input, "h": FFN input, "f": w_1 out}}
        self.register_load_state_dict_post_hook(lambda mod, keys: mod.invalidate_packed())

    # ---- precision / packed weights --------------------------------------------------------------
    def set_precision(self, dtype, vp_dtype=None):
        """dtype of the FFT blocks / attention / mel_linear / PostNet ('fp32' | 'bf16' | 'fp8'); vp_dtype
        of the three VariancePredictors ('bf16x3' default | 'fp32' exact | 'bf16'; the bf16 forms only
        take effect in bf16 / fp8 mode, fp32 mode always runs them exact f32)."""
        if dtype not in ("fp32", "bf16", "fp8") or vp_dtype not in (None, "fp32", "bf16", "bf16x3"):
            raise ValueError("precision must be 'fp32', 'bf16' or 'fp8' (vp_dtype 'fp32' / 'bf16' / 'bf16x3')")
        self._precision = dtype
        if vp_dtype is not None:
            self._vp_precision = vp_dtype
        return self

    @property
    def precision(self):
        return self._precision

    def calibrate_fp8(self, **batch):
        """Static fp8 activation scales (cfg5): one bf16 forward on ``batch`` records, per FFT
        block, max|x| (block input, the Q|K|V GEMM's), max|h| (input of the FFN Conv1d k=9) and
        max|relu(w_1 h)| (input of w_2) over the valid frames; fp8 packing derives s = amax / 448
        from them. Returns the scales."""
        from . import runtime

        prev = self._precision
        self._precision = "bf16"
        runtime.CALIB = {}
        try:
            with torch.no_grad():
                self.forward(**batch)
            self._fp8_scales = {k: dict(v) for k, v in runtime.CALIB.items()}
        finally:
            runtime.CALIB = None
            self._precision = prev
        return self._fp8_scales

    def invalidate_packed(self):
        self._packs = {}

    def _replicate_for_data_parallel(self):
        # nn.DataParallel (reference train.py:42) shallow-copies __dict__ into each replica; a shared
        # _packs dict would let replicas reuse weights packed before later optimizer steps (their
        # broadcast parameters all carry the same _version sum). Each replica packs its own.
        replica = super()._replicate_for_data_parallel()
        replica._packs = {}
        return replica

    def _fingerprint(self):
        return sum(p._version for p in self.parameters()) + sum(b._version for b in self.buffers())

    def packed(self, device):
        from .packing import pack_model

        key = (self._precision, self._vp_precision, str(device))
        fp = (self._fingerprint(), id(self._fp8_scales))
        ent = self._packs.get(key)
        if ent is None or ent[0] != fp:
            ent = (fp, pack_model(self, device, self._precision, self._vp_precision, self._fp8_scales))
            self._packs[key] = ent
        return ent[1]

    # ---- forward ---------------------------------------------------------------------------------
    def forward(self, speakers, emotions, arousals, valences, texts, src_lens, max_src_len, mels=None, mel_lens=None,
                max_mel_len=None, p_targets=None, e_targets=None, d_targets=None, p_control=1.0, e_control=1.0,
                d_control=1.0):
        if self.training:
            # train.py step: dropout, batch-statistic BatchNorm, autograd (fs2amd/training.py)
            from .training import train_forward

            return train_forward(self, speakers, emotions, arousals, valences, texts, src_lens, max_src_len, mels,
                                 mel_lens, max_mel_len, p_targets, e_targets, d_targets, p_control, e_control,
                                 d_control)
        from .runtime import run_forward

        return run_forward(self, speakers, emotions, arousals, valences, texts, src_lens, max_src_len, mels, mel_lens,
                           max_mel_len, p_targets, e_targets, d_targets, p_control, e_control, d_control)
