"""Deterministic, counter-based synthetic weights for the 240-key FastSpeech2 state_dict.

The reference's trained checkpoints are Git-LFS pointers, so every parity
run uses seeded synthetic weights. They are generated from a counter, not from a
stateful RNG, so the GPU box regenerates exactly the weights the golden fixtures were
captured with, without shipping 139 MB of parameters:

    value[name][i] = scale(name) * u(splitmix64(fnv1a64(name) ^ seed_mix + (i+1) * PHI))

where ``u`` maps the top 53 bits to [-1, 1). Keys that the reference constructor computes
itself (``*.position_enc``, ``variance_adaptor.{pitch,energy}_bins``,
``*.num_batches_tracked``) are left alone.
"""
import re

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_PHI = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def fnv1a64(text):
    h = 0xCBF29CE484222325
    for b in text.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix64(x):
    """Vectorised splitmix64 finaliser over a uint64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = x.copy()
        z ^= z >> np.uint64(30)
        z *= _C1
        z ^= z >> np.uint64(27)
        z *= _C2
        z ^= z >> np.uint64(31)
    return z


def uniform(name, n, seed=0):
    """n values in [-1, 1) for parameter ``name`` (float64)."""
    base = np.uint64((fnv1a64(name) ^ (seed * 0xD1B54A32D192ED03)) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        ctr = (np.arange(1, n + 1, dtype=np.uint64) * _PHI) + base
    z = splitmix64(ctr)
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -52) - 1.0


SKIP_SUFFIXES = ("position_enc", "pitch_bins", "energy_bins", "num_batches_tracked")


def _role(name, shape):
    """(kind, scale, offset) for a parameter: value = offset + scale * u."""
    leaf = name.rsplit(".", 1)[-1]
    is_bn = re.fullmatch(r"postnet\.convolutions\.\d+\.1\.\w+", name) is not None
    if "layer_norm" in name or is_bn:
        # LayerNorm / BatchNorm affine and running stats
        if leaf == "weight":
            return 1.0, 0.1
        if leaf == "bias":
            return 0.0, 0.1
        if leaf == "running_mean":
            return 0.0, 0.1
        if leaf == "running_var":
            return 1.0, 0.25
    if name == "variance_adaptor.duration_predictor.linear_layer.bias":
        # log-duration head biased to ~1.2 so free-running synthesis yields ~3-10 frames per
        # phoneme (a zero-duration utterance makes the reference decoder raise).
        return 1.2, 0.05
    if name.endswith("emb.weight") or name.endswith("embedding.weight"):
        return 0.0, float(np.sqrt(3.0))  # unit variance, like nn.Embedding's N(0,1) init
    if leaf == "bias":
        return 0.0, 0.1
    if leaf == "weight":
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else int(shape[0])
        return 0.0, float(np.sqrt(3.0 / fan_in))  # variance 1/fan_in
    raise KeyError(name)


def synth_state_dict(shapes, seed=0):
    """Map {name: shape} -> {name: float32 ndarray} for every generated key."""
    out = {}
    for name, shape in shapes.items():
        if name.endswith(SKIP_SUFFIXES):
            continue
        n = int(np.prod(shape)) if len(shape) else 1
        offset, scale = _role(name, shape)
        v = (offset + scale * uniform(name, n, seed)).astype(np.float32).reshape(shape)
        if name == "encoder.src_word_emb.weight":
            v[0] = 0.0  # padding_idx=0 row stays zero (ref transformer/Models.py:54-56)
        out[name] = v
    return out


def _vocoder_role(name, shape, ups_meta):
    """HiFi-GAN generator keys (hifigan/models.py, weight-normed convs): weight_v uniform with
    variance 1 / (elements per output-channel row), so each row has norm ~1; weight_g (the row
    norm the effective weight gets) ~1 for Conv1d and sqrt(Cout * stride / Cin) for the
    ConvTranspose1d upsamplers, so every layer keeps unit activation variance; biases +-0.05."""
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "bias":
        return 0.0, 0.05
    if leaf == "weight_v" or leaf == "weight":
        row = int(np.prod(shape[1:]))
        return 0.0, float(np.sqrt(3.0 / row))
    if leaf == "weight_g":
        if name.startswith("ups."):
            cin, cout, u = ups_meta[int(name.split(".")[1])]
            return float(np.sqrt(cout * u / cin)), 0.1 * float(np.sqrt(cout * u / cin))
        return 1.0, 0.1
    raise KeyError(name)


def synth_vocoder_state_dict(shapes, ups_meta, seed=0):
    """{name: shape} of a HiFi-GAN Generator -> {name: float32 ndarray} (counter-based, as above).
    ups_meta[i] = (Cin, Cout, stride) of upsampler i."""
    out = {}
    for name, shape in shapes.items():
        n = int(np.prod(shape)) if len(shape) else 1
        offset, scale = _vocoder_role(name, shape, ups_meta)
        out[name] = (offset + scale * uniform("vocoder." + name, n, seed)).astype(np.float32).reshape(shape)
    return out


def fill_vocoder(module, h, seed=0):
    """Overwrite a HiFi-GAN Generator's parameters in place (reference or fs2amd.vocoder)."""
    import torch

    sd = module.state_dict()
    c0 = h["upsample_initial_channel"]
    meta = [(c0 // 2 ** i, c0 // 2 ** (i + 1), u) for i, u in enumerate(h["upsample_rates"])]
    gen = synth_vocoder_state_dict({k: tuple(v.shape) for k, v in sd.items()}, meta, seed)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in gen.items()}, strict=True)
    return module


def fill_module(module, seed=0):
    """Overwrite a torch module's generated parameters/buffers in place (CPU copy)."""
    import torch

    sd = module.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items()}
    gen = synth_state_dict(shapes, seed)
    new = {k: torch.from_numpy(v) for k, v in gen.items()}
    missing = [k for k in sd if k not in new]
    for k in missing:
        new[k] = sd[k]
    module.load_state_dict(new, strict=True)
    return module
