"""Shared helpers for the test-suite (oracle state dict, golden loading)."""
import functools
import json
import os
import tempfile

import numpy as np
import torch

from fs2amd import config as C
from fs2amd.synth_weights import synth_state_dict

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

GOLDEN_CASES = ["cfg1_teacher", "cfg1_free", "mini_teacher", "mini_targets", "mini_free_ctrl",
                "mini_free_ctrl2", "pad_base", "pad_ph1", "pad_ph2", "pad_ph3", "pad_fr9", "pad_fr10", "pad_fr30"]
OUT_NAMES = ["mel", "postnet_mel", "p_pred", "e_pred", "log_d", "d_rounded", "src_masks", "mel_masks",
             "src_lens_out", "mel_lens_out"]


@functools.lru_cache(maxsize=1)
def manifest():
    with open(os.path.join(GOLDEN, "weights_manifest.json")) as f:
        return json.load(f)


@functools.lru_cache(maxsize=1)
def side_dir():
    return C.write_side_files(tempfile.mkdtemp(prefix="fs2_side_"))


def configs():
    return C.synthetic_configs(side_dir())


@functools.lru_cache(maxsize=1)
def oracle_state_dict():
    from oracle import fs2_oracle as O
    pc, mc, _ = configs()
    shapes = {k: tuple(v["shape"]) for k, v in manifest()["keys"].items()}
    gen = synth_state_dict(shapes, seed=0)
    return O.build_state_dict(mc, pc, C.SYNTH_STATS, gen)


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    args, outs = {}, {}
    for k in z.files:
        if k.startswith("in_"):
            v = z[k]
            args[k[3:]] = int(v) if v.ndim == 0 else torch.from_numpy(v)
        elif k.startswith("out_"):
            outs[k[4:]] = z[k]
    controls = tuple(float(c) for c in z["controls"])
    return args, controls, outs, z


def load_train_case(name="train_grads"):
    """tests/golden/<name>.npz (train_grads: B=4, train_b16: the cfg3 shape B=16, lengths
    U{16..64}): inputs, reference losses, per-parameter gradient sums / sums of squares / 16
    sampled elements, BN running stats after the step."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    args = {}
    for k in z.files:
        if k.startswith("in_"):
            v = z[k]
            args[k[3:]] = int(v) if v.ndim == 0 else torch.from_numpy(v)
    return z, args


def check_train_grads(z, named_grads, rtol, sample_atol_frac):
    """Compare {name: grad} with the reference fixture: per-key sum of squares (relative),
    sum (relative to sqrt(numel)*rms) and sampled elements (to a fraction of the key's rms)."""
    keys = [str(k) for k in z["grad_keys"]]
    assert set(keys) == set(named_grads.keys()), set(keys) ^ set(named_grads.keys())
    # gradients that are analytically zero (attention key biases: softmax ignores a per-row
    # shift) are roundoff noise on both sides: bounded absolutely against the model-wide scale
    rms_all = [(float(z["grad_sumsq"][j]) / named_grads[k].numel()) ** 0.5 for j, k in enumerate(keys)]
    scale = max(rms_all)
    worst = {}
    for j, k in enumerate(keys):
        g = named_grads[k].detach().double().cpu().reshape(-1)
        ss_ref, s_ref = float(z["grad_sumsq"][j]), float(z["grad_sum"][j])
        rms = (ss_ref / g.numel()) ** 0.5
        if rms < 1e-5 * scale:
            assert float(g.abs().max()) <= 1e-4 * scale, (k, float(g.abs().max()), scale)
            continue
        e_ss = abs(float((g * g).sum()) - ss_ref) / ss_ref
        e_s = abs(float(g.sum()) - s_ref) / (rms * g.numel() ** 0.5)
        idx = torch.from_numpy(z[f"gidx_{j}"])
        e_v = float((g[idx] - torch.from_numpy(z[f"gval_{j}"]).double()).abs().max()) / rms
        worst[k] = (e_ss, e_s, e_v)
        assert e_ss <= rtol and e_s <= rtol and e_v <= sample_atol_frac, (k, e_ss, e_s, e_v)
    return worst
