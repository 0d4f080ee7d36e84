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
                "mini_free_ctrl2", "pad_base"]
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
