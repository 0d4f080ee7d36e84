"""HiFi-GAN generator host side (CPU): the state-dict contract, the oracle against the reference
generator's own outputs (tests/golden/vocoder.npz, bit-exact: same ATen ops in the same order),
and the ConvTranspose1d -> phase-conv rewrite the HIP path relies on."""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _common import GOLDEN


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "vocoder.npz"))


def _gen(seed=0):
    from fs2amd.synth_weights import fill_vocoder
    from fs2amd.vocoder import V1_CONFIG, Generator

    g = Generator(V1_CONFIG)
    fill_vocoder(g, V1_CONFIG, seed=seed)
    return g


def test_state_dict_keys_match_reference(golden):
    g = _gen()
    assert list(g.state_dict().keys()) == [str(k) for k in golden["keys"]]


@pytest.mark.parametrize("case", ["cfg1", "mini2"])
def test_oracle_bit_exact_vs_reference_generator(golden, case):
    from oracle import hifigan_oracle as HO
    from fs2amd.vocoder import V1_CONFIG

    sd = {k: v.detach() for k, v in _gen().state_dict().items()}
    with torch.no_grad():
        y = HO.forward(sd, V1_CONFIG, torch.from_numpy(golden[f"{case}__mel"]))
    np.testing.assert_array_equal(y.numpy(), golden[f"{case}__wav"])


@pytest.mark.parametrize("cin,cout,k,u", [(64, 32, 16, 8), (32, 16, 4, 2), (16, 8, 8, 4)])
def test_phase_conv_equals_conv_transpose(cin, cout, k, u):
    """ConvTranspose1d(k, stride u, padding (k-u)/2) == Conv1d over the input with u*Cout phase
    outputs, reshaped [T, u*Cout] -> [T*u, Cout] (float64, exact up to summation order)."""
    from fs2amd.vocoder import phase_conv_weights

    g = torch.Generator().manual_seed(1)
    p = (k - u) // 2
    w = torch.randn(cin, cout, k, generator=g, dtype=torch.float64)
    x = torch.randn(2, cin, 13, generator=g, dtype=torch.float64)
    ref = F.conv_transpose1d(x, w, stride=u, padding=p)  # [2, Cout, 13*u]
    wp, pad = phase_conv_weights(w, u, p)
    y = F.conv1d(x, wp, padding=pad)[..., :13]            # [2, u*Cout, 13]
    y = y.transpose(1, 2).reshape(2, 13 * u, cout).transpose(1, 2)
    assert ref.shape == y.shape
    assert float((ref - y).abs().max()) < 1e-12


def test_weight_norm_folding():
    from fs2amd.vocoder import _weight

    g = _gen()
    m = g.resblocks[4].convs1[2]
    ref = m.weight_g * m.weight_v / m.weight_v.norm(dim=(1, 2), keepdim=True)
    assert torch.allclose(_weight(m), ref, atol=1e-6)
    g.remove_weight_norm()
    assert "conv_pre.weight" in g.state_dict() and "conv_pre.weight_g" not in g.state_dict()
