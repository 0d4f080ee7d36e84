"""Pin the oracle (oracle/fs2_oracle.py) against golden vectors captured from the reference."""
import hashlib

import numpy as np
import pytest
import torch

from _common import GOLDEN_CASES, OUT_NAMES, configs, load_case, manifest, oracle_state_dict
from oracle import fs2_oracle as O


def test_weight_generator_matches_manifest():
    """The counter-based generator regenerates exactly the weights the goldens were made with."""
    sd = oracle_state_dict()
    man = manifest()["keys"]
    assert set(sd) == set(man) and len(sd) == 240
    for k, meta in man.items():
        v = sd[k]
        assert list(v.shape) == meta["shape"], k
        digest = hashlib.sha256(v.detach().cpu().contiguous().numpy().tobytes()).hexdigest()
        assert digest == meta["sha256"], k


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_oracle_bit_exact_vs_reference(case):
    torch.set_num_threads(8)
    args, (p_c, e_c, d_c), outs, _ = load_case(case)
    pc, mc, _ = configs()
    got = O.forward(oracle_state_dict(), mc, pc, **args, p_control=p_c, e_control=e_c, d_control=d_c)
    for name, g in zip(OUT_NAMES, got):
        ref = outs[name]
        g = g.numpy()
        assert g.shape == ref.shape, name
        assert g.dtype == ref.dtype, name
        np.testing.assert_array_equal(g, ref, err_msg=f"{case}:{name}")


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_oracle_lr_index_map(case):
    args, _, outs, z = load_case(case)
    dur = torch.from_numpy(outs["d_rounded"]) if "d_targets" not in args else args["d_targets"]
    im, ml = O.length_regulate_index_map(dur, args.get("max_mel_len"))
    np.testing.assert_array_equal(im.numpy(), z["lr_index_map"])
    np.testing.assert_array_equal(ml.numpy(), z["lr_mel_len"])


def test_oracle_lr_cases(golden_dir):
    z = np.load(f"{golden_dir}/lr_cases.npz")
    names = sorted({k.split("__")[0] for k in z.files})
    assert len(names) >= 6
    for n in names:
        ml = int(z[f"{n}__max_len"])
        out, mel_len = O.length_regulate(torch.from_numpy(z[f"{n}__x"]), torch.from_numpy(z[f"{n}__d"]),
                                         None if ml < 0 else ml)
        np.testing.assert_array_equal(out.numpy(), z[f"{n}__out"], err_msg=n)
        np.testing.assert_array_equal(mel_len.numpy(), z[f"{n}__mel_len"], err_msg=n)


def test_oracle_training_step_matches_reference_gradients():
    """Train-mode forward (dropout disabled, BN batch statistics) + FastSpeech2Loss + backward of
    the oracle against the reference's own gradients (tests/golden/train_grads.npz)."""
    from _common import check_train_grads, load_train_case, oracle_state_dict
    from oracle import fs2_oracle as O

    z, args = load_train_case()
    pc, mc, _ = configs()
    sd = {k: v.clone() for k, v in oracle_state_dict().items()}  # train mode updates BN buffers in place
    keys = [str(k) for k in z["grad_keys"]]
    for k in keys:
        sd[k] = sd[k].clone().requires_grad_(True)
    out = O.forward(sd, mc, pc, **args, training=True)
    losses = O.loss(pc, args["mels"], args["p_targets"], args["e_targets"], args["d_targets"], out)
    np.testing.assert_allclose([float(l) for l in losses], z["losses"], rtol=1e-6)
    losses[0].backward()
    named = {k: sd[k].grad for k in keys}
    check_train_grads(z, named, rtol=1e-5, sample_atol_frac=1e-4)
    for k in z.files:
        if k.startswith("bn_"):
            np.testing.assert_allclose(sd[k[3:]].detach().numpy(), z[k], rtol=1e-5, atol=1e-6)



def test_padding_classes_of_the_reference():
    """the reference's output for one utterance depends on its phoneme padding
    class {0, 1, >=2} and frame padding class {0..9, >=10}; within a class it is bitwise equal.
    The pad_* fixtures (utterance 0 = the same base utterance) must show exactly that, so the
    parity tests that use them pin the padding semantics, not just one padded batch."""
    T0 = int(load_case("pad_ph1")[0]["mel_lens"][0])  # the base utterance's frames in every pad_* case
    ph = {e: load_case(f"pad_ph{e}")[2]["postnet_mel"][0] for e in (1, 2, 3)}
    fr = {e: load_case(f"pad_fr{e}")[2]["postnet_mel"][0] for e in (9, 10, 30)}
    # phoneme padding: +2 and +3 equal, +1 differs from them
    assert np.array_equal(ph[2][:T0], ph[3][:T0])
    assert not np.array_equal(ph[1][:T0], ph[2][:T0])
    # frame padding: +10 and +30 equal on the valid frames, +9 differs (PostNet +-10 receptive field)
    assert np.array_equal(fr[10][:T0], fr[30][:T0])
    assert not np.array_equal(fr[9][:T0], fr[10][:T0])


def test_oracle_cfg2_free_running_checksums():
    """Free-running cfg2 (rounded predicted durations -> LR -> decoder): the oracle reproduces the
    reference's rounded durations, mel lengths, index map and per-utterance checksums exactly."""
    args, _, outs, z = load_case("cfg2_free")
    torch.set_num_threads(8)
    pc, mc, _ = configs()
    got = O.forward(oracle_state_dict(), mc, pc, **args)
    np.testing.assert_array_equal(got[5].numpy(), outs["d_rounded"])
    np.testing.assert_array_equal(got[9].numpy(), outs["mel_lens_out"])
    im, ml = O.length_regulate_index_map(got[5], None)
    np.testing.assert_array_equal(im.numpy(), z["lr_index_map"])
    post = got[1].double()
    valid = (torch.arange(post.shape[1])[None, :] < got[9][:, None]).double()[..., None]
    np.testing.assert_array_equal((post * valid).sum((1, 2)).numpy(), z["ck_post_valid_sum"])
    np.testing.assert_array_equal((post * post).sum((1, 2)).numpy(), z["ck_post_sq"])


def test_oracle_training_step_b16_matches_reference_gradients():
    """The cfg3 shape (B=16, lengths U{16..64}) training step of the oracle against the
    reference's own gradients (tests/golden/train_b16.npz)."""
    from _common import check_train_grads, load_train_case

    z, args = load_train_case("train_b16")
    pc, mc, _ = configs()
    sd = {k: v.clone() for k, v in oracle_state_dict().items()}  # train mode updates BN buffers in place
    keys = [str(k) for k in z["grad_keys"]]
    for k in keys:
        sd[k] = sd[k].clone().requires_grad_(True)
    out = O.forward(sd, mc, pc, **args, training=True)
    losses = O.loss(pc, args["mels"], args["p_targets"], args["e_targets"], args["d_targets"], out)
    np.testing.assert_allclose([float(l) for l in losses], z["losses"], rtol=1e-6)
    losses[0].backward()
    check_train_grads(z, {k: sd[k].grad for k in keys}, rtol=1e-5, sample_atol_frac=1e-4)
