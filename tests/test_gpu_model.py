"""End-to-end parity of FastSpeech2.forward on the HIP path against the reference's golden
vectors and the oracle.

Tolerances (written here, per the north star's "stated fp32 tolerance"):
* fp32 mode: |mel - ref| <= 2e-3 absolute (outputs are O(1); the kernels run exact-f32
  MFMA/FMA chains, only summation order and exp/rsqrt last-bit differ), p/e/log-duration
  predictions <= 5e-4; discrete outputs (durations, mel_lens, masks) EXACT.
* bf16 mode (teacher-forced durations, targets for pitch/energy so no bucket can flip):
  |postnet_mel - ref| <= 0.15 absolute, mean abs <= 0.02.
"""
import numpy as np
import pytest
import torch

from _common import GOLDEN_CASES, OUT_NAMES, configs, load_case, oracle_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from fs2amd.model import FastSpeech2

    pc, mc, _ = configs()
    m = FastSpeech2(pc, mc)
    m.load_state_dict(oracle_state_dict())
    return m.to(DEV).eval()


def _run(model, args, controls, prec):
    from fs2amd.data import to_device

    model.set_precision(prec)
    p_c, e_c, d_c = controls
    with torch.no_grad():
        out = model(**to_device(args, DEV), p_control=p_c, e_control=e_c, d_control=d_c)
    torch.cuda.synchronize()
    return out


def _np(v):
    return v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_fp32_matches_reference_goldens(model, case):
    args, controls, outs, z = load_case(case)
    got = _run(model, args, controls, "fp32")
    for name, g in zip(OUT_NAMES, got):
        ref = outs[name]
        g = _np(g)
        assert g.shape == ref.shape, (case, name, g.shape, ref.shape)
        if name in ("mel", "postnet_mel"):
            assert np.abs(g - ref).max() <= 2e-3, (case, name, np.abs(g - ref).max())
        elif name in ("p_pred", "e_pred", "log_d"):
            assert np.abs(g - ref).max() <= 5e-4, (case, name, np.abs(g - ref).max())
        elif name == "d_rounded":
            np.testing.assert_array_equal(g.astype(ref.dtype), ref, err_msg=f"{case}:{name}")
        else:
            np.testing.assert_array_equal(g, ref, err_msg=f"{case}:{name}")


@pytest.mark.parametrize("case", ["mini_targets", "cfg1_teacher"])
def test_bf16_within_tolerance(model, case):
    args, controls, outs, _ = load_case(case)
    if "p_targets" not in args:
        # pin pitch/energy buckets with the reference's own predictions (no bf16 bucket flips)
        args = dict(args, p_targets=torch.from_numpy(outs["p_pred"]) / controls[0],
                    e_targets=torch.from_numpy(outs["e_pred"]) / controls[0])
    got = _run(model, args, controls, "bf16")
    ref = outs["postnet_mel"]
    g = _np(got[1])
    err = np.abs(g - ref)
    assert err.max() <= 0.15 and err.mean() <= 0.02, (err.max(), err.mean())
    np.testing.assert_array_equal(_np(got[9]), outs["mel_lens_out"])


def test_cfg2_fp32_checksums(model, golden_dir):
    """Full cfg2 shape (B=64, L=64, T=430) against the reference's per-sequence checksums and
    the LR index map (the full outputs are not committed)."""
    from fs2amd.data import synth_batch

    z = np.load(f"{golden_dir}/cfg2_checksums.npz")
    args = synth_batch(64, 64, seed=1)
    assert int(args["max_mel_len"]) == int(z["out_shape_mel"][1])
    got = _run(model, args, (1.0, 1.0, 1.0), "fp32")
    mel, post = got[0].double().cpu(), got[1].double().cpu()
    ml = got[9].cpu()
    valid = (torch.arange(mel.shape[1])[None, :] < ml[:, None]).double()[..., None]
    np.testing.assert_allclose((post * valid).sum((1, 2)).numpy(), z["ck_post_valid_sum"], rtol=0, atol=0.5)
    np.testing.assert_allclose((post.abs() * valid).sum((1, 2)).numpy(), z["ck_post_valid_abs"], rtol=1e-5)
    np.testing.assert_allclose((post * post).sum((1, 2)).numpy(), z["ck_post_sq"], rtol=1e-5)
    np.testing.assert_allclose(_np(got[2]), z["out_p_pred"], atol=5e-4)
    np.testing.assert_array_equal(ml.numpy(), z["out_mel_lens_out"])


def test_cfg2_bf16_vs_fp32_hip(model):
    """bf16 perf path vs the fp32 HIP path at the bench shape (teacher-forced durations; pitch /
    energy pinned to the fp32 predictions so no bucket flips): the bf16 tolerance."""
    from fs2amd.data import synth_batch

    args = synth_batch(64, 64, seed=1)
    f = _run(model, args, (1.0, 1.0, 1.0), "fp32")
    args = dict(args, p_targets=f[2].cpu(), e_targets=f[3].cpu())
    b = _run(model, args, (1.0, 1.0, 1.0), "bf16")
    err = (b[1] - f[1]).abs()
    assert float(err.max()) <= 0.2 and float(err.mean()) <= 0.02, (float(err.max()), float(err.mean()))


def test_cpu_tensors_fail_loudly(model):
    from fs2amd.model import FastSpeech2
    from fs2amd.data import synth_batch

    pc, mc, _ = configs()
    m = FastSpeech2(pc, mc).eval()
    with pytest.raises(RuntimeError, match="HIP"):
        with torch.no_grad():
            m(**synth_batch(1, 8, seed=3))


def test_cfg4_variable_length_fp32_checksums(model, golden_dir):
    """cfg4 (B=256, 16-160 phonemes, T_max 971): LR-stress shape, ragged padding everywhere."""
    from fs2amd.data import synth_batch

    z = np.load(f"{golden_dir}/cfg4_checksums.npz")
    args = synth_batch(256, 16, 160, seed=1)
    got = _run(model, args, (1.0, 1.0, 1.0), "fp32")
    post = got[1].double().cpu()
    ml = got[9].cpu()
    assert tuple(got[0].shape) == tuple(z["out_shape_mel"])
    valid = (torch.arange(post.shape[1])[None, :] < ml[:, None]).double()[..., None]
    ok = np.isclose((post * valid).sum((1, 2)).numpy(), z["ck_post_valid_sum"], rtol=0, atol=1.0)
    ok &= np.isclose((post.abs() * valid).sum((1, 2)).numpy(), z["ck_post_valid_abs"], rtol=2e-5, atol=0)
    ok &= np.isclose(post.sum((1, 2)).numpy(), z["ck_post_all_sum"], rtol=0, atol=2.0)
    # fp32 summation order differs from the reference's: a pitch / energy prediction within
    # ~1e-7 of a bucket edge can land in the neighbouring bucket (the utterance then differs by
    # one embedding row). Allowed only where a prediction is that close to an edge, <= 2 of 256.
    bad = np.flatnonzero(~ok)
    assert len(bad) <= 2, bad
    va = model.variance_adaptor
    src_valid = ~z["out_src_masks"]
    for b in bad:
        dp = np.abs(z["out_p_pred"][b][src_valid[b]][:, None] - va.pitch_bins.cpu().numpy()[None, :]).min()
        de = np.abs(z["out_e_pred"][b][src_valid[b]][:, None] - va.energy_bins.cpu().numpy()[None, :]).min()
        assert min(dp, de) < 1e-4, (b, dp, de)
    np.testing.assert_allclose(_np(got[2]), z["out_p_pred"], atol=5e-4)
    keep = np.setdiff1d(np.arange(len(ok)), bad)  # energy sees the flipped pitch embedding
    np.testing.assert_allclose(_np(got[3])[keep], z["out_e_pred"][keep], atol=5e-4)
    np.testing.assert_allclose(_np(got[4]), z["out_log_d"], atol=5e-4)
    np.testing.assert_array_equal(ml.numpy(), z["out_mel_lens_out"])
    np.testing.assert_array_equal(_np(got[6]), z["out_src_masks"])
    np.testing.assert_array_equal(_np(got[7]), z["out_mel_masks"])
