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


def _checksums(got):
    mel, post = got[0].double().cpu(), got[1].double().cpu()
    ml = got[9].cpu()
    valid = (torch.arange(mel.shape[1])[None, :] < ml[:, None]).double()[..., None]
    return {"ck_mel_valid_sum": (mel * valid).sum((1, 2)).numpy(), "ck_post_valid_sum": (post * valid).sum((1, 2)).numpy(),
            "ck_post_valid_abs": (post.abs() * valid).sum((1, 2)).numpy(), "ck_post_all_sum": post.sum((1, 2)).numpy(),
            "ck_post_sq": (post * post).sum((1, 2)).numpy()}


def _lr_index_map(dur, max_len):
    """The HIP LengthRegulator's source-index map for these durations (fs2_lr_expand)."""
    from fs2amd import ops

    d = dur.to(DEV)
    x = torch.zeros(d.shape[0], d.shape[1], 8, device=DEV)
    _, ml, im = ops.length_regulate(x, d, max_len, return_index_map=True)
    return im.cpu().numpy(), ml.cpu().numpy()


def test_cfg2_fp32_checksums(model):
    """Full cfg2 shape (B=64, L=64, T=430) on the COMMITTED reference inputs against every field
    the reference's fixture stores: per-utterance checksums (valid-frame sums of mel / postnet,
    |postnet|, all-frame postnet sum incl. the padding, sum of squares), the predictions, the
    masks, mel lengths and the LR index map (the full outputs are not committed).
    Tolerances: sums atol 0.5 (a sum over ~31k values of O(1) with |err| <= 2e-3 each),
    |.| and squares rtol 1e-5, predictions 5e-4; discrete outputs exact."""
    args, controls, outs, z = load_case("cfg2_checksums")
    assert tuple(args["texts"].shape) == (64, 64) and args["max_mel_len"] == int(z["out_shape_mel"][1])
    got = _run(model, args, controls, "fp32")
    assert tuple(got[0].shape) == tuple(z["out_shape_mel"])
    ck = _checksums(got)
    for k in ("ck_mel_valid_sum", "ck_post_valid_sum", "ck_post_all_sum"):
        np.testing.assert_allclose(ck[k], z[k], rtol=0, atol=0.5, err_msg=k)
    for k in ("ck_post_valid_abs", "ck_post_sq"):
        np.testing.assert_allclose(ck[k], z[k], rtol=1e-5, err_msg=k)
    for i, name in ((2, "p_pred"), (3, "e_pred"), (4, "log_d")):
        np.testing.assert_allclose(_np(got[i]), outs[name], atol=5e-4, err_msg=name)
    np.testing.assert_array_equal(_np(got[5]), outs["d_rounded"])  # the d_targets, passed through
    np.testing.assert_array_equal(_np(got[6]), outs["src_masks"])
    np.testing.assert_array_equal(_np(got[7]), outs["mel_masks"])
    np.testing.assert_array_equal(_np(got[9]), outs["mel_lens_out"])
    im, ml = _lr_index_map(args["d_targets"], args["max_mel_len"])
    np.testing.assert_array_equal(im, z["lr_index_map"])
    np.testing.assert_array_equal(ml, z["lr_mel_len"])


def test_cfg2_free_running_fp32(model):
    """Free-running cfg2 (the synthesis path: predicted log-durations -> round -> LengthRegulator,
    modules.py:131-137) on the committed reference inputs: rounded durations, mel lengths, masks
    and the LR index map bit-exact; checksums as in the teacher-forced test."""
    args, controls, outs, z = load_case("cfg2_free")
    assert "d_targets" not in args and "max_mel_len" not in args
    got = _run(model, args, controls, "fp32")
    np.testing.assert_array_equal(_np(got[5]), outs["d_rounded"])
    np.testing.assert_array_equal(_np(got[9]), outs["mel_lens_out"])
    np.testing.assert_array_equal(_np(got[6]), outs["src_masks"])
    np.testing.assert_array_equal(_np(got[7]), outs["mel_masks"])
    assert tuple(got[0].shape) == tuple(z["out_shape_mel"])
    im, ml = _lr_index_map(got[5], None)
    np.testing.assert_array_equal(im, z["lr_index_map"])
    np.testing.assert_array_equal(ml, z["lr_mel_len"])
    for i, name in ((2, "p_pred"), (3, "e_pred"), (4, "log_d")):
        np.testing.assert_allclose(_np(got[i]), outs[name], atol=5e-4, err_msg=name)
    ck = _checksums(got)
    for k in ("ck_mel_valid_sum", "ck_post_valid_sum", "ck_post_all_sum"):
        np.testing.assert_allclose(ck[k], z[k], rtol=0, atol=1.0, err_msg=k)
    for k in ("ck_post_valid_abs", "ck_post_sq"):
        np.testing.assert_allclose(ck[k], z[k], rtol=1e-5, err_msg=k)


# Measured bounds on the discrete decisions the bf16 perf mode changes in free-running synthesis
# (cfg2 committed inputs, 4,096 valid phonemes; SURVEY.md §0 trap 2; tools/flip_rate.py). The
# bf16 encoder moves the VariancePredictors' inputs by ~2^-8 relative, so their outputs move by
# |dp|, |de| <= 0.02 = half a bucket width (0.039 / 0.041) and |d log_d| <= 0.025: measured
# 1.29 % of rounded durations and 10.6 % of pitch buckets land one step over, 9.8 % of energy
# buckets with the pitch buckets pinned. Unpinned, a flipped pitch bucket swaps a whole (random-
# init) embedding row into the energy predictor's input and energy flips compound (44.8 %, up to
# 57 buckets): bounded separately below. Asserted bounds (margin over the measurement):
FLIP_MAX_DUR, FLIP_MAX_BUCKET, PRED_MAX_ERR = 0.02, 0.15, 0.04


def _flips(f, b, va):
    valid = ~f[6]
    n = int(valid.sum())
    pb = [torch.bucketize(t[2], va.pitch_bins) for t in (f, b)]
    eb = [torch.bucketize(t[3], va.energy_bins) for t in (f, b)]
    return {"n": n, "dur": int(((f[5] != b[5]) & valid).sum()) / n, "dur_step": float((f[5] - b[5]).abs()[valid].max()),
            "pitch": int(((pb[0] != pb[1]) & valid).sum()) / n, "pitch_step": int((pb[0] - pb[1]).abs().max()),
            "energy": int(((eb[0] != eb[1]) & valid).sum()) / n, "energy_step": int((eb[0] - eb[1]).abs().max()),
            "dp": float((f[2] - b[2]).abs()[valid].max()), "de": float((f[3] - b[3]).abs()[valid].max())}


def test_cfg2_bf16_free_running_flip_rate(model):
    args, controls, _, _ = load_case("cfg2_free")
    va = model.variance_adaptor
    f = _run(model, args, controls, "fp32")
    b = _run(model, args, controls, "bf16")
    r = _flips(f, b, va)
    print("bf16 free-running:", r)
    assert r["dur"] <= FLIP_MAX_DUR and r["dur_step"] <= 1.0, r
    assert r["pitch"] <= FLIP_MAX_BUCKET and r["pitch_step"] <= 1 and r["dp"] <= PRED_MAX_ERR, r
    # compounded through flipped pitch embedding rows (see above): measured 44.8 % with the fused
    # split-hidden encoder FFN (rounds 2-5) and 46.3 % with fs2_ffn_wide (round 6: the same hidden and
    # pre-norm sums, LayerNorm row statistics summed in another order -- a 1-ulp change that moves
    # ~60 near-tie pitch buckets and everything downstream of their embedding rows); the kernels are
    # deterministic, so a rate is reproducible per build; bound = the larger measurement + 1.2 points
    # (~50 of the 4,096 phonemes)
    assert r["energy"] <= 0.475, r
    # away from the flipped pitch buckets (no flip within the energy predictor's receptive field,
    # +-2 phonemes: two k=3 convs) the energy buckets behave as in the pinned run below
    valid = ~f[6]
    pflip = ((torch.bucketize(f[2], va.pitch_bins) != torch.bucketize(b[2], va.pitch_bins)) & valid).float()
    near = torch.nn.functional.max_pool1d(pflip[:, None], 5, 1, 2)[:, 0] > 0
    clean = valid & ~near
    eflip = (torch.bucketize(f[3], va.energy_bins) != torch.bucketize(b[3], va.energy_bins)) & clean
    r_clean = int(eflip.sum()) / max(1, int(clean.sum()))
    print("energy flips away from pitch flips:", r_clean, "of", int(clean.sum()))
    assert int(clean.sum()) >= 0.3 * r["n"] and r_clean <= FLIP_MAX_BUCKET, (r_clean, int(clean.sum()))
    # the output length follows the rounded durations exactly
    np.testing.assert_array_equal(_np(b[9]), _np(b[5]).sum(1).astype(np.int64))
    # energy on its own: pitch buckets pinned to the fp32 predictions
    pinned = dict(args, p_targets=f[2].cpu())
    f2 = _run(model, pinned, controls, "fp32")
    b2 = _run(model, pinned, controls, "bf16")
    r2 = _flips(f2, b2, va)
    print("bf16 free-running, pitch pinned:", r2)
    assert r2["energy"] <= FLIP_MAX_BUCKET and r2["energy_step"] <= 1 and r2["de"] <= PRED_MAX_ERR, r2


def test_cfg2_bf16_vs_fp32_hip(model):
    """bf16 perf path vs the fp32 HIP path at the bench shape (teacher-forced durations; pitch /
    energy pinned to the fp32 predictions so no bucket flips): the bf16 tolerance."""
    args, _, _, _ = load_case("cfg2_checksums")
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


def test_cfg4_variable_length_fp32_checksums(model):
    """cfg4 (B=256, 16-160 phonemes, T_max 971) on the committed reference inputs: LR-stress
    shape, ragged padding everywhere."""
    args, _, _, z = load_case("cfg4_checksums")
    assert tuple(args["texts"].shape)[0] == 256
    got = _run(model, args, (1.0, 1.0, 1.0), "fp32")
    post = got[1].double().cpu()
    ml = got[9].cpu()
    assert tuple(got[0].shape) == tuple(z["out_shape_mel"])
    valid = (torch.arange(post.shape[1])[None, :] < ml[:, None]).double()[..., None]
    ok = np.isclose((post * valid).sum((1, 2)).numpy(), z["ck_post_valid_sum"], rtol=0, atol=1.0)
    ok &= np.isclose((post.abs() * valid).sum((1, 2)).numpy(), z["ck_post_valid_abs"], rtol=2e-5, atol=0)
    ok &= np.isclose(post.sum((1, 2)).numpy(), z["ck_post_all_sum"], rtol=0, atol=2.0)
    # fp32 summation order differs from the reference's: a pitch / energy prediction that sits on a
    # bucket edge can land in the neighbouring bucket (the utterance then differs by one embedding
    # row). Allowed, <= 2 of 256, only where that is what happened: the utterance has a phoneme
    # whose bucket differs between this run and the reference, and there the two predictions agree
    # within FLIP_EPS (so the reference value lies within FLIP_EPS of the edge between them).
    # Energy flips count only in an utterance without a pitch flip (a flipped pitch row changes
    # the energy predictor's input).
    FLIP_EPS = 4e-6
    bad = np.flatnonzero(~ok)
    assert len(bad) <= 2, bad
    va = model.variance_adaptor
    src_valid = ~z["out_src_masks"]
    pbins, ebins = va.pitch_bins.cpu().numpy(), va.energy_bins.cpu().numpy()
    for b in bad:
        v = src_valid[b]
        gp, rp = _np(got[2])[b][v], z["out_p_pred"][b][v]
        ge, re = _np(got[3])[b][v], z["out_e_pred"][b][v]
        fp = np.searchsorted(pbins, gp, side="left") != np.searchsorted(pbins, rp, side="left")
        fe = np.searchsorted(ebins, ge, side="left") != np.searchsorted(ebins, re, side="left")
        d = np.abs(gp - rp)[fp] if fp.any() else np.abs(ge - re)[fe]
        print(f"cfg4 fp32 flip: utterance {b}: pitch flips {int(fp.sum())}, energy flips {int(fe.sum())}, "
              f"|d pred| at the flips {d.tolist()}")
        assert fp.any() or fe.any(), (b, "checksum mismatch without a bucket flip")
        assert float(d.max()) <= FLIP_EPS, (b, d.tolist())
    np.testing.assert_allclose(_np(got[2]), z["out_p_pred"], atol=5e-4)
    keep = np.setdiff1d(np.arange(len(ok)), bad)  # energy sees the flipped pitch embedding
    np.testing.assert_allclose(_np(got[3])[keep], z["out_e_pred"][keep], atol=5e-4)
    np.testing.assert_allclose(_np(got[4]), z["out_log_d"], atol=5e-4)
    np.testing.assert_array_equal(ml.numpy(), z["out_mel_lens_out"])
    np.testing.assert_array_equal(_np(got[6]), z["out_src_masks"])
    np.testing.assert_array_equal(_np(got[7]), z["out_mel_masks"])
    np.testing.assert_array_equal(_np(got[5]), z["out_d_rounded"])
    im, iml = _lr_index_map(args["d_targets"], args["max_mel_len"])
    np.testing.assert_array_equal(im, z["lr_index_map"])
    np.testing.assert_array_equal(iml, z["lr_mel_len"])
    ck = _checksums(got)
    np.testing.assert_allclose(ck["ck_mel_valid_sum"][keep], z["ck_mel_valid_sum"][keep], rtol=0, atol=1.0)
    np.testing.assert_allclose(ck["ck_post_sq"][keep], z["ck_post_sq"][keep], rtol=2e-5)


# ---- round-3 fixtures: pitch / energy TARGETS at the bench shapes (no bucket can flip), so the
# bf16 perf path is checked against the reference itself at full size; the eval PE-recompute
# branch (> max_seq_len positions)
def _valid_err(got_post, ref_post, ml):
    T = ref_post.shape[1]
    valid = (np.arange(T)[None, :] < ml[:, None])[..., None]
    e = np.abs(got_post - ref_post) * valid
    return float(e.max()), float(e.sum() / (valid.sum() * ref_post.shape[2]))


@pytest.mark.parametrize("case,head", [("cfg2_targets", 4), ("cfg4_targets", 2)])
def test_targets_fp32_vs_reference(model, case, head):
    """fp32 at the bench shapes (cfg2 64 x 64, cfg4 256 x U{16..160}) with teacher-forced
    durations and pitch / energy targets: the first utterances element-wise (2e-3, the fp32
    tolerance), every utterance's checksums as test_cfg2_fp32_checksums, discrete outputs exact."""
    args, controls, outs, z = load_case(case)
    got = _run(model, args, controls, "fp32")
    assert tuple(got[0].shape) == tuple(z["out_shape_mel"])
    ml = _np(got[9])
    np.testing.assert_array_equal(ml, outs["mel_lens_out"])
    mx, _ = _valid_err(_np(got[1][:head]), outs["postnet_mel_head"], ml[:head])
    assert mx <= 2e-3, mx
    ck = _checksums(got)
    for k in ("ck_mel_valid_sum", "ck_post_valid_sum", "ck_post_all_sum"):
        np.testing.assert_allclose(ck[k], z[k], rtol=0, atol=0.5, err_msg=k)
    for k in ("ck_post_valid_abs", "ck_post_sq"):
        np.testing.assert_allclose(ck[k], z[k], rtol=1e-5, err_msg=k)
    np.testing.assert_array_equal(_np(got[6]), outs["src_masks"])
    np.testing.assert_array_equal(_np(got[7]), outs["mel_masks"])


# bf16 perf path against the reference at the bench shapes (targets pinned: no discrete decision
# differs). Measured round 3 (fused FFN): cfg2 head max 0.033 / mean 0.0061, |postnet| checksum
# rel 1.7e-3, per-value sum error 1.5e-3; cfg4 0.036 / 0.0067 / 2.0e-3 / 1.7e-3. Bounds ~2x that.
@pytest.mark.parametrize("case,head", [("cfg2_targets", 4), ("cfg4_targets", 2)])
def test_targets_bf16_vs_reference(model, case, head):
    args, controls, outs, z = load_case(case)
    got = _run(model, args, controls, "bf16")
    ml = _np(got[9])
    np.testing.assert_array_equal(ml, outs["mel_lens_out"])
    mx, mean = _valid_err(_np(got[1][:head]), outs["postnet_mel_head"], ml[:head])
    ck = _checksums(got)
    rel_abs = np.abs(ck["ck_post_valid_abs"] - z["ck_post_valid_abs"]) / z["ck_post_valid_abs"]
    n_valid = ml.astype(np.float64) * 80
    mean_sum_err = np.abs(ck["ck_post_valid_sum"] - z["ck_post_valid_sum"]) / n_valid
    print(f"{case} bf16 vs reference: head max {mx:.4f} mean {mean:.5f}; |post| checksum rel max "
          f"{rel_abs.max():.2e}; per-frame-value sum error max {mean_sum_err.max():.2e}")
    assert mx <= 0.075 and mean <= 0.0125, (mx, mean)
    assert rel_abs.max() <= 4e-3, rel_abs.max()
    assert mean_sum_err.max() <= 4e-3, mean_sum_err.max()


def test_long_eval_pe_recompute_fp32(model):
    """Eval with 2004 phonemes and 2004 frames, past max_seq_len = 2000: the encoder and the
    decoder recompute the sinusoid table for the sequence length (transformer/Models.py:82-87,
    145-152) instead of slicing the 2001-row one. Frames 0-31 and 1960-2003 element-wise (2e-3),
    checksums, exact lengths / masks."""
    args, controls, outs, z = load_case("long_eval")
    assert args["texts"].shape[1] == 2004 and args["max_mel_len"] == 2004
    got = _run(model, args, controls, "fp32")
    assert tuple(got[0].shape) == (1, 2004, 80)
    post = _np(got[1])
    for a, b in ((0, 32), (1960, 2004)):
        e = float(np.abs(post[:, a:b] - z[f"out_postnet_mel_f{a}_{b}"]).max())
        assert e <= 2e-3, (a, b, e)
    ck = _checksums(got)
    for k in ("ck_mel_valid_sum", "ck_post_valid_sum", "ck_post_all_sum"):
        np.testing.assert_allclose(ck[k], z[k], rtol=0, atol=0.5, err_msg=k)
    np.testing.assert_allclose(ck["ck_post_sq"], z["ck_post_sq"], rtol=1e-5)
    np.testing.assert_array_equal(_np(got[9]), outs["mel_lens_out"])
    np.testing.assert_array_equal(_np(got[7]), outs["mel_masks"])
