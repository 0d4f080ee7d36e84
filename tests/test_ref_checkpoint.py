"""A checkpoint written by the REFERENCE's own train loop (tests/golden/gen_golden.py ckpt_case:
train.py:82-97 steps with the reference ScheduledOptim, :151-161 torch.save) restored through
fs2amd's drop-in get_model(train=True) (utils/model.py:11-34, weights_only load), then the
reference's step 3 replayed: same clipped gradients in, every parameter and the learning rate
out must equal the reference's.

The checkpoint is the reference's toy-width configuration (golden/ref_ckpt/model_config.json;
PostNet zero and frozen, so it has no gradient and no Adam state) and is stored gzip-compressed:
the test restores the exact bytes the reference wrote. CPU: plain torch Adam on both sides,
bit-identical; GPU: the fused Adam fs2amd uses on the device, within 1e-6 of each parameter's
scale.
"""
import gzip
import json
import os
import shutil
import types

import numpy as np
import pytest
import torch

from _common import GOLDEN, side_dir


def _restore(tmp_path, device):
    from fs2amd import config as C
    from fs2amd.checkpoint import get_model

    d = tmp_path / "ckpt"
    d.mkdir()
    with gzip.open(os.path.join(GOLDEN, "ref_ckpt", "2.pth.tar.gz"), "rb") as fi, open(d / "2.pth.tar", "wb") as fo:
        shutil.copyfileobj(fi, fo)
    with open(os.path.join(GOLDEN, "ref_ckpt", "model_config.json")) as f:
        mc = json.load(f)
    pc, _, tc = C.synthetic_configs(side_dir())
    tc["path"]["ckpt_path"] = str(d)
    return get_model(types.SimpleNamespace(restore_step=2), (pc, mc, tc), device, train=True)


def _replay_step3(model, optim, device):
    z = np.load(os.path.join(GOLDEN, "ref_ckpt_next.npz"))
    keys = [str(k) for k in z["keys"]]
    params = dict(model.named_parameters())
    for p in model.parameters():
        p.grad = None
    for i, k in enumerate(keys):
        params[k].grad = torch.from_numpy(z[f"g_{i}"]).to(device)
    optim.step_and_update_lr()
    return z, keys, params


def test_reference_checkpoint_restores_and_steps_cpu(tmp_path):
    model, optim = _restore(tmp_path, "cpu")
    assert model.training and optim.current_step == 2
    st = optim._optimizer.state_dict()
    assert len(st["state"]) == 73 and all(float(s["step"]) == 2.0 for s in st["state"].values())
    z, keys, params = _replay_step3(model, optim, "cpu")
    assert optim.current_step == int(z["current_step"]) == 3
    assert optim._optimizer.param_groups[0]["lr"] == float(z["lr"])
    for i, k in enumerate(keys):
        np.testing.assert_array_equal(params[k].detach().numpy(), z[f"p_{i}"], err_msg=k)
    # the frozen PostNet is untouched
    assert all(not p.any() for p in model.postnet.parameters())


@pytest.mark.gpu
def test_reference_checkpoint_restores_and_steps_gpu(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    model, optim = _restore(tmp_path, torch.device("cuda:0"))
    assert optim._optimizer.defaults.get("fused"), "device training uses the fused Adam"
    z, keys, params = _replay_step3(model, optim, torch.device("cuda:0"))
    torch.cuda.synchronize()
    assert abs(float(optim._optimizer.param_groups[0]["lr"]) - float(z["lr"])) <= 1e-12
    for i, k in enumerate(keys):
        ref = z[f"p_{i}"]
        got = params[k].detach().cpu().numpy()
        scale = max(float(np.abs(ref).max()), 1e-6)
        assert float(np.abs(got - ref).max()) <= 1e-6 * scale, (k, float(np.abs(got - ref).max()))
