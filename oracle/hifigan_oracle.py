"""TEST INFRASTRUCTURE ONLY — the CPU restatement of the HiFi-GAN V1 generator forward.

Restates hifigan/models.py:112-165 (Generator.forward) and :96-105 (ResBlock.forward) in plain
PyTorch fp32 on CPU over a state dict (weight-normed ``weight_g`` / ``weight_v`` keys or plain
``weight`` keys after remove_weight_norm). Pinned against the reference generator's own outputs
(tests/golden/vocoder.npz, made by tests/golden/gen_golden.py by running hifigan.Generator here).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import it; the product path
(fs2amd.vocoder) never does.
"""
import torch
import torch.nn.functional as F

LRELU_SLOPE = 0.1  # hifigan/models.py:7


def _w(sd, prefix):
    """Effective weight of one conv: weight norm g * v / ||v|| (dim 0), hifigan/models.py:23-88."""
    if prefix + ".weight_g" in sd:
        return torch._weight_norm(sd[prefix + ".weight_v"], sd[prefix + ".weight_g"], 0)
    return sd[prefix + ".weight"]


def _pad(k, d=1):
    return int((k * d - d) / 2)  # get_padding, hifigan/models.py:16-17


def resblock(sd, prefix, x, k, dilations):
    """ResBlock1.forward (hifigan/models.py:96-105)."""
    for i, d in enumerate(dilations):
        xt = F.leaky_relu(x, LRELU_SLOPE)
        xt = F.conv1d(xt, _w(sd, f"{prefix}.convs1.{i}"), sd[f"{prefix}.convs1.{i}.bias"], dilation=d, padding=_pad(k, d))
        xt = F.leaky_relu(xt, LRELU_SLOPE)
        xt = F.conv1d(xt, _w(sd, f"{prefix}.convs2.{i}"), sd[f"{prefix}.convs2.{i}.bias"], padding=_pad(k))
        x = xt + x
    return x


def forward(sd, h, x):
    """Generator.forward (hifigan/models.py:146-165): mel [B, 80, T] -> wav [B, 1, T * prod(u)]."""
    x = F.conv1d(x, _w(sd, "conv_pre"), sd["conv_pre.bias"], padding=3)
    nk = len(h["resblock_kernel_sizes"])
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        x = F.leaky_relu(x, LRELU_SLOPE)
        x = F.conv_transpose1d(x, _w(sd, f"ups.{i}"), sd[f"ups.{i}.bias"], stride=u, padding=(k - u) // 2)
        xs = None
        for j, (rk, rd) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
            r = resblock(sd, f"resblocks.{i * nk + j}", x, rk, rd)
            xs = r if xs is None else xs + r
        x = xs / nk
    x = F.leaky_relu(x)
    x = F.conv1d(x, _w(sd, "conv_post"), sd["conv_post.bias"], padding=3)
    return torch.tanh(x)
