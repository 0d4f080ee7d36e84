"""Debug helper: fused FFN vs the two-launch path; error pattern by row block / column block."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
import torch  # noqa: E402

from fs2amd import _lib as L, ops  # noqa: E402

DEV = "cuda:0"
g = torch.Generator(device=DEV).manual_seed(0)
F, ks = 1024, 9
w1 = torch.randn(F, 256, ks, device=DEV, generator=g) / (256 * ks) ** 0.5
w2 = torch.randn(256, F, 1, device=DEV, generator=g) / F ** 0.5
b1 = 0.1 * torch.randn(F, device=DEV, generator=g)
b2 = 0.1 * torch.randn(256, device=DEV, generator=g)
ln = (torch.ones(256, device=DEV), torch.zeros(256, device=DEV), 1e-5)
B, T = int(sys.argv[1]) if len(sys.argv) > 1 else 1, int(sys.argv[2]) if len(sys.argv) > 2 else 224
lens = torch.full((B,), T, dtype=torch.int64, device=DEV)
x = torch.randn(B, T, 256, device=DEV, generator=g).to(torch.bfloat16)
fused = ops.ffn(x, ops.pack_ffn_weights(w1, w2), b1, b2, ks=ks, pad=4, ln=ln, lens=lens).float()
kw = dict(compute=L.FS2_BF16, out_dtype=L.FS2_BF16)
f = ops.conv1d(x, ops.pack_conv_weight(w1, L.FS2_BF16), b1, cin=256, ks=ks, pad=4, epilogue=L.EPI_BIAS_RELU, **kw)
two = ops.conv1d(f, ops.pack_conv_weight(w2, L.FS2_BF16), b2, cin=1024, ks=1, pad=0, epilogue=L.EPI_RES_LN,
                 residual=x, ln=ln, lens=lens, **kw).float()
d = (fused - two).abs().reshape(-1, 256)
print("max", float(d.max()), "mean", float(d.mean()))
rb = d.reshape(-1, 16, 256).amax(dim=(1, 2))
print("per 16-row block max:", [round(float(v), 3) for v in rb[:16]])
cb = d.reshape(-1, 256).amax(dim=0).reshape(16, 16).amax(dim=1)
print("per 16-col block max:", [round(float(v), 3) for v in cb])
