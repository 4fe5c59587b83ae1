"""Diagnostic 2: identity centre-tap weights -> y should equal x; report which input pixel/channel
permutation the kernel actually produced."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
B, H, W, C = 1, 16, 16, 64
x = torch.randn(B, H, W, C, generator=g).to(dev, torch.bfloat16)
w = torch.zeros(C, C, 3, 3, device=dev, dtype=torch.bfloat16)
w[:, :, 1, 1] = torch.eye(C, device=dev, dtype=torch.bfloat16)
y = K.conv3x3_nhwc(x, K.pack_conv3x3_weight(w, 1), None, 1, None).float()
xf = x.float().reshape(-1, C)
yf = y.reshape(-1, C)
print("max |y - x|:", (yf - xf).abs().max().item())
# per output pixel: best-matching input pixel (channel order kept) and channel permutation of pixel 0
d = torch.cdist(yf, xf)
best = d.argmin(dim=1)
print("best input pixel for output pixels 0..15:", best[:16].tolist(), "dist", d.min(dim=1).values[:4].tolist())
dc = torch.cdist(yf.t(), xf.t())
print("best input channel for output channels 0..15:", dc.argmin(dim=1)[:16].tolist(), "dist", dc.min(dim=1).values[:4].tolist())
print("y[0,:8]", yf[0, :8].tolist())
print("x[0,:8]", xf[0, :8].tolist())
print("y[1,:8]", yf[1, :8].tolist())
print("x[1,:8]", xf[1, :8].tolist())
