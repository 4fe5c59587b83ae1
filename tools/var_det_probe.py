"""Which VQVAE-decode ops are run-to-run deterministic on this ROCm stack (bf16, channels-last)."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)


def rep(name, fn, n=3):
    outs = [fn() for _ in range(n)]
    torch.cuda.synchronize()
    eq = all(torch.equal(outs[0], o) for o in outs[1:])
    print(f"{name:48s} equal={eq} maxdiff={max(float((outs[0].float() - o.float()).abs().max()) for o in outs[1:]):.3g}",
          flush=True)


for (c, hw) in ((160, 256), (320, 64), (640, 16)):
    x = torch.randn((8, c, hw, hw), generator=g, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn((c, c, 3, 3), generator=g, device=dev) / (3 * c ** 0.5)).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    b = torch.zeros(c, device=dev, dtype=torch.bfloat16)
    gn = torch.nn.GroupNorm(32, c, eps=1e-6).to(dev, torch.bfloat16)
    rep(f"conv3x3 c{c} hw{hw} bf16 cl", lambda: F.conv2d(x, w, b, padding=1))
    rep(f"conv3x3 c{c} hw{hw} bf16 contiguous", lambda: F.conv2d(x.contiguous(), w.contiguous(), b, padding=1))
    rep(f"groupnorm c{c} hw{hw} bf16 cl", lambda: gn(x))
    rep(f"groupnorm c{c} hw{hw} bf16 contiguous", lambda: gn(x.contiguous()))
    rep(f"nearest up c{c}", lambda: F.interpolate(x, scale_factor=2, mode="nearest"))
    w1 = (torch.randn((c, c, 1, 1), generator=g, device=dev) / c ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    rep(f"conv1x1 c{c} hw{hw} bf16 cl", lambda: F.conv2d(x, w1, b))
    if hw == 16:
        q = torch.randn((8, 1, 256, c), generator=g, device=dev).to(torch.bfloat16)
        rep(f"sdpa hd{c}", lambda: F.scaled_dot_product_attention(q, q, q, scale=c ** -0.5))
