"""Sana cross-attention (B 128, 20 heads, hd 112, N 1024, L 300): SDPA at hd 112 vs zero-padded to
hd 128 with the 1/sqrt(112) scale passed explicitly (exact: zero dims add nothing).
usage: python tools/xattn_pad_probe.py"""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tools.gemm_probe_util import bench  # noqa: E402

dev = torch.device("cuda:0")
B, h, d, N, L = 128, 20, 112, 1024, 300
q = torch.randn(B, N, h, d, device=dev, dtype=torch.bfloat16).transpose(1, 2)
k = torch.randn(B, L, h, d, device=dev, dtype=torch.bfloat16).transpose(1, 2)
v = torch.randn(B, L, h, d, device=dev, dtype=torch.bfloat16).transpose(1, 2)
mb = torch.zeros(B, 1, 1, L, device=dev, dtype=torch.bfloat16)
mb[..., 150:] = -10000.0
sc = d ** -0.5


def padded(q, k, v):
    qp, kp, vp = (F.pad(t, (0, 128 - d)) for t in (q, k, v))
    return F.scaled_dot_product_attention(qp, kp, vp, attn_mask=mb, scale=sc)[..., :d]


qp, kp, vp = (F.pad(t, (0, 128 - d)) for t in (q, k, v))
res = {}
for _ in range(3):
    res.setdefault("hd112", []).append(bench(lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=mb), 5))
    res.setdefault("hd128_incl_pad", []).append(bench(lambda: padded(q, k, v), 5))
    res.setdefault("hd128_sdpa_only", []).append(bench(lambda: F.scaled_dot_product_attention(qp, kp, vp, attn_mask=mb, scale=sc), 5))
    res.setdefault("hd128_nomask", []).append(bench(lambda: F.scaled_dot_product_attention(qp, kp, vp, scale=sc), 5))
for kk, vv in res.items():
    print(kk, round(min(vv), 3), "ms", flush=True)
a = F.scaled_dot_product_attention(q, k, v, attn_mask=mb).float()
b = padded(q, k, v).float()
print("max|112 - 128pad|", (a - b).abs().max().item(), "rel", ((a - b).norm() / a.norm()).item())
