"""Sana cross-attention at the bench shape (B = 128 images, 20 heads x 112, N = 1024 image tokens,
L = 300 caption tokens): SDPA with the additive key-padding mask vs without, vs key-sliced.
usage: python tools/xattn_probe.py"""
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
valid = 120
mask = torch.zeros(B, 1, 1, L, device=dev, dtype=torch.bfloat16)
mask[..., valid:] = float("-inf")
res = {}
for _ in range(3):
    res.setdefault("mask", []).append(bench(lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=mask), 5))
    res.setdefault("nomask", []).append(bench(lambda: F.scaled_dot_product_attention(q, k, v), 5))
    ks, vs = k[:, :, :valid], v[:, :, :valid]
    res.setdefault("sliced", []).append(bench(lambda: F.scaled_dot_product_attention(q, ks, vs), 5))
    res.setdefault("sliced_contig", []).append(bench(lambda: F.scaled_dot_product_attention(q, ks.contiguous(), vs.contiguous()), 5))
for kk, vv in res.items():
    print(kk, round(min(vv), 3), "ms", flush=True)
a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask).float()
b = F.scaled_dot_product_attention(q, k[:, :, :valid], v[:, :, :valid]).float()
print("max|mask - sliced|", (a - b).abs().max().item(), "max|y|", a.abs().max().item())

qc = q.contiguous()
mb = torch.zeros(B, 1, 1, L, device=dev, dtype=torch.bfloat16)
mb[..., valid:] = -10000.0


def explicit(q, k, v, mb):
    s = torch.matmul(q, k.transpose(-1, -2))                     # [B, h, N, L] bf16, fp32 accumulate
    p = torch.softmax(s.float() * (d ** -0.5) + mb.float(), dim=-1).to(torch.bfloat16)
    return torch.matmul(p, v)


res = {}
for _ in range(3):
    res.setdefault("sdpa_qcontig_mask", []).append(bench(lambda: F.scaled_dot_product_attention(qc, k, v, attn_mask=mb), 5))
    res.setdefault("sdpa_mask", []).append(bench(lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=mb), 5))
    res.setdefault("explicit", []).append(bench(lambda: explicit(q, k, v, mb), 5))
for kk, vv in res.items():
    print(kk, round(min(vv), 3), "ms", flush=True)
a = F.scaled_dot_product_attention(q, k, v, attn_mask=mb).float()
e = explicit(q, k, v, mb).float()
print("max|sdpa - explicit|", (a - e).abs().max().item(), "rel", ((a - e).norm() / a.norm()).item())
