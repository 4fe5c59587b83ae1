"""Sana cross-attention SDPA at the bench shape: with the padding mask (current), without, trimmed,
and per-distinct-prompt grouped (queries of the R images of one prompt as one sequence per member)."""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
n, m, R, N, H, hd, L = 8, 4, 4, 1024, 20, 128, 300
B = n * m * R
q = torch.randn((B, H, N, hd), generator=g, device=dev).to(torch.bfloat16)
ku = torch.randn((n * m, H, L, hd), generator=g, device=dev).to(torch.bfloat16)
vu = torch.randn((n * m, H, L, hd), generator=g, device=dev).to(torch.bfloat16)
lens = [37, 150, 233, 300]
mask_u = torch.zeros((n * m, 1, 1, L), device=dev, dtype=torch.bfloat16)
for j, lj in enumerate(lens):
    mask_u.view(n, m, 1, 1, L)[:, j, :, :, lj:] = -10000.0
idx = torch.arange(B, device=dev)
enc_index = (idx // (m * R)) * m + (idx % m)
k, v, mask = ku.index_select(0, enc_index), vu.index_select(0, enc_index), mask_u.index_select(0, enc_index)
res = {}
res["masked_full"] = timeit(lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=112 ** -0.5))
res["nomask_full"] = timeit(lambda: F.scaled_dot_product_attention(q, k, v, scale=112 ** -0.5))
res["nomask_L160"] = timeit(lambda: F.scaled_dot_product_attention(q, k[:, :, :160], v[:, :, :160], scale=112 ** -0.5))
res["index_select_kv"] = timeit(lambda: (ku.index_select(0, enc_index), vu.index_select(0, enc_index)))


def grouped():
    o = torch.empty_like(q)
    qv = q.view(n, R, m, H, N, hd)
    ov = o.view(n, R, m, H, N, hd)
    for j, lj in enumerate(lens):
        qj = qv[:, :, j].permute(0, 2, 1, 3, 4).reshape(n, H, R * N, hd)
        kj = ku.view(n, m, H, L, hd)[:, j, :, :lj]
        vj = vu.view(n, m, H, L, hd)[:, j, :, :lj]
        oj = F.scaled_dot_product_attention(qj, kj, vj, scale=112 ** -0.5)
        ov[:, :, j] = oj.view(n, H, R, N, hd).permute(0, 2, 1, 3, 4)
    return o


res["grouped_trimmed"] = timeit(grouped)
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
q2 = torch.randn((B * N, H * 112), generator=g, device=dev).to(torch.bfloat16)
k2 = torch.randn((n * m * L, H * 112), generator=g, device=dev).to(torch.bfloat16)
v2 = torch.randn((n * m * L, H * 112), generator=g, device=dev).to(torch.bfloat16)
res["eggroll_cross_attention"] = timeit(lambda: K.cross_attention(q2, k2, v2, B, N, H, 112, L, 112 ** -0.5,
                                                                   bias=mask_u.view(n * m, L), enc_index=enc_index))
ref = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=112 ** -0.5)
res["grouped_maxdiff"] = float((grouped().float() - ref.float()).abs().max())
print(json.dumps({k2: round(v2, 4) for k2, v2 in res.items()}))
