"""Linear attention (eggroll_linear_attention: k_la_kv -> k_la_reduce -> k_la_out) at the epoch's
shapes: Sana attn1 (128 images x 1024 tokens x 70 heads, separate q/k/v) and the DC-AE multiscale
attention (8 images, interleaved q|k|v per head, ReLU on q/k).  Per-kernel times come from rocprof;
this prints the whole call's time and HBM rate on the algorithmic bytes (q, k, v read once, out
written once).  usage: python tools/la_probe.py"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402

dev = torch.device("cuda:0")
for B, N, heads, inter in ((128, 1024, 70, False), (8, 16384, 16, True), (8, 4096, 32, True), (8, 1024, 32, True),
                           (8, 16384, 16, "planar"), (8, 4096, 32, "planar"), (8, 1024, 32, "planar")):
    if inter == "planar":  # [B*N, 3*inner] = Q | K | V planes, head h = columns 32h of each
        qkv = torch.randn(B * N, 3 * heads * 32, device=dev).to(torch.bfloat16)
        q, k, v, hs = qkv, qkv[:, heads * 32:], qkv[:, 2 * heads * 32:], 32
    elif inter:  # [B*N, 3*inner], head h = columns [96h, 96h + 96) = q | k | v
        qkv = torch.randn(B * N, 3 * heads * 32, device=dev).to(torch.bfloat16)
        q, k, v, hs = qkv, qkv[:, 32:], qkv[:, 64:], 96
    else:
        q, k, v = (torch.randn(B * N, heads * 32, device=dev).abs().to(torch.bfloat16) for _ in range(3))
        hs = 32
    out = torch.empty(B * N, heads * 32, device=dev, dtype=torch.bfloat16)
    ms = min(bench(lambda: K.linear_attention(q, k, v, B, N, heads, hs, relu_qk=bool(inter), out=out), 5) for _ in range(3))
    nbytes = 2.0 * B * N * heads * 32 * 4
    print(json.dumps({"shape": f"B{B} N{N} h{heads}" + (" planar" if inter == "planar" else ""), "ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 2)}),
          flush=True)
