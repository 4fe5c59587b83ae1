"""SDPA at the Z-Image main-stack attention shape (one GPU's 256 images x (576 image + 96 caption)
tokens, 30 heads x 128): layout (strided [B,S,H,D] views vs contiguous [B,H,S,D]) x key-padding mask
(none vs additive [B,1,1,S]) x SDPA backend (flash / efficient / math), ms per call.
usage: python tools/zimage_attn_probe.py [out.json]"""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tools.gemm_probe_util import bench  # noqa: E402

dev = torch.device("cuda:0")
B, S, H, D = 256, 672, 30, 128
g = torch.Generator(device=dev).manual_seed(0)
qkv = [torch.randn(B, S, H, D, generator=g, device=dev).bfloat16() for _ in range(3)]
mask = torch.zeros(B, 1, 1, S, device=dev, dtype=torch.bfloat16)
mask[:, :, :, -40:] = float("-inf")
rows = []
for layout in ("strided", "contiguous"):
    q, k, v = ((t.transpose(1, 2) if layout == "strided" else t.transpose(1, 2).contiguous()) for t in qkv)
    for masked in (False, True):
        for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.MATH):
            if be == SDPBackend.MATH and not masked:
                continue
            try:
                with sdpa_kernel([be]):
                    fn = lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=mask if masked else None,  # noqa: E731
                                                                scale=D ** -0.5)
                    ms = min(bench(fn, it=3) for _ in range(3))
                fl = 4.0 * B * H * S * S * D
                r = {"layout": layout, "mask": masked, "backend": be.name, "ms": round(ms, 3),
                     "tflops": round(fl / ms / 1e9, 1)}
            except RuntimeError as e:
                r = {"layout": layout, "mask": masked, "backend": be.name, "error": str(e)[:120]}
            rows.append(r)
            print(json.dumps(r), flush=True)
            torch.cuda.empty_cache()
if len(sys.argv) > 1:
    Path(sys.argv[1]).write_text(json.dumps(rows, indent=1))
