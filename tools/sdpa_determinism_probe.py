"""Run-to-run determinism of F.scaled_dot_product_attention with an additive mask at the tiny Sana attn2
shape (the path CrossAttention takes when the head dim is not 112) vs eggroll_cross_attention."""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from hyperscalees_t2i_amd import kernels as K
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for B, N, H, hd, L in ((128, 1024, 2, 64, 300), (128, 1024, 20, 112, 300)):
        q = torch.randn(B, H, N, hd, device=dev, generator=g).to(torch.bfloat16)
        k = torch.randn(B, H, L, hd, device=dev, generator=g).to(torch.bfloat16)
        v = torch.randn(B, H, L, hd, device=dev, generator=g).to(torch.bfloat16)
        m = torch.zeros(B, 1, 1, L, device=dev, dtype=torch.bfloat16)
        m[..., 200:] = -10000.0
        f = lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=m, scale=hd ** -0.5)  # noqa: E731
        base = f()
        res[f"sdpa_hd{hd}"] = sum(int(not torch.equal(base, f())) for _ in range(20))
        if hd == 112:
            qq = q.transpose(1, 2).reshape(B * N, H * hd).contiguous()
            kk = k.transpose(1, 2).reshape(B * L, H * hd).contiguous()
            vv = v.transpose(1, 2).reshape(B * L, H * hd).contiguous()
            fk = lambda: K.cross_attention(qq, kk, vv, B, N, H, hd, L, hd ** -0.5, bias=m.view(B, L).contiguous())  # noqa: E731
            bk = fk()
            res["eggroll_xattn_hd112"] = sum(int(not torch.equal(bk, fk())) for _ in range(20))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
