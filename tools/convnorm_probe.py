"""ResBlock conv2 tail: conv + RMSNorm + residual fused in the conv epilogue vs the plain conv followed by
one eggroll_rownorm pass (w, b, residual), at the DC-AE shapes (8 images)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def t(fn, it=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(5_000_000)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for B, C, hw in [(8, 128, 1024), (8, 256, 512)]:
    x = torch.randn(B, hw, hw, C, device=dev, dtype=torch.bfloat16)
    res = torch.randn(B, hw, hw, C, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    nw = torch.randn(C, device=dev).to(torch.bfloat16)
    nb = torch.randn(C, device=dev).to(torch.bfloat16)
    wp = K.pack_conv3x3_weight(w, 1)
    y = torch.empty_like(x)
    fused = t(lambda: K.conv3x3_rmsnorm_nhwc(x, wp, None, 1, 1e-5, nw, nb, res))
    plain = t(lambda: K.conv3x3_nhwc(x, wp, None, 1, None, out=y))
    z = K.conv3x3_nhwc(x, wp, None, 1, None)
    norm = t(lambda: K.rownorm(z, 1e-5, layer=False, w=nw, b=nb, res=res))
    a = K.conv3x3_rmsnorm_nhwc(x, wp, None, 1, 1e-5, nw, nb, res)
    bb = K.rownorm(K.conv3x3_nhwc(x, wp, None, 1, None), 1e-5, layer=False, w=nw, b=nb, res=res)
    print(json.dumps({"shape": [B, hw, hw, C], "fused_ms": round(fused, 3), "conv_ms": round(plain, 3),
                      "rownorm_ms": round(norm, 3), "separate_ms": round(plain + norm, 3),
                      "maxdiff": float((a.float() - bb.float()).abs().max())}), flush=True)
