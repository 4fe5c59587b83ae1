"""GLUMBConv pieces at the epoch's shapes: depthwise conv with / without the input SiLU, and the
inverted 1x1 conv GEMM on hipBLASLt (F.linear) vs libeggroll's 8-phase GEMM (r = 0)."""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402


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
out = {}
# (B, H, W, Cin of the block, 2h)
for name, (B, H, W, C, C2) in {"sana_ffn": (128, 32, 32, 2240, 11200), "dcae_s3": (8, 128, 128, 512, 4096),
                               "dcae_s4": (8, 64, 64, 1024, 8192), "dcae_s5": (8, 32, 32, 1024, 8192)}.items():
    x = torch.randn((B, H, W, C), generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn((C2, C), generator=g, device=dev) / C ** 0.5).to(torch.bfloat16)
    b = torch.zeros(C2, device=dev, dtype=torch.bfloat16)
    wdw = (torch.randn((9, C2), generator=g, device=dev) / 3).to(torch.bfloat16)
    bdw = torch.zeros(C2, device=dev, dtype=torch.bfloat16)
    h = F.linear(x, w, b)
    M = B * H * W
    fl = 2.0 * M * C * C2
    t_hb = timeit(lambda: F.linear(x, w, b))
    t_eg = timeit(lambda: K.lora_linear_pop(x.view(M, C), w, b, None, 0, 0, 0, 0.0, M))
    t_dw1 = timeit(lambda: K.dwconv_nhwc(h, wdw, bdw, 3, pre_silu=True, glu=True))
    t_dw0 = timeit(lambda: K.dwconv_nhwc(h, wdw, bdw, 3, pre_silu=False, glu=True))
    out[name] = {"gemm_hipblaslt_ms": t_hb, "gemm_eggroll_ms": t_eg, "hipblaslt_tf": fl / t_hb / 1e9,
                 "eggroll_tf": fl / t_eg / 1e9, "dwconv_presilu_ms": t_dw1, "dwconv_nosilu_ms": t_dw0}
    print(name, json.dumps({k: round(v, 3) for k, v in out[name].items()}), flush=True)
