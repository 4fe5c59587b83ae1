"""DC-AE multiscale branch kernel (5x5 depthwise + grouped 1x1 on MFMA) at the epoch's three shapes."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402


def timeit(fn, iters=20):
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
for (B, H, W, C) in ((8, 128, 128, 1536), (8, 64, 64, 3072), (8, 32, 32, 3072)):
    x = torch.randn((B, H, W, C), generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn((25, C), generator=g, device=dev) / 5).to(torch.bfloat16)
    pw = (torch.randn((C // 32, 32, 32), generator=g, device=dev) / 6).to(torch.bfloat16)
    ms = timeit(lambda: K.dwconv_pw_nhwc(x, w, pw, 5))
    gb = 2 * 2 * x.numel() / 1e9
    print(json.dumps({"shape": [B, H, W, C], "ms": round(ms, 4), "TBps": round(gb / ms, 3)}), flush=True)
