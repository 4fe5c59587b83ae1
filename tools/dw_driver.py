"""Runs the Sana FFN depthwise conv (SiLU -> dw3x3 -> GLU, 128 images x 32x32 x 11200 channels) and
the DC-AE 128x128x4096 one a few times, for rocprofv3 --pmc passes on k_dwconv_nhwc.
usage: python tools/dw_driver.py [reps]   (diagnostic)"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
for B, H, W, C in ((128, 32, 32, 11200), (8, 128, 128, 4096)):
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(9, C, device=dev) * 0.2).to(torch.bfloat16)
    b = (torch.randn(C, device=dev) * 0.1).to(torch.bfloat16)
    out = torch.empty(B, H, W, C // 2, device=dev, dtype=torch.bfloat16)
    for _ in range(reps):
        K.dwconv_nhwc(x, w, b, 3, pre_silu=True, glu=True, out=out)
torch.cuda.synchronize()
print("done")
