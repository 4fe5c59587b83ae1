"""Runs eggroll_flash_attention at the Z-Image main-stack shape (64 x 676 x 676, 30 heads) a few times, for
rocprofv3 --pmc passes on k_flash_attn (diagnostic).  usage: python tools/flash_driver.py [reps]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
q = (torch.randn(64, 676, 30, 128, device=dev) * 0.3).bfloat16()
k = (torch.randn(64, 676, 30, 128, device=dev) * 0.3).bfloat16()
v = (torch.randn(64, 676, 30, 128, device=dev) * 0.3).bfloat16()
for _ in range(reps):
    K.flash_attention(q, k, v, 128 ** -0.5)
torch.cuda.synchronize()
print("done")
