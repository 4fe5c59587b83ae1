"""DC-AE decoder head (RMSNorm + ReLU + 3x3 conv 128 -> 3) at the epoch shape (8 x 1024^2 x 128)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn((8, 1024, 1024, 128), generator=g, device=dev).to(torch.bfloat16)
nw = torch.ones(128, device=dev, dtype=torch.bfloat16)
nb = torch.zeros(128, device=dev, dtype=torch.bfloat16)
w = (torch.randn((3, 128, 3, 3), generator=g, device=dev) / 30).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
b = torch.zeros(3, device=dev, dtype=torch.bfloat16)
K.dcae_head(x, 1e-5, nw, nb, w, b)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    K.dcae_head(x, 1e-5, nw, nb, w, b)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(json.dumps({"dcae_head_ms": round(ms, 4), "TBps": round(x.numel() * 2 / ms / 1e9, 3)}))
