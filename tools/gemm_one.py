"""Run one LoRA GEMM variant N times at the Sana attention shape (for rocprofv3 --pmc passes).
usage: python tools/gemm_one.py <tile> [reps] [r]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import _lib  # noqa: E402
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

tile = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
r = int(sys.argv[3]) if len(sys.argv) > 3 else 2
dev = torch.device("cuda:0")
M, N, Kd, rpm = 131072, 2240, 2240, 16384
x = (torch.rand(M, Kd, device=dev) * 2 - 1).bfloat16()
W = ((torch.rand(N, Kd, device=dev) * 2 - 1) * 0.05).bfloat16()
b = torch.randn(N, device=dev).bfloat16()
tp = torch.randn(M // rpm, 2 * Kd + 2 * N + 8, device=dev) * 0.1
y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
T = torch.randn(M, 2, device=dev)
for _ in range(reps):
    K.lora_gemm(x, W, b, T if r else None, tp if r else None, 2 * Kd, r, 4.0, rpm, out=y, kernel=tile)
torch.cuda.synchronize()
print("done")
