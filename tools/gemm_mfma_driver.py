"""The Sana epoch's dominant LoRA-GEMM launches at their product shape (131072 x 2240 x 2240, LoRA r 2,
8 members of 16 images x 1024 tokens) in the three forms the epoch runs: no epilogue op (attn1 q / k / v,
attn2 q), res32 (attn2 to_out: x32 += y) and gated32 (attn1 to_out: x32 = fma(gate, y, x32)), `reps`
launches each, T precomputed.  For rocprofv3 --pmc passes (tools/gemm_mfma_summary.py).
usage: python tools/gemm_mfma_driver.py [reps]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
M, N, Kd, r, n = 131072, 2240, 2240, 2, 8
rpm = M // n
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
W = (torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
b = torch.zeros(N, device=dev, dtype=torch.bfloat16)
tp = torch.randn(n, 2 * Kd + 2 * N + 4, device=dev, generator=g) * 0.02
T = K.lora_project(x, tp, 0, r, rpm)
y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
res = torch.randn(M, N, device=dev, generator=g)
gate = torch.randn(n * 16, N, device=dev, generator=g)
sh = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for _ in range(reps):
    K.lora_gemm(x, W, b, T, tp, 2 * Kd, r, 4.0, rpm, out=y)
for _ in range(reps):
    K.lora_gemm_epi(x, W, b, T, tp, 2 * Kd, r, 4.0, rpm, "res32", res=res, out=sh)
for _ in range(reps):
    K.lora_gemm_epi(x, W, b, T, tp, 2 * Kd, r, 4.0, rpm, "gated32", res=res, gate=gate, rows_per_group=1024, out=sh)
torch.cuda.synchronize()
print("ok", reps)
