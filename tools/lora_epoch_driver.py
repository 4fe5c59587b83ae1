"""Replays one ES epoch's population LoRA-GEMM launch mix (Sana-Sprint 1.6B, 1024 px, 8 members)
on synthetic data: project + GEMM per LoRA target, in bench order.  Used for PMC passes
(rocprofv3 --pmc ... --kernel-include-regex k_lora_gemm) where running the full model would
be slow.  usage: python tools/lora_epoch_driver.py [reps]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from tools.sana_layers import sana_lora_layers  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
members = 8
dev = torch.device("cuda:0")
bufs = []
for rows, Kd, N, cnt in sana_lora_layers():
    M = rows * members
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, Kd, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.zeros(N, device=dev, dtype=torch.bfloat16)
    tp = torch.randn(members, 2 * Kd + 2 * N + 4, device=dev) * 0.02
    T = torch.empty(M, 2, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    bufs.append((rows, Kd, N, cnt, x, W, b, tp, T, y))
for _ in range(reps):
    for rows, Kd, N, cnt, x, W, b, tp, T, y in bufs:
        for _ in range(cnt):
            K.lora_project(x, tp, 0, 2, rows, out=T)
            K.lora_gemm(x, W, b, T, tp, 2 * Kd, 2, 4.0, rows, out=y)
torch.cuda.synchronize()
print("launches per epoch:", sum(c for *_, c in [(0, 0, 0, cnt) for _, _, _, cnt, *rest in bufs]))
