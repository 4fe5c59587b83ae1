"""Launches the population LoRA GEMM (kernels 8 and 10, 131072 x 2240 x 2240, r 2, random operands)
back to back for a counter pass: `rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace`, then
tools/gemm_clock_summary.py gives the effective clock per kernel = GRBM_GUI_ACTIVE / 8 XCDs / kernel
duration (MI355X_MICROARCH.md 'DVFS give-back').  usage: python tools/gemm_clock_driver.py [reps]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
M, N, Kd, rpm = 131072, 2240, 2240, 16384
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.rand((M, Kd), generator=g, device=dev) * 2 - 1).bfloat16()
W = ((torch.rand((N, Kd), generator=g, device=dev) * 2 - 1) * 0.05).bfloat16()
b = torch.randn(N, generator=g, device=dev).bfloat16()
tp = torch.randn((M // rpm, 2 * Kd + 2 * N + 8), generator=g, device=dev) * 0.1
T = K.lora_project(x, tp, 0, 2, rpm)
y = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
for kern in (8, 10, 8, 10):
    for _ in range(reps):
        K.lora_gemm(x, W, b, T, tp, 2 * Kd, 2, 4.0, rpm, out=y, kernel=kern)
    torch.cuda.synchronize()
print("done")
