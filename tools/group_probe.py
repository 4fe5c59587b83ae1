"""Time the 8-phase LoRA GEMM (tile 8) at the Sana shapes with whatever libeggroll EGGROLL_LIB names
(rasterisation-group A/B: tools/gpu_group.sh builds one library per EGG_GROUP_M).
usage: EGGROLL_LIB=... python tools/group_probe.py <label>"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import _lib  # noqa: E402
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402

dev = torch.device("cuda:0")
out = {"label": sys.argv[1] if len(sys.argv) > 1 else ""}
for (M, N, Kd, rpm) in [(8 * 16384, 2240, 2240, 16384), (8 * 4800, 2240, 2240, 4800)]:
    x = (torch.rand(M, Kd, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand(N, Kd, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    tp = torch.randn(M // rpm, 2 * Kd + 2 * N + 8, device=dev) * 0.1
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    T = torch.empty(M, 2, device=dev)
    K.lora_project(x, tp, 0, 2, rpm, out=T)
    ms = min(bench(lambda: K.lora_gemm(x, W, b, T, tp, 2 * Kd, 2, 4.0, rpm, out=y, kernel=8)) for _ in range(5))
    out[f"M{M}"] = round(2 * M * N * Kd / ms / 1e9, 1)
print(json.dumps(out), flush=True)
