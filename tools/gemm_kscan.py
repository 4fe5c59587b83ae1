"""Fixed vs per-K-tile cost of the population LoRA GEMM: time at K = 1120/2240/4480 (M = 131072,
N = 2240), r = 0 and r = 2, interleaved rounds; t(K) = fixed + slope * K.  (diagnostic)"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import _lib  # noqa: E402
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402

tile = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
M, N, rpm = 131072, 2240, 16384
res = {}
bufs = {}
for Kd in (1152, 2240, 4608):
    x = (torch.rand(M, Kd, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand(N, Kd, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    tp = torch.randn(M // rpm, 2 * Kd + 2 * N + 8, device=dev) * 0.1
    bufs[Kd] = (x, W, b, tp, torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.randn(M, 2, device=dev))
for _ in range(3):
    for Kd, (x, W, b, tp, y, T) in bufs.items():
        for r in (0, 2):
            res.setdefault((Kd, r), []).append(
                bench(lambda: K.lora_gemm(x, W, b, T if r else None, tp if r else None, 2 * Kd, r, 4.0, rpm, out=y, kernel=tile)))
out = {}
for (Kd, r), v in res.items():
    ms = min(v)
    out[f"K{Kd}_r{r}_ms"] = round(ms, 4)
    out[f"K{Kd}_r{r}_tf"] = round(2 * M * N * Kd / ms / 1e9, 1)
for r in (0, 2):
    slope = (out[f"K4608_r{r}_ms"] - out[f"K1152_r{r}_ms"]) / 3456
    out[f"r{r}_fixed_ms"] = round(out[f"K2240_r{r}_ms"] - slope * 2240, 4)
    out[f"r{r}_loop_tf"] = round(2 * M * N / slope / 1e9, 1)
print(json.dumps(out), flush=True)
