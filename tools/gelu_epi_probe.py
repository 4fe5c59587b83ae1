"""Infinity fc1 (M = 2 members x 32 rows x 1024 tokens, K 3584, N 14336, LoRA r 2): the GEMM + torch GELU
vs the GEMM with the GELU(tanh) epilogue (kernel 8 / 10), HIP events, median of rounds.
usage: python tools/gelu_epi_probe.py   (diagnostic)"""
import json
import statistics
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
M, Kd, N, r, n = 65536, 3584, 14336, 2, 2
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, Kd, generator=g, device=dev).bfloat16()
W = (torch.randn(N, Kd, generator=g, device=dev) / Kd ** 0.5).bfloat16()
b = torch.zeros(N, device=dev).bfloat16()
tp = torch.randn(n, Kd * r + N * r + 8, generator=g, device=dev) * 0.02
ws = torch.empty(K.lora_workspace_numel(M, Kd, r, M // n), device=dev)


def t(fn, it=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


cases = {
    "gemm_only_k0": lambda: K.lora_linear_pop(x, W, b, tp, 0, Kd * r, r, 4.0, M // n, T_ws=ws),
    "gemm+torch_gelu": lambda: F.gelu(K.lora_linear_pop(x, W, b, tp, 0, Kd * r, r, 4.0, M // n, T_ws=ws), approximate="tanh"),
    "epi_gelu_k0": lambda: K.lora_linear_pop_epi(x, W, b, tp, 0, Kd * r, r, 4.0, M // n, "gelu", T_ws=ws),
    "epi_gelu_k8": lambda: K.lora_linear_pop_epi(x, W, b, tp, 0, Kd * r, r, 4.0, M // n, "gelu", T_ws=ws, kernel=8),
    "epi_gelu_k10": lambda: K.lora_linear_pop_epi(x, W, b, tp, 0, Kd * r, r, 4.0, M // n, "gelu", T_ws=ws, kernel=10),
    "epi_silu_k0": lambda: K.lora_linear_pop_epi(x, W, b, tp, 0, Kd * r, r, 4.0, M // n, "silu", T_ws=ws),
}
res = {k: [] for k in cases}
for _ in range(5):
    for k, f in cases.items():
        res[k].append(t(f))
print(json.dumps({k: round(statistics.median(v), 1) for k, v in res.items()}))
