"""Plain bf16 GEMMs at small M (Infinity's early scales: 64 .. 4608 rows, the 8B block widths): libeggroll's
automatic kernel vs F.linear (hipBLASLt), HIP events, median us (diagnostic).
usage: python tools/small_m_gemm_probe.py"""
import json
import statistics
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for M in (64, 256, 1024, 2304, 4096, 9216):
    row = {}
    for name, Kd, N in (("qkv", 3584, 10752), ("proj", 3584, 3584), ("fc1", 3584, 14336), ("fc2", 14336, 3584)):
        x = torch.randn(M, Kd, device=dev).bfloat16()
        W = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).bfloat16()
        b = torch.zeros(N, device=dev).bfloat16()
        r = {"ours": [], "hipblaslt": []}
        for _ in range(3):
            r["ours"].append(t(lambda: K.lora_linear_pop(x, W, b, None, 0, 0, 0, 0.0, M)))
            r["hipblaslt"].append(t(lambda: F.linear(x, W, b)))
        row[name] = (round(statistics.median(r["ours"]), 1), round(statistics.median(r["hipblaslt"]), 1))
    print(json.dumps({f"M{M}": row}), flush=True)
