"""GEMM + epilogue at the Infinity block shapes (M = 2 members x 32 rows x 1024 tokens): the 256x256
(kernel 8) vs 256x320 (kernel 10) 8-phase tiles, bf16 residual / gated epilogues and plain, HIP events,
median of rounds; bitwise equality of the two (diagnostic).
usage: python tools/epi_kernel_probe.py"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


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


M = 65536
for name, Kd, N, epi in (("fc2_gated", 14336, 3584, "gated"), ("sa_proj_gated", 3584, 3584, "gated"),
                         ("ca_proj_res", 3584, 3584, "res"), ("mat_qkv", 3584, 10752, None), ("mat_q", 3584, 3584, None)):
    g = torch.Generator(device=dev).manual_seed(Kd)
    x = torch.randn(M, Kd, generator=g, device=dev).bfloat16()
    W = (torch.randn(N, Kd, generator=g, device=dev) / Kd ** 0.5).bfloat16()
    b = torch.zeros(N, device=dev).bfloat16()
    res0 = torch.randn(M, N, generator=g, device=dev).bfloat16()
    gate = torch.randn(M // 1024, N, generator=g, device=dev).bfloat16()
    outs = {}

    def run(k):
        if epi is None:
            return K.lora_linear_pop(x, W, b, None, 0, 0, 0, 0.0, M, kernel=k)
        r = res0.clone()
        return K.lora_linear_pop_epi(x, W, b, None, 0, 0, 0, 0.0, M, epi, res=r, gate=gate if epi == "gated" else None,
                                     rows_per_group=1024, kernel=k)
    res = {8: [], 10: []}
    for _ in range(4):
        for k in (8, 10):
            res[k].append(t(lambda: run(k)))
    eq = torch.equal(run(8), run(10))
    print(json.dumps({name: {"k8_us": round(statistics.median(res[8]), 1), "k10_us": round(statistics.median(res[10]), 1),
                             "bitwise_equal": eq}}), flush=True)
