"""A/B of the population LoRA GEMM variants vs torch (hipBLASLt) at Sana shapes, interleaved rounds
in one process (cdna_hip_programming.md §5.4 rule 24).  usage: python tools/gemm_probe.py [rounds]"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import _lib  # noqa: E402
from hyperscalees_t2i_amd import kernels as K  # noqa: E402


from tools.gemm_probe_util import bench  # noqa: E402


def _unused(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
for (M, N, Kd, rpm) in [(8 * 16384, 2240, 2240, 16384), (8 * 4800, 2240, 2240, 4800), (8 * 16384, 11200, 2240, 16384)]:
    x = (torch.rand(M, Kd, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand(N, Kd, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    tp = torch.randn(M // rpm, 2 * Kd + 2 * N + 8, device=dev) * 0.1
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    T = torch.empty(M, 2, device=dev)
    K.lora_project(x, tp, 0, 2, rpm, out=T)
    res = {}
    ws = torch.empty(K.lora_workspace_numel(M, Kd, 2, rpm), device=dev)
    for _ in range(rounds):
        for tile in (256, 9, 8):
            res.setdefault(f"gemm_t{tile}", []).append(bench(lambda: K.lora_gemm(x, W, b, T, tp, 2 * Kd, 2, 4.0, rpm, out=y, kernel=tile)))
        res.setdefault("linear_pop_auto", []).append(
            bench(lambda: K.lora_linear_pop(x, W, b, tp, 0, 2 * Kd, 2, 4.0, rpm, out=y, T_ws=ws)))
        res.setdefault("project", []).append(bench(lambda: K.lora_project(x, tp, 0, 2, rpm, out=T)))
        res.setdefault("torch", []).append(bench(lambda: torch.nn.functional.linear(x, W, b)))
    fl = 2 * M * N * Kd
    out = {"M": M, "N": N, "K": Kd}
    for k, v in res.items():
        ms = min(v)
        out[k + "_ms"] = round(ms, 4)
        if k != "project":
            out[k + "_tflops"] = round(fl / ms / 1e9, 1)
        else:
            out["project_GBps"] = round(M * Kd * 2 / ms / 1e6, 1)
    print(json.dumps(out), flush=True)
