"""Main-loop-only (tile 10: no epilogue, no C stores) vs the full 8-phase kernel (tile 8) vs
hipBLASLt at the Sana attention shape, interleaved rounds — bounds what the epilogue/prologue costs.
usage: python tools/gemm_diag.py [rounds]   (diagnostic)"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import _lib  # noqa: E402
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
for (M, N, Kd, rpm) in [(131072, 2240, 2240, 16384), (131072, 2240, 4480, 16384)]:
    x = (torch.rand(M, Kd, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand(N, Kd, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    tp = torch.randn(M // rpm, 2 * Kd + 2 * N + 8, device=dev) * 0.1
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    T = torch.randn(M, 2, device=dev)
    res = {}
    for _ in range(rounds):
        for tile in (8, 10):
            _lib.call("eggroll_lora_gemm_tile", tile)
            res.setdefault(f"t{tile}", []).append(bench(lambda: K.lora_gemm(x, W, b, T, tp, 2 * Kd, 2, 4.0, rpm, out=y)))
        _lib.call("eggroll_lora_gemm_tile", 0)
        res.setdefault("torch", []).append(bench(lambda: torch.nn.functional.linear(x, W, b)))
    out = {"M": M, "N": N, "K": Kd}
    for k, v in res.items():
        out[k + "_ms"] = round(min(v), 4)
        out[k + "_tf"] = round(2 * M * N * Kd / min(v) / 1e9, 1)
    print(json.dumps(out), flush=True)
