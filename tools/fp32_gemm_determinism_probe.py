"""Run-to-run determinism of the torch fp32 GEMMs the build uses (LoRALinear.forward_fp32: F.linear on
fp32 copies + the member LoRA term as torch.bmm) at the Sana proj_out shape, repeated N times; with and
without torch.use_deterministic_algorithms and per BLAS library.

    python tools/fp32_gemm_determinism_probe.py
"""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def rep(fn, n=12):
    base = fn()
    bad = 0
    for _ in range(n):
        bad += int(not torch.equal(base, fn()))
    return bad


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M, K, N, n, r = 8 * 16 * 1024, 2240, 32, 8, 2
    x = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    b = torch.randn(N, device=dev, generator=g)
    A = torch.randn(n, r, K, device=dev, generator=g) * 0.02
    B = torch.randn(n, N, r, device=dev, generator=g) * 0.02
    lin = lambda: F.linear(x, W, b)  # noqa: E731
    bmm1 = lambda: torch.bmm(x.view(n, M // n, K), A.transpose(1, 2))  # noqa: E731
    t = bmm1()
    bmm2 = lambda: torch.bmm(t, B.transpose(1, 2))  # noqa: E731
    te = torch.randn(128, 256, device=dev, generator=g)
    We = torch.randn(2240, 256, device=dev, generator=g)
    small = lambda: F.linear(te, We)  # noqa: E731
    res = {}
    for lib in ("default", "cublas", "cublaslt"):
        if lib != "default":
            try:
                torch.backends.cuda.preferred_blas_library(lib)
            except Exception as e:  # noqa: BLE001
                res[lib] = str(e)
                continue
        for det in (False, True):
            torch.use_deterministic_algorithms(det, warn_only=True)
            res[f"{lib}/det{int(det)}"] = {"linear": rep(lin), "bmm_xA": rep(bmm1), "bmm_tB": rep(bmm2),
                                           "small_linear": rep(small)}
        torch.use_deterministic_algorithms(False)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
