"""A/B of the 256x256 (kernel 8) and 256x320 (kernel 10) 8-phase LoRA GEMMs at the epoch's shapes,
interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); outputs compared bitwise.
usage: python tools/gemm10_probe.py [rounds] [out.json]"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
rows = []
# (M, N, K, r, rows_per_member, epi): attn1 q/k/v/out + attn2 q/out (131072 x 2240^2), attn2 k/v on the distinct
# captions (8 x 1200 rows), the Sana FFN inverted conv (r 0, SiLU epilogue, N 11200), a gated-residual to_out
for (M, N, Kd, r, rpm, epi) in [(131072, 2240, 2240, 2, 16384, None), (9600, 2240, 2240, 2, 1200, None),
                                (131072, 11200, 2240, 0, 131072, "silu"), (131072, 2240, 2240, 2, 16384, "gated")]:
    g = torch.Generator(device=dev).manual_seed(M + N)
    x = (torch.rand((M, Kd), generator=g, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand((N, Kd), generator=g, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, generator=g, device=dev).bfloat16()
    tp = torch.randn((M // rpm, 2 * Kd + 2 * N + 8), generator=g, device=dev) * 0.1 if r else None
    T = K.lora_project(x, tp, 0, r, rpm) if r else None
    res = torch.randn((M, N), generator=g, device=dev).bfloat16()
    gate = torch.randn((M // 1024, N), generator=g, device=dev).bfloat16()
    outs = {}

    def run(kern):
        if epi is None:
            return K.lora_gemm(x, W, b, T, tp, r * Kd, r, 4.0, rpm, out=outs.setdefault(kern, torch.empty_like(res)),
                               kernel=kern)
        kw = dict(res=outs.setdefault(("r", kern), res.clone())) if epi != "silu" else \
            dict(out=outs.setdefault(kern, torch.empty_like(res)))
        if epi == "gated":
            kw.update(gate=gate, rows_per_group=1024)
        return K.lora_linear_pop_epi(x, W, b, tp, 0, r * Kd, r, 4.0, rpm, epi, kernel=kern, **kw)

    if epi != "gated":
        same = torch.equal(run(8), run(10))
    else:
        same = torch.equal(run(8).clone(), run(10).clone()) if False else None
    t = {8: [], 10: []}
    for _ in range(rounds):
        for kern in (8, 10):
            t[kern].append(bench(lambda: run(kern)))
    fl = 2.0 * M * N * Kd + 2.0 * M * N * r
    row = {"M": M, "N": N, "K": Kd, "r": r, "epi": epi, "bitexact": same}
    for kern in (8, 10):
        row[f"k{kern}_ms_min"] = round(min(t[kern]), 4)
        row[f"k{kern}_ms_med"] = round(statistics.median(t[kern]), 4)
        row[f"k{kern}_tflops"] = round(fl / min(t[kern]) / 1e9, 1)
    row["speedup"] = round(min(t[8]) / min(t[10]), 4)
    rows.append(row)
    print(json.dumps(row), flush=True)
if len(sys.argv) > 2:
    Path(sys.argv[2]).write_text(json.dumps(rows, indent=1))
