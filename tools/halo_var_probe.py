"""DC-AE 3x3 convs at the epoch shapes (8 images): tap-staged (1) vs halo 512x128 / 256x256 (2) vs
halo 256x128 two-workgroups-per-CU (3), plain / SiLU / RMSNorm+residual tails.  TFLOP/s per variant."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def t(fn, it=6):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(5_000_000)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


KERNS = tuple(int(k) for k in (sys.argv[sys.argv.index("--kernels") + 1].split(",") if "--kernels" in sys.argv else "1,2,3".split(",")))
shapes = [(8, 1024, 128)] + ([(8, 512, 256), (8, 256, 512)] if "--all" in sys.argv else [])
for B, hw, C in shapes:
    x = torch.randn(B, hw, hw, C, device=dev, dtype=torch.bfloat16)
    res = torch.randn(B, hw, hw, C, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16)
    nw = torch.randn(C, device=dev).to(torch.bfloat16)
    nb = torch.randn(C, device=dev).to(torch.bfloat16)
    bias = torch.randn(C, device=dev).to(torch.bfloat16)
    wp = K.pack_conv3x3_weight(w, 1)
    y = torch.empty_like(x)
    flop = 2.0 * B * hw * hw * C * C * 9
    row = {"shape": [B, hw, hw, C]}
    ref = None
    for kern in KERNS:
        for tail in ("plain", "silu", "norm"):
            if tail == "norm":
                fn = lambda: K.conv3x3_rmsnorm_nhwc(x, wp, None, 1, 1e-5, nw, nb, res, kernel=kern)  # noqa: E731
            else:
                fn = lambda: K.conv3x3_nhwc(x, wp, None, 1, "silu" if tail == "silu" else None, out=y, kernel=kern)  # noqa: E731
            try:
                ms = t(fn)
            except Exception as ex:  # a variant that does not apply to the shape
                row[f"k{kern}_{tail}"] = str(ex)[:60]
                continue
            row[f"k{kern}_{tail}_ms"] = round(ms, 3)
            row[f"k{kern}_{tail}_TF"] = round(flop / ms * 1e-9, 1)
        if kern in (2, 3, 4):
            outs = [K.conv3x3_nhwc(x, wp, bias, 1, act, kernel=kern) for act in (None, "silu")]
            try:
                outs.append(K.conv3x3_rmsnorm_nhwc(x, wp, None, 1, 1e-5, nw, nb, res, kernel=kern))
            except Exception:
                pass
            ref = outs if ref is None else ref
            row[f"k{kern}_vs_first_maxdiff"] = [float((a.float() - r.float()).abs().max()) for a, r in zip(outs, ref)]
    print(json.dumps(row), flush=True)
