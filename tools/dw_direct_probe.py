"""3x3 depthwise conv at the epoch's shapes: the LDS-tiled kernel (0, automatic) vs the direct register-
window kernel (3), HIP events, median of rounds, bitwise equality, HBM fraction of the algorithmic bytes
(diagnostic).  usage: python tools/dw_direct_probe.py"""
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


for B, H, W, C, pre, glu, ldo in ((128, 32, 32, 11200, False, True, 5632), (8, 128, 128, 4096, False, True, 0),
                                  (8, 64, 64, 8192, True, True, 0), (8, 32, 32, 8192, True, True, 0),
                                  (4, 40, 24, 320, False, False, 0), (2, 9, 13, 1024, True, False, 0)):
    g = torch.Generator(device=dev).manual_seed(C + H)
    x = torch.randn(B, H, W, C, generator=g, device=dev).bfloat16()
    w = (torch.randn(9, C, generator=g, device=dev) * 0.2).bfloat16()
    b = (torch.randn(C, generator=g, device=dev) * 0.1).bfloat16()
    r = {0: [], 3: []}
    for _ in range(4):
        for k in (0, 3):
            r[k].append(t(lambda: K.dwconv_nhwc(x, w, b, 3, pre, glu, kernel=k, ldo=ldo)))
    a = K.dwconv_nhwc(x, w, b, 3, pre, glu, kernel=0, ldo=ldo)
    d = K.dwconv_nhwc(x, w, b, 3, pre, glu, kernel=3, ldo=ldo)
    co = C // 2 if glu else C
    nbytes = 2.0 * B * H * W * (C + (ldo or co))
    m0, m3 = statistics.median(r[0]), statistics.median(r[3])
    print(json.dumps({f"{B}x{H}x{W}x{C} pre{int(pre)} glu{int(glu)} ldo{ldo}": {
        "k0_us": round(m0, 1), "k3_us": round(m3, 1), "k3_vs_k0": round(m0 / m3, 3),
        "k0_frac_hbm": round(nbytes / m0 / 8e6, 3), "k3_frac_hbm": round(nbytes / m3 / 8e6, 3),
        "bitwise_equal": bool(torch.equal(a, d))}}), flush=True)
