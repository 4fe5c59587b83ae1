"""eggroll_flash_attention vs SDPA (aotriton) at the Z-Image main-stack shape and Infinity's last-scale
KV-cache shape: median us, TF/s, relative error vs fp32 (diagnostic).
usage: python tools/flash_probe.py"""
import json
import statistics
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

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


out = {}
for name, B, Nq, Lk, H, ltot in (("zimage_main", 64, 676, 676, 30, 676), ("infinity_last", 64, 1024, 2521, 28, 2521),
                                 ("infinity_s7", 64, 400, 921, 28, 2521)):
    g = torch.Generator(device=dev).manual_seed(0)
    q = (torch.randn(B, Nq, H, 128, generator=g, device=dev) * 0.3).bfloat16()
    cache = (torch.randn(2, B, ltot, H * 128, generator=g, device=dev) * 0.3).bfloat16()
    k, v = cache[0, :, :Lk].view(B, Lk, H, 128), cache[1, :, :Lk].view(B, Lk, H, 128)
    sc = 128 ** -0.5
    fa = lambda: K.flash_attention(q, k, v, sc, qf=2)  # noqa: E731
    fa4 = lambda: K.flash_attention(q, k, v, sc, qf=1)  # noqa: E731  (the A/B variant: 16 queries per wave)
    sd = lambda: F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=sc)  # noqa: E731
    r = {"fa": [], "fa4": [], "sdpa": []}
    for _ in range(5):
        r["fa"].append(t(fa))
        r["fa4"].append(t(fa4))
        r["sdpa"].append(t(sd))
    fl = 4.0 * B * H * Nq * Lk * 128
    a, b = fa().float(), sd().transpose(1, 2).float()
    out[name] = {k_: round(statistics.median(v_), 1) for k_, v_ in r.items()}
    a4 = fa4().float()
    out[name].update({"fa4_tflops": round(fl / out[name]["fa4"] / 1e6, 1), "fa4_rel_err": ((a4 - b).norm() / b.norm()).item(),
                      "fa_tflops": round(fl / out[name]["fa"] / 1e6, 1), "sdpa_tflops": round(fl / out[name]["sdpa"] / 1e6, 1),
                      "rel_err_vs_sdpa": ((a - b).norm() / b.norm()).item()})
    print(json.dumps({name: out[name]}), flush=True)
