"""GroupNorm(32) + SiLU on NHWC bf16 activations (the FLUX / Infinity VAE decoders): the current fp32
torch restatement (flux_vae.GroupNorm) vs F.group_norm on the channels-last view (+ silu_), median us
and max difference (diagnostic).
usage: python tools/gn_probe.py"""
import json
import statistics
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd.dcae import nchw, nhwc  # noqa: E402
from hyperscalees_t2i_amd.flux_vae import GroupNorm  # noqa: E402

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


for B, H, W, C in ((16, 384, 384, 128), (16, 192, 192, 256), (16, 512, 512, 160), (16, 128, 128, 640)):
    x = (torch.randn(B, H, W, C, device=dev) * 2 + 0.5).bfloat16()
    gn = GroupNorm(C).to(dev)
    with torch.no_grad():
        gn.weight.copy_(1 + 0.1 * torch.randn(C, device=dev))
        gn.bias.copy_(0.1 * torch.randn(C, device=dev))
    gn.use_kernel = False
    a = lambda: gn(x)  # noqa: E731
    b = lambda: nhwc(F.silu(F.group_norm(nchw(x), 32, gn.weight, gn.bias, gn.eps)))  # noqa: E731
    from hyperscalees_t2i_amd import kernels as K
    c = lambda: K.group_norm_nhwc(x, 32, gn.weight, gn.bias, gn.eps, silu=True)  # noqa: E731
    r = {"torch_fp32": [], "group_norm_cl": [], "eggroll": []}
    for _ in range(3):
        r["torch_fp32"].append(t(a))
        r["group_norm_cl"].append(t(b))
        r["eggroll"].append(t(c))
    ya, yb, yc = a().float(), b().float(), c().float()
    print(json.dumps({f"{B}x{H}x{W}x{C}": {k: round(statistics.median(v), 1) for k, v in r.items()},
                      "max_abs_diff": (ya - yb).abs().max().item(), "eggroll_max_abs_diff": (ya - yc).abs().max().item(),
                      "eggroll_GBps": round(3 * x.numel() * 2 / statistics.median(r["eggroll"]) / 1e3, 1), "out_contig_cl": b().is_contiguous()}), flush=True)
