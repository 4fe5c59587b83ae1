"""Same-process A/B of the halo-staged 3x3 conv: kernel 2 (one tile per workgroup, halo rows padded to 8
pixels), kernel 3 (the same, unpadded round-2 layout) and kernel 4 (one workgroup streams a stack of
tiles, the next tile's halo + weights prefetched during the epilogue) at
the DC-AE decoder's ResBlock shapes (8 images), plain / bias+SiLU / RMSNorm+residual; interleaved
rounds, median ms; bitwise equality of the two kernels checked on every shape.
usage: python tools/halo_mt_probe.py [rounds]"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5


def t(fn, it=5):
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


out = {}
for B, C, hw in [(8, 128, 1024), (8, 256, 512), (8, 512, 256)]:
    g = torch.Generator(device=dev).manual_seed(C)
    x = torch.randn(B, hw, hw, C, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5).to(torch.bfloat16)
    b = torch.randn(C, device=dev, generator=g).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(C, device=dev, generator=g)).to(torch.bfloat16)
    nb = (0.1 * torch.randn(C, device=dev, generator=g)).to(torch.bfloat16)
    res = torch.randn(B, hw, hw, C, device=dev, generator=g).to(torch.bfloat16)
    wp = K.pack_conv3x3_weight(w, 1)
    fl = 2.0 * B * hw * hw * C * C * 9
    o2, o4 = torch.empty_like(x), torch.empty_like(x)
    ks = (2, 3, 4)   # padded one-tile, unpadded one-tile (round 2), multi-tile
    cases = {
        "plain": lambda o, k: K.conv3x3_nhwc(x, wp, None, 1, None, out=o, kernel=k),
        "bias_silu": lambda o, k: K.conv3x3_nhwc(x, wp, b, 1, "silu", out=o, kernel=k),
    }
    if C in (128, 256):  # (allocates its output: the caching allocator hands back the same block)
        cases["rmsnorm_res"] = lambda o, k: K.conv3x3_rmsnorm_nhwc(x, wp, b, 1, 1e-5, nw, nb, res, kernel=k)
    row = {}
    for name, fn in cases.items():
        ys = {k: fn(o2 if k == 2 else o4, k).clone() for k in ks}
        torch.cuda.synchronize()
        same = all(bool(torch.equal(ys[2], ys[k])) for k in ks)
        del ys
        ms = {k: [] for k in ks}
        for _ in range(rounds):
            for k in ks:
                ms[k].append(t(lambda: fn(o2 if k == 2 else o4, k)))
        med = {k: statistics.median(v) for k, v in ms.items()}
        row[name] = {**{f"k{k}_ms": round(med[k], 4) for k in ks}, **{f"k{k}_tflops": round(fl / med[k] / 1e9, 1) for k in ks},
                     "bitexact": same}
        print(f"[halo-mt] {B}x{hw}x{hw}x{C} {name}: {row[name]}", flush=True)
    out[f"{B}x{hw}x{hw}x{C}"] = row
print(json.dumps(out))
