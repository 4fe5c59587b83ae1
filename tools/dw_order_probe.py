"""Same-process A/B of the depthwise conv's block order (eggroll_dwconv_nhwc_sel / _pw_nhwc_sel kernel 1 =
channel slice fastest, 2 = column sweep) at the epoch's shapes; interleaved rounds, median us, bitwise
equality of the two orders, HBM fraction of the algorithmic bytes (input read once, output written once).
usage: python tools/dw_order_probe.py [rounds]"""
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
    return s.elapsed_time(e) / it * 1e3


out = {}
cases = [("glu", 128, 32, 32, 11200, 3, False), ("glu", 8, 128, 128, 4096, 3, False), ("glu", 8, 64, 64, 8192, 3, True),
         ("glu", 8, 32, 32, 8192, 3, True), ("pw", 8, 128, 128, 1536, 5, False), ("pw", 8, 64, 64, 3072, 5, False),
         ("pw", 8, 32, 32, 3072, 5, False)]
for kind, B, H, W, C, ks, pre in cases:
    g = torch.Generator(device=dev).manual_seed(C + H)
    x = torch.randn(B, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(ks * ks, C, device=dev, generator=g) * 0.2).to(torch.bfloat16)
    if kind == "glu":
        b = (torch.randn(C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        o1, o2 = (torch.empty(B, H, W, C // 2, device=dev, dtype=torch.bfloat16) for _ in range(2))
        fn = lambda o, k: K.dwconv_nhwc(x, w, b, ks, pre, True, out=o, kernel=k)  # noqa: E731
        nbytes = 2.0 * B * H * W * (C + C // 2)
    else:
        pw = (torch.randn(C // 32, 32, 32, device=dev, generator=g) / 32 ** 0.5).to(torch.bfloat16)
        o1, o2 = torch.empty_like(x), torch.empty_like(x)
        fn = lambda o, k: K.dwconv_pw_nhwc(x, w, pw, ks, out=o, kernel=k)  # noqa: E731
        nbytes = 4.0 * B * H * W * C
    fn(o1, 1)
    fn(o2, 2)
    torch.cuda.synchronize()
    same = bool(torch.equal(o1, o2))
    us = {1: [], 2: []}
    for _ in range(rounds):
        for k in (1, 2):
            us[k].append(t(lambda: fn(o1 if k == 1 else o2, k)))
    m1, m2 = statistics.median(us[1]), statistics.median(us[2])
    key = f"{kind}{ks} {B}x{H}x{W}x{C}"
    out[key] = {"order1_us": round(m1, 1), "order2_us": round(m2, 1), "order1_frac": round(nbytes / m1 / 8e6, 3),
                "order2_frac": round(nbytes / m2 / 8e6, 3), "speedup": round(m1 / m2, 3), "bitexact": same}
    print(f"[dw-order] {key}: {out[key]}", flush=True)
print(json.dumps(out))
