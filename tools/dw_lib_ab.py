"""A/B of two builds of libeggroll on the depthwise convs (eggroll_dwconv_nhwc_sel / _pw_nhwc_sel) at the
epoch's shapes: Sana GLUMBConv (128 x 32 x 32 x 11200, GLU), DC-AE GLUMBConv (8 x 128 x 128 x 4096 GLU,
8 x 64 x 64 x 8192 GLU + SiLU on the input) and the multi-scale attention's fused dw5x5 + grouped 1x1
(8 x 128 x 128 x 1536).  Outputs compared bitwise, then interleaved timing (median of rounds).
usage: python tools/dw_lib_ab.py <libA.so> <libB.so>"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import _lib  # noqa: E402
from es_lib_ab import bind, timed  # noqa: E402


def main(pa, pb, rounds=7):
    libs = [bind(pa), bind(pb)]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(1)
    out = {}
    for B, H, W, C, ks, pre, glu, pw in ((128, 32, 32, 11200, 3, 0, 1, False), (128, 32, 32, 11200, 3, 1, 1, False),
                                         (8, 128, 128, 4096, 3, 0, 1, False), (8, 128, 128, 4096, 3, 1, 1, False),
                                         (8, 64, 64, 8192, 3, 1, 1, False), (8, 128, 128, 1536, 5, 0, 0, True)):
        x = torch.randn(B, H, W, C, device=dev, generator=g).bfloat16()
        w = (torch.randn(ks * ks, C, device=dev, generator=g) * 0.2).bfloat16()
        b = torch.randn(C, device=dev, generator=g).bfloat16()
        pwt = (torch.randn(C // 32, 32, 32, device=dev, generator=g) * 0.2).bfloat16()
        co = C // 2 if glu else C
        ys = [torch.empty(B, H, W, co, device=dev, dtype=torch.bfloat16) for _ in libs]

        def run(i):
            if pw:
                rc = libs[i].eggroll_dwconv_pw_nhwc_sel(x.data_ptr(), w.data_ptr(), pwt.data_ptr(), B, H, W, C, ks,
                                                        ys[i].data_ptr(), 0, st)
            else:
                rc = libs[i].eggroll_dwconv_nhwc_sel(x.data_ptr(), w.data_ptr(), b.data_ptr(), B, H, W, C, ks, pre, glu,
                                                     ys[i].data_ptr(), 0, st)
            assert rc == 0, rc
        run(0)
        run(1)
        torch.cuda.synchronize()
        same = torch.equal(ys[0], ys[1])
        us = [[], []]
        for _ in range(rounds):
            for i in (0, 1):
                us[i].append(timed(lambda: run(i)))
        a, bb = statistics.median(us[0]), statistics.median(us[1])
        byt = 2.0 * B * H * W * (C + co)
        key = f"{B}x{H}x{W}x{C} ks{ks} pre{pre} glu{glu}{' pw' if pw else ''}"
        out[key] = {"A_us": round(a, 1), "B_us": round(bb, 1), "B_vs_A": round(a / bb, 4),
                    "B_frac_hbm": round(byt / bb / 8e6, 3), "bitwise_equal": same}
        print(json.dumps({key: out[key]}), flush=True)
        if not same:
            d = (ys[0].float() - ys[1].float()).abs()
            print(json.dumps({key: {"max_abs_diff": float(d.max()), "n_diff": int((d > 0).sum()), "numel": d.numel(), "max_rel": float((d / ys[0].float().abs().clamp_min(1e-3)).max())}}), flush=True)
        del x, ys
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
