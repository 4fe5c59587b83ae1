"""A/B of builds of libeggroll on the fused DC-AE decoder head (eggroll_dcae_head): bitwise equality of
the outputs (epoch shape 8 x 1024^2 x 128 and a ragged 3 x 100 x 70 one whose band count is not a
multiple of the bands-per-block), then interleaved timing at the epoch shape (median of rounds, HIP
events on the launch stream).
usage: python tools/head_lib_ab.py <libA.so> <libB.so> [<libC.so> ...]"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from es_lib_ab import bind, timed  # noqa: E402


def main(paths, rounds=9):
    libs = [bind(p) for p in paths]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)
    nw = (torch.rand(128, device=dev, generator=g) + 0.5).bfloat16()
    nb = (torch.randn(128, device=dev, generator=g) * 0.1).bfloat16()
    w = (torch.randn((3, 3, 3, 128), generator=g, device=dev) / 30).bfloat16().contiguous()
    cb = (torch.randn(3, device=dev, generator=g) * 0.1).bfloat16()
    out = {}
    for B, H, W in ((3, 100, 70), (8, 1024, 1024)):
        x = torch.randn((B, H, W, 128), generator=g, device=dev).bfloat16()
        ys = [torch.empty(B, H, W, 3, device=dev, dtype=torch.bfloat16) for _ in libs]

        def run(i):
            rc = libs[i].eggroll_dcae_head(x.data_ptr(), B, H, W, 128, 1e-5, nw.data_ptr(), nb.data_ptr(),
                                           w.data_ptr(), cb.data_ptr(), ys[i].data_ptr(), st)
            assert rc == 0, rc
        for i in range(len(libs)):
            run(i)
        torch.cuda.synchronize()
        same = [torch.equal(ys[0], y) for y in ys[1:]]
        key = f"{B}x{H}x{W}x128"
        rec = {"bitwise_equal_to_A": same}
        if H >= 512:
            us = [[] for _ in libs]
            for _ in range(rounds):
                for i in range(len(libs)):
                    us[i].append(timed(lambda: run(i)))
            med = [statistics.median(u) for u in us]
            rec.update({Path(p).name: {"us": round(m, 1), "TBps_in": round(x.numel() * 2 / m / 1e6, 3)}
                        for p, m in zip(paths, med)})
        out[key] = rec
        print(json.dumps({key: rec}), flush=True)
        assert all(same), key
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1:])
