"""A/B of two builds of libeggroll on the softmax cross-attention kernel (eggroll_cross_attention) at
the epoch's shapes: Sana attn2 (128 images x 1024 queries x 20 heads x 112, 300 caption keys shared by
32 images each through enc_index, masked) and the CLIP towers' self-attention (CLIP-H/14: 128 x 257 x 16
heads x 80; CLIP-B/32: 128 x 50 x 12 x 64).  Bitwise comparison (with --tol: the largest difference
from A in bf16 ulps of the output and vs an fp32 softmax reference instead), then interleaved timing.
usage: python tools/xattn_lib_ab.py <libA.so> <libB.so> [--tol]"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from es_lib_ab import bind, timed  # noqa: E402


def main(pa, pb, rounds=7, tol=False):
    libs = [bind(pa), bind(pb)]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(2)
    out = {}
    for B, N, heads, hd, L, U in ((128, 1024, 20, 112, 300, 4), (128, 257, 16, 80, 257, 128), (128, 50, 12, 64, 50, 128)):
        q = torch.randn(B * N, heads * hd, device=dev, generator=g).bfloat16()
        k = torch.randn(U * L, heads * hd, device=dev, generator=g).bfloat16()
        v = torch.randn(U * L, heads * hd, device=dev, generator=g).bfloat16()
        cross = U != B
        bias = torch.where(torch.rand(U, L, device=dev, generator=g) < 0.2, -1e4, 0.0).bfloat16() if cross else None
        enc = (torch.arange(B, device=dev, dtype=torch.int32) // (B // U)).contiguous() if cross else None
        ys = [torch.empty(B * N, heads * hd, device=dev, dtype=torch.bfloat16) for _ in libs]

        def run(i):
            rc = libs[i].eggroll_cross_attention(q.data_ptr(), q.stride(0), k.data_ptr(), v.data_ptr(), k.stride(0),
                                                 bias.data_ptr() if bias is not None else None,
                                                 enc.data_ptr() if enc is not None else None, B, N, heads, hd, L, U,
                                                 hd ** -0.5, ys[i].data_ptr(), ys[i].stride(0), st)
            assert rc == 0, rc
        run(0)
        run(1)
        torch.cuda.synchronize()
        same = torch.equal(ys[0], ys[1])
        us = [[], []]
        for _ in range(rounds):
            for i in (0, 1):
                us[i].append(timed(lambda: run(i)))
        a, b = statistics.median(us[0]), statistics.median(us[1])
        key = f"B{B} N{N} h{heads}x{hd} L{L}"
        out[key] = {"A_us": round(a, 1), "B_us": round(b, 1), "B_vs_A": round(a / b, 4), "bitwise_equal": same}
        if tol:
            # fp32 reference on a sample of images
            nb = 4
            qf = q.view(B, N, heads, hd)[:nb].float().transpose(1, 2)
            uu = enc[:nb].long() if enc is not None else torch.arange(nb, device=dev)
            kf = k.view(U, L, heads, hd)[uu].float().transpose(1, 2)
            vf = v.view(U, L, heads, hd)[uu].float().transpose(1, 2)
            sc = qf @ kf.transpose(-1, -2) * hd ** -0.5
            if bias is not None:
                sc = sc + bias.float()[uu][:, None, None, :]
            ref = (sc.softmax(-1) @ vf).transpose(1, 2).reshape(nb * N, heads * hd)
            for i, nm in ((0, "A"), (1, "B")):
                e = (ys[i][:nb * N].float() - ref).abs()
                out[key][f"{nm}_max_err_vs_fp32"] = float(e.max())
                out[key][f"{nm}_mean_err_vs_fp32"] = float(e.mean())
            out[key]["A_B_max_diff"] = float((ys[0].float() - ys[1].float()).abs().max())
        print(json.dumps({key: out[key]}), flush=True)
        assert same or tol, key
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], tol="--tol" in sys.argv[3:])
