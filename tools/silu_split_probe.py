"""GLUMBConv's conv_inverted -> SiLU -> dw3x3 -> GLU at the epoch's shapes, two ways: SiLU in the GEMM
epilogue (lora_linear_pop_epi "silu" + dwconv pre_silu=False, the round-2 fusion) vs SiLU in the depthwise
conv's staging (plain GEMM + dwconv pre_silu=True).  Both compute silu of the bf16-rounded GEMM output with
the same device silu, so the dwconv outputs are compared bitwise.  HIP events, median of rounds.
usage: python tools/silu_split_probe.py   (diagnostic)"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402


def t(fn, it=3):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main(rounds=5):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    # (name, B, H, W, C_in, hidden(2h), ldo) : Sana FFN (2240 -> 11200, 32x32 x 128 images, GLU out padded
    # to 5632) and the DC-AE 512-channel GLUMBConv (512 -> 4096 at 128^2 x 8 images)
    for name, B, H, W, C, H2, ldo in (("sana_ffn", 128, 32, 32, 2240, 11200, 5632), ("dcae_512", 8, 128, 128, 512, 4096, 0)):
        x = (torch.randn(B * H * W, C, device=dev, generator=g) * 0.5).bfloat16()
        wi = (torch.randn(H2, C, device=dev, generator=g) * C ** -0.5).bfloat16()
        bi = (torch.randn(H2, device=dev, generator=g) * 0.1).bfloat16()
        wd = (torch.randn(9, H2, device=dev, generator=g) * 0.2).bfloat16()
        bd = (torch.randn(H2, device=dev, generator=g) * 0.1).bfloat16()
        M = B * H * W
        hbuf = torch.empty(M, H2, device=dev, dtype=torch.bfloat16)

        def fused():
            h = K.lora_linear_pop_epi(x, wi, bi, None, 0, 0, 0, 0.0, M, "silu", out=hbuf)
            return K.dwconv_nhwc(h.view(B, H, W, H2), wd, bd, 3, pre_silu=False, glu=True, ldo=ldo)

        def split():
            h = K.lora_linear_pop(x, wi, bi, None, 0, 0, 0, 0.0, M, out=hbuf)
            return K.dwconv_nhwc(h.view(B, H, W, H2), wd, bd, 3, pre_silu=True, glu=True, ldo=ldo)

        def gemm_epi():
            K.lora_linear_pop_epi(x, wi, bi, None, 0, 0, 0, 0.0, M, "silu", out=hbuf)

        def gemm_plain():
            K.lora_linear_pop(x, wi, bi, None, 0, 0, 0, 0.0, M, out=hbuf)
        h0 = K.lora_linear_pop(x, wi, bi, None, 0, 0, 0, 0.0, M).view(B, H, W, H2)

        def dw_pre():
            K.dwconv_nhwc(h0, wd, bd, 3, pre_silu=True, glu=True, ldo=ldo)

        def dw_plain():
            K.dwconv_nhwc(h0, wd, bd, 3, pre_silu=False, glu=True, ldo=ldo)
        same = torch.equal(fused().clone(), split().clone())
        res = {"bitwise_equal": same}
        for nm, fn in (("fused", fused), ("split", split), ("gemm_silu_epi", gemm_epi), ("gemm_plain", gemm_plain),
                       ("dw_pre_silu", dw_pre), ("dw_plain", dw_plain)):
            res[nm + "_us"] = round(statistics.median(t(fn) for _ in range(rounds)), 1)
        out[name] = res
        print(json.dumps({name: res}), flush=True)
        del x, hbuf, h0
    print(json.dumps(out))


if __name__ == "__main__":
    main()
