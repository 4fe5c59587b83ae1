"""Implicit-GEMM 3x3 conv (eggroll_conv3x3_nhwc) vs MIOpen (F.conv2d, channels-last, cudnn.benchmark)
at the DC-AE decoder's ResBlock shapes (8 images of 1024 px), plus the fused bias+SiLU variant vs
MIOpen conv + eggroll bias_act.  usage: python tools/conv_gemm_probe.py"""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")


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


for B, C, hw, pxs in [(8, 128, 1024, (2, 1)), (8, 256, 512, (1, 2)), (8, 512, 256, (1,))]:
    x = torch.randn(B, hw, hw, C, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    b = torch.randn(C, device=dev).to(torch.bfloat16)
    fl = 2.0 * B * hw * hw * C * C * 9
    xn = x.permute(0, 3, 1, 2)
    ms_m = t(lambda: F.conv2d(xn, w, None, padding=1))
    y = F.conv2d(xn, w, None, padding=1).permute(0, 2, 3, 1).contiguous()
    ms_ba = t(lambda: K.bias_act_(y, b, "silu"))
    row = {"shape": f"{B}x{hw}x{hw}x{C}", "miopen_ms": round(ms_m, 3), "miopen_tflops": round(fl / ms_m / 1e9, 1),
           "bias_act_ms": round(ms_ba, 3)}
    for px in pxs:
        wp = K.pack_conv3x3_weight(w, px)
        out = torch.empty_like(x)
        if px == 1:  # tap-staged (1) vs halo-staged (2) kernel
            for kern in (1, 2, 3):
                ms_k = t(lambda: K.conv3x3_nhwc(x, wp, None, px, None, out=out, kernel=kern))
                row[f"k{kern}_ms"] = round(ms_k, 3)
                row[f"k{kern}_tflops"] = round(fl / ms_k / 1e9, 1)
        ms = t(lambda: K.conv3x3_nhwc(x, wp, None, px, None, out=out))
        ms_f = t(lambda: K.conv3x3_nhwc(x, wp, b.repeat(px), px, "silu", out=out))
        ref = F.conv2d(xn.float()[:1], w.float(), None, padding=1).permute(0, 2, 3, 1)
        K.conv3x3_nhwc(x, wp, None, px, None, out=out)
        err = (out[:1].float() - ref).abs().max().item() / ref.abs().max().item()
        row[f"px{px}_ms"] = round(ms, 3)
        row[f"px{px}_tflops"] = round(fl / ms / 1e9, 1)
        row[f"px{px}_bias_silu_ms"] = round(ms_f, 3)
        row[f"px{px}_relerr"] = float(f"{err:.2e}")
        if wp.shape[0] == 256 or (px == 1 and C == 128):  # conv2 + RMSNorm + residual fused
            nw = torch.ones(C, device=dev, dtype=torch.bfloat16)
            row[f"px{px}_norm_ms"] = round(t(lambda: K.conv3x3_rmsnorm_nhwc(x, wp, None, px, 1e-5, nw, nw, x)), 3)
            if px == 1:
                for kern in (1, 3) if C == 128 else (1,):
                    row[f"k{kern}_norm_ms"] = round(t(lambda: K.conv3x3_rmsnorm_nhwc(x, wp, None, px, 1e-5, nw, nw, x,
                                                                                      kernel=kern)), 3)
            row["rownorm_ms"] = round(t(lambda: K.rownorm(out, 1e-5, layer=False, w=nw, b=nw, res=x)), 3)
    print(json.dumps(row), flush=True)
    del x, y, out


# DC-AE up-block sub-pixel phase convs (2x2, pad 1, 4*Cout outputs) at the bench's 8-image batch
for B, cin, cout, hw in [(8, 256, 128, 512), (8, 512, 256, 256), (8, 512, 512, 128), (8, 1024, 512, 64)]:
    x = torch.randn(B, hw, hw, cin, device=dev, dtype=torch.bfloat16)
    w4 = (torch.randn(4 * cout, cin, 2, 2, device=dev) / (4 * cin) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    fl = 2.0 * B * (hw + 1) ** 2 * 4 * cout * 4 * cin
    xn = x.permute(0, 3, 1, 2)
    ms_m = t(lambda: F.conv2d(xn, w4, None, padding=1))
    wp = K.pack_conv3x3_weight(w4, 1)
    ms = t(lambda: K.conv_nhwc(x, wp, None, 2))
    print(json.dumps({"upblock": f"{B}x{hw}x{hw}x{cin}->{4 * cout}", "miopen_ms": round(ms_m, 3),
                      "miopen_tflops": round(fl / ms_m / 1e9, 1), "ours_ms": round(ms, 3),
                      "ours_tflops": round(fl / ms / 1e9, 1)}), flush=True)
