"""DC-AE up-blocks at the epoch's shapes: phase conv + sub-pixel interleave/shortcut as two launches
(conv_nhwc ks 2 + subpixel_shortcut[_f32]) vs one (conv2x2_subpixel), bf16 and fp32-stream forms; outputs
compared bitwise, HIP events, median of rounds.
usage: python tools/subpix_fuse_probe.py   (diagnostic)"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from hyperscalees_t2i_amd.dcae import subpixel_phase_weights  # noqa: E402


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
    for B, H, W, cin, cout in ((8, 512, 512, 256, 128), (8, 256, 256, 512, 256), (8, 128, 128, 512, 512),
                               (8, 64, 64, 1024, 512)):
        w3 = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * (9 * cin) ** -0.5
        wp = K.pack_conv3x3_weight(subpixel_phase_weights(w3).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last), 1)
        bias = (torch.randn(cout, device=dev, generator=g) * 0.1).bfloat16()
        x = torch.randn(B, H, W, cin, device=dev, generator=g).bfloat16()
        for f32 in (False, True):
            src = x.float() if f32 else x
            sh = torch.empty(B, 2 * H, 2 * W, cout, device=dev, dtype=torch.bfloat16) if f32 else None
            sh2 = torch.empty_like(sh) if f32 else None

            def two():
                y4 = K.conv_nhwc(x, wp, None, 2)
                return (K.subpixel_shortcut_f32(y4, src, bias=bias, shadow=sh) if f32
                        else K.subpixel_shortcut(y4, x, bias=bias))

            def one():
                return K.conv2x2_subpixel(x, wp, src, bias=bias, shadow=sh2)
            same = torch.equal(two(), one()) and (not f32 or torch.equal(sh, sh2))
            a = statistics.median(t(two) for _ in range(rounds))
            b = statistics.median(t(one) for _ in range(rounds))
            key = f"{B}x{H}x{W}x{cin}->{cout} {'f32' if f32 else 'bf16'}"
            out[key] = {"two_launch_us": round(a, 1), "fused_us": round(b, 1), "speedup": round(a / b, 4),
                        "bitwise_equal": same}
            print(json.dumps({key: out[key]}), flush=True)
        del x, src
    print(json.dumps(out))


if __name__ == "__main__":
    main()
