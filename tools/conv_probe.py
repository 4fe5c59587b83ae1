"""Diagnostic: MIOpen conv throughput for the Sana/DC-AE conv shapes under different settings."""
import os, sys, json, time
mode = sys.argv[1] if len(sys.argv) > 1 else "fast"
if mode == "fast":
    os.environ["MIOPEN_FIND_MODE"] = "FAST"
import torch, torch.nn.functional as F
torch.backends.cudnn.benchmark = (mode == "bench")
dev = torch.device("cuda:0")

def t(fn, it=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it

cases = [("dense3x3_128_1024px_b8", 8, 128, 128, 1024, 3, 1),
         ("dense3x3_256_512px_b8", 8, 256, 256, 512, 3, 1),
         ("dense3x3_512_256px_b8", 8, 512, 512, 256, 3, 1),
         ("dw3x3_11200_32px_b128", 128, 11200, 11200, 32, 3, 11200),
         ("dw3x3_8192_32px_b8", 8, 8192, 8192, 32, 3, 8192),
         ("dw5x5_3072_128px_b8", 8, 3072, 3072, 128, 5, 3072)]
for name, B, ci, co, hw, k, g in cases:
    for cl in (True, False):
        x = torch.randn(B, ci, hw, hw, device=dev, dtype=torch.bfloat16)
        if cl: x = x.contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, ci // g, k, k, device=dev, dtype=torch.bfloat16) * 0.05
        if cl: w = w.contiguous(memory_format=torch.channels_last)
        try:
            ms = t(lambda: F.conv2d(x, w, None, padding=k // 2, groups=g))
        except Exception as ex:
            ms = float("nan")
        fl = 2 * B * co * (ci // g) * k * k * hw * hw
        by = 2 * (x.numel() + B * co * hw * hw)
        print(json.dumps(dict(mode=mode, case=name, channels_last=cl, ms=ms, tflops=fl / ms / 1e9, GBps=by / ms / 1e6)), flush=True)
