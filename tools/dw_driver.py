"""Runs the epoch's depthwise-conv launches at their product shapes a few times, for rocprofv3 --pmc /
--kernel-trace passes on k_dwconv_nhwc (tools/pmc_dw.sh, tools/pmc_dw_summary.py):
  Sana FFN           128 x 32 x 32 x 11200, dw3x3 -> GLU (SiLU fused upstream)     k_dwconv_nhwc<3,0,1>
  DC-AE GLUMBConv    8 x 128 x 128 x 4096,  dw3x3 -> GLU                             k_dwconv_nhwc<3,0,1>
  DC-AE GLUMBConv    8 x 64 x 64 x 8192,    SiLU -> dw3x3 -> GLU                     k_dwconv_nhwc<3,1,1>
  DC-AE LiteMLA agg  8 x 128 x 128 x 1536,  dw5x5 -> grouped 1x1                     k_dwconv_nhwc<5,0,0,1>
usage: python tools/dw_driver.py [reps]   (diagnostic)"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

SHAPES = ((128, 32, 32, 11200, 3, False, True), (8, 128, 128, 4096, 3, False, True),
          (8, 64, 64, 8192, 3, True, True), (8, 128, 128, 1536, 5, False, False))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    for B, H, W, C, ks, pre, glu in SHAPES:
        x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(ks * ks, C, device=dev) * 0.2).to(torch.bfloat16)
        b = (torch.randn(C, device=dev) * 0.1).to(torch.bfloat16)
        if glu:
            out = torch.empty(B, H, W, C // 2, device=dev, dtype=torch.bfloat16)
            for _ in range(reps):
                K.dwconv_nhwc(x, w, b, ks, pre_silu=pre, glu=True, out=out)
        else:
            pw = (torch.randn(C // 32, 32, 32, device=dev) * 0.2).to(torch.bfloat16)
            out = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
            for _ in range(reps):
                K.dwconv_pw_nhwc(x, w, pw, ks, out=out)
        del x, out
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
