"""Diagnostic for eggroll_conv3x3_nhwc: where (interior / border pixels) the kernel differs from torch,
for full and single-tap weights."""
import math
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
B, H, W, Cin, Cout = 1, 16, 16, 64, 64
x = torch.randn(B, H, W, Cin, generator=g).to(dev, torch.bfloat16)
wfull = (torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)).to(dev, torch.bfloat16)
for name, taps in [("full", None), ("center", [(1, 1)]), ("tap00", [(0, 0)]), ("tap22", [(2, 2)]), ("tap01", [(0, 1)])]:
    w = wfull.clone()
    if taps is not None:
        m = torch.zeros(3, 3, device=dev, dtype=torch.bfloat16)
        for a, b in taps:
            m[a, b] = 1
        w = w * m
    for px in (1, 2):
        y = K.conv3x3_nhwc(x, K.pack_conv3x3_weight(w, px), None, px, None).float()
        ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), None, padding=1).permute(0, 2, 3, 1)
        e = (y - ref).abs().amax(dim=-1)[0]  # [H, W]
        bad = e > 1e-2 * ref.abs().max()
        border = torch.zeros(H, W, dtype=torch.bool, device=dev)
        border[0, :] = border[-1, :] = True
        border[:, 0] = border[:, -1] = True
        print(f"{name:7s} px{px}: bad interior {int((bad & ~border).sum())}/{int((~border).sum())}, "
              f"bad border {int((bad & border).sum())}/{int(border.sum())}, max err {e.max().item():.3e}", flush=True)
        if name == "center" and px == 1:
            rows = bad.nonzero()[:8].tolist()
            print("   first bad (y,x):", rows, flush=True)
            if rows:
                yy, xx = rows[0]
                print("   ours", y[0, yy, xx, :6].tolist(), "\n   ref ", ref[0, yy, xx, :6].tolist(), flush=True)
