"""Per-call census of the DC-AE decoder's dense convs (MIOpen via F.conv2d) at the bench shape:
8 images, 1024 px output.  Times every F.conv2d call of one decode with HIP events (after a warm-up
decode so MIOpen Find has run) and prints shape, bias flag, FLOP and TF/s.  (diagnostic)
usage: python tools/conv_census.py"""
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd.dcae import DCAEDecoder  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
with torch.device(dev):
    vae = DCAEDecoder(32)
vae.init_weights(1)
z = torch.randn(8, 32, 32, 32, device=dev)
_conv = F.conv2d
records = []


def timed_conv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    y = _conv(x, w, b, stride, padding, dilation, groups)
    e1.record()
    records.append((tuple(x.shape), tuple(w.shape), b is not None, groups, e0, e1, y.shape))
    return y


F.conv2d = timed_conv
with torch.no_grad():
    for it in range(3):
        records.clear()
        vae(z)
    torch.cuda.synchronize()
agg = defaultdict(lambda: [0, 0.0, 0.0])
for xs, ws, hb, g, e0, e1, ys in records:
    ms = e0.elapsed_time(e1)
    fl = 2.0 * ys[0] * ys[2] * ys[3] * ws[0] * ws[1] * ws[2] * ws[3]
    k = (xs, ws, hb, g)
    agg[k][0] += 1
    agg[k][1] += ms
    agg[k][2] += fl
tot = sum(v[1] for v in agg.values())
print(f"total conv ms per decode: {tot:.2f}")
for (xs, ws, hb, g), (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(json.dumps({"x": xs, "w": ws, "bias": hb, "groups": g, "n": n, "ms": round(ms, 3),
                      "tflops": round(fl / ms / 1e9, 1)}))
