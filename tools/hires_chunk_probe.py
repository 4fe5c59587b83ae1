"""DC-AE decode time vs images per call of the two high-resolution stages (DCAEDecoder.hi_res_chunk):
at 8 images one 1024^2 x 128 activation is 2.15 GB (streamed from HBM by every conv); at 1 image it is
268 MB, near the 256-MB MALL, so a ResBlock's intermediate may be re-read from the last-level cache.
Full-size Sana DC-AE f32c32 decoder (synthetic weights), 16 latents at 1024 px (one member's images),
interleaved rounds; outputs compared bitwise to hi_res_chunk 8 (the kernels are per-image).
usage: python tools/hires_chunk_probe.py [out.json]"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd.dcae import DCAEDecoder  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
with torch.no_grad():
    vae = DCAEDecoder().to(dev)
    vae.init_weights(1)
    z = torch.randn(16, 32, 32, 32, device=dev)
    ref = None
    same = {}
    t = {c: [] for c in (8, 4, 2, 1)}
    for c in t:
        vae.hi_res_chunk = c
        y = vae(z)
        if ref is None:
            ref = y.clone()
        same[c] = bool(torch.equal(y, ref))
        del y
    for _ in range(3):
        for c in t:
            vae.hi_res_chunk = c
            t[c].append(bench(lambda: vae(z), it=2))
    out = {"ms_per_16_images": {c: round(min(v), 2) for c, v in t.items()}, "bitwise_equal_to_8": same,
           "peak_mem_GiB": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)}
print(json.dumps(out), flush=True)
if len(sys.argv) > 1:
    Path(sys.argv[1]).write_text(json.dumps(out, indent=1))
