"""DC-AE decode time per image vs images per decoder call (the pipeline's vae_chunk): the full-size
Sana DC-AE f32c32 decoder (synthetic weights), 32 latents at 1024 px decoded in chunks of 4 / 8 / 16 / 32,
interleaved rounds; ms per 32 images.
usage: python tools/vae_chunk_probe.py [out.json]"""
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
    z = torch.randn(32, 32, 32, 32, device=dev)
    t = {c: [] for c in (8, 16, 32)}    # vae_chunk (images per decoder call); high-res stages chunk by 8
    for _ in range(3):
        for c in t:
            t[c].append(bench(lambda: [vae(z[s:s + c]) for s in range(0, 32, c)], it=2))
    out = {c: round(min(v), 2) for c, v in t.items()}
    out["peak_mem_GiB"] = round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)
print(json.dumps(out), flush=True)
if len(sys.argv) > 1:
    Path(sys.argv[1]).write_text(json.dumps(out, indent=1))
