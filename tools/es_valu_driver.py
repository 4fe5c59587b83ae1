"""Launch the engine-default (seeded) ES kernels back to back for rocprofv3 PMC / kernel-trace passes:
eggroll_perturb_seeded (8 local members) and eggroll_update_seeded without caps, at one GPU's share of
configs[2] (Sana layout, pop 64, egg rank 1) and configs[3] (Sana layout at egg rank 4, pop 128: 16 local
members).  The factors are regenerated inside both kernels (Philox4x32-10 + Box-Muller), so they are priced
against the VALU issue rate, not HBM: tools/es_valu_summary.py.
usage: python tools/es_valu_driver.py [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from hyperscalees_t2i_amd.sana import sana_lora_shapes  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
for rank, pop, local in ((1, 64, 8), (4, 128, 16)):
    lay = K.ThetaLayout(sana_lora_shapes(), rank)
    theta = torch.randn(lay.D, device=dev) * 0.01
    tp = torch.empty((local, lay.D), device=dev)
    S = torch.randn(pop, 4, device=dev) + 21
    fit = K.fitness(S, True)
    ws = K.UpdateWorkspace(lay, dev)
    out = torch.empty_like(theta)
    for _ in range(it):
        K.perturb_seeded(theta, 7, lay, pop, True, 0, local, 1e-2, dev, out=tp)
        K.update_seeded(theta, 7, fit, lay, pop, True, 1e-3, 0.0, 0.0, out=out, workspace=ws)
    torch.cuda.synchronize()
    print(f"rank {rank} pop {pop} local {local}: D {lay.D} done", flush=True)
