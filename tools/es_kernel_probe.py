"""Launch the ES arithmetic kernels back to back at the Sana-Sprint 1.6B theta layout (D = 1,515,456)
for rocprofv3 --kernel-trace --stats: noise, perturb (8 local members), fitness, update with caps
off (one launch) and on (k_update + k_update_caps), for pop 8 / 64 / 128 (egg rank 1) and pop 128
at egg rank 4 (Z-Image's configs[3] rank).
usage: python tools/es_kernel_probe.py [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from hyperscalees_t2i_amd.sana import sana_lora_shapes  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
for rank, pop in ((1, 8), (1, 64), (1, 128), (4, 128)):
    lay = K.ThetaLayout(sana_lora_shapes(), rank)
    nb = K.n_base_samples(pop, True)
    theta = torch.randn(lay.D, device=dev) * 0.01
    fac = K.noise_factors(0, nb, lay, dev)
    tp = torch.empty((8, lay.D), device=dev)
    S = torch.randn(pop, 4, device=dev) + 21
    fit = K.fitness(S, True)
    ws = K.UpdateWorkspace(lay, dev)
    out = torch.empty_like(theta)
    for _ in range(it):
        K.noise_factors(0, nb, lay, dev, out=fac)
        K.perturb(theta, fac, lay, pop, True, 0, 8, 1e-2, out=tp)
        K.fitness(S, True)
        K.update(theta, fac, fit, lay, pop, True, 1e-3, 0.0, 0.0, out=out, workspace=ws)
        K.update(theta, fac, fit, lay, pop, True, 1e-3, 0.0, 40.0, out=out, workspace=ws)
    torch.cuda.synchronize()
    print(f"rank {rank} pop {pop}: D {lay.D} tiles {lay.n_tiles} done", flush=True)
