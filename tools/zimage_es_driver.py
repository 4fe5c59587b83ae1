"""Launch the ES kernels at configs[3]'s Z-Image-Turbo layout (egg rank 4, pop 128, 16 local members)
a few times for rocprofv3 counter passes (noise, perturb, update with the theta cap set).
usage: python tools/zimage_es_driver.py [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from hyperscalees_t2i_amd.model_shapes import zimage_turbo_lora_shapes  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
lay = K.ThetaLayout(zimage_turbo_lora_shapes(), 4)
pop, nloc = 128, 16
nb = K.n_base_samples(pop, True)
theta = torch.randn(lay.D, device=dev) * 0.01
S = torch.randn(pop, 4, device=dev) + 21
fit = K.fitness(S, True)
ws = K.UpdateWorkspace(lay, dev)
fac = K.noise_factors(0, nb, lay, dev)
tp = torch.empty((nloc, lay.D), device=dev)
out = torch.empty_like(theta)
for _ in range(it):
    K.noise_factors(0, nb, lay, dev, out=fac)
    K.perturb(theta, fac, lay, pop, True, 0, nloc, 1e-2, out=tp)
    K.update(theta, fac, fit, lay, pop, True, 1e-3, 0.0, 40.0, out=out, workspace=ws)
torch.cuda.synchronize()
print("ok", lay.D, lay.n_tiles)
