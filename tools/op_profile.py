"""torch.profiler attribution of one VAE chunk and one transformer forward (diagnostic)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
torch.backends.cudnn.benchmark = True
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig  # noqa: E402
from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params  # noqa: E402

dev = torch.device("cuda:0")
be = SanaBackend(str(dev), SanaConfig(synthetic_weights=True))
be.init_and_attach_lora()
params, shapes = be.collect_lora_params()
theta = flatten_params(params).to(dev)
nz = EggRollNoiser(shapes, 1e-2, 1e-1, 1, True)
fac = nz.sample_factors(8, dev, seed=0)
tp = nz.perturb(theta, fac, 8, 0, 8)
flat = be.step_sampling_info(0)["flat_ids"]
for _ in range(2):  # warm (MIOpen find)
    be.generate_population(flat, 0, 4.5, tp)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU], record_shapes=True) as prof:
    be.generate_population(flat, 0, 4.5, tp)
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=45,
                                                          max_name_column_width=40, max_shapes_column_width=70))
