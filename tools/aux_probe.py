"""Roofline of the HBM-bound ES kernels at the Sana-Sprint 1.6B theta layout (D = 1,515,456,
r_e = 1) for pop 8 (configs[1]), 64 (configs[2]: 8 local members, all 32 base samples) and 128, and
at configs[3] (Z-Image-Turbo, egg rank 4, 16 of pop 128) / configs[4] (Infinity-8B, 4 of pop 32).
usage: python tools/aux_probe.py"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd.kernels import ThetaLayout  # noqa: E402
from hyperscalees_t2i_amd.measure import aux_kernel_rooflines  # noqa: E402
from hyperscalees_t2i_amd.sana import sana_lora_shapes  # noqa: E402

dev = torch.device("cuda:0")
lay = ThetaLayout(sana_lora_shapes(), 1)
from hyperscalees_t2i_amd.model_shapes import infinity_lora_shapes, zimage_turbo_lora_shapes  # noqa: E402

cases = [("sana", lay, pop, 8) for pop in (8, 64, 128)]
cases += [("zimage_r4", ThetaLayout(zimage_turbo_lora_shapes(), 4), 128, 16),
          ("infinity", ThetaLayout(infinity_lora_shapes(), 1), 32, 4)]
for name, lo, pop, nl in cases:
    r = aux_kernel_rooflines(lo, pop, 0, nl, dev)
    print(json.dumps({"layout": name, **{k: ({kk: round(vv, 4) if isinstance(vv, float) else vv for kk, vv in v.items()})
                                         for k, v in r.items()}}), flush=True)
