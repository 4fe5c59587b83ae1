"""torch.profiler kernel table of the fused CLIP tower vs transformers' tower (one call each)."""
import sys
from pathlib import Path

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd.clip_tower import CLIPVisionTower  # noqa: E402
from hyperscalees_t2i_amd.rewards import CLIP_B32, CLIP_H14, _image_features, build_clip  # noqa: E402

dev = torch.device("cuda:0")
which = sys.argv[1] if len(sys.argv) > 1 else "b32"
model = build_clip(CLIP_B32 if which == "b32" else CLIP_H14, dev, seed=5)
px = torch.randn((128, 3, 224, 224), device=dev)
tw = CLIPVisionTower(model)
for fn, name in ((lambda: tw(px), "tower"), (lambda: _image_features(model, px), "hf")):
    fn(); fn()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    print("=====", name)
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=12, max_name_column_width=70))
