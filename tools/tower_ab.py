"""Same-process A/B of the CLIP reward towers' fp32 residual stream: fused residual + LayerNorm
(eggroll_resid_layernorm) vs the torch ops it replaces, CLIP-B/32 and CLIP-H/14 at 128 images (one
bench epoch's reward batch); interleaved rounds, median ms, and the embeddings' max relative difference.
usage: python tools/tower_ab.py [rounds]"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd.clip_tower import CLIPVisionTower  # noqa: E402
from hyperscalees_t2i_amd.rewards import CLIP_B32, CLIP_H14, build_clip  # noqa: E402

dev = torch.device("cuda:0")
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5


def t(fn, it=3):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


out = {}
px = torch.randn((128, 3, 224, 224), device=dev)
for name, cfg in (("b32", CLIP_B32), ("h14", CLIP_H14)):
    model = build_clip(cfg, dev, seed=5)
    fused, plain = CLIPVisionTower(model, fused_residual_ln=True), CLIPVisionTower(model, fused_residual_ln=False)
    ef, ep = fused(px), plain(px)
    rel = float(((ef - ep).norm(dim=-1) / ep.norm(dim=-1)).max())
    ms = {"fused": [], "torch": []}
    for _ in range(rounds):
        ms["fused"].append(t(lambda: fused(px)))
        ms["torch"].append(t(lambda: plain(px)))
    out[name] = {k: round(statistics.median(v), 3) for k, v in ms.items()}
    out[name]["max_rel_diff"] = rel
    print(f"[tower-ab] {name}: {out[name]}", flush=True)
    del model, fused, plain
print(json.dumps(out))
