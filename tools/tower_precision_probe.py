"""Reward-tower precision vs cost at the bench's full size (CLIP-B/32 + CLIP-H/14, 128 images of
1024 px): per-image combined reward of the plain-bf16 towers and of the fp32-residual towers
against fp32 towers with the same weights (oracle.member_eval_fp32.Rewards32), plus the time of
RewardModels.score for both modes.   python tools/tower_precision_probe.py [n_images]"""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd.rewards import RewardModels  # noqa: E402
from oracle.member_eval_fp32 import Rewards32  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    dev = torch.device("cuda:0")
    torch.backends.cuda.matmul.allow_tf32 = False
    rw = RewardModels.build(dev, synthetic=True)
    r32 = Rewards32(rw)
    g = torch.Generator(device=dev).manual_seed(0)
    # smooth synthetic "decoder outputs" in [-1, 1]
    base = torch.rand((n, 3, 32, 32), generator=g, device=dev) * 2 - 1
    imgs = torch.nn.functional.interpolate(base, size=(1024, 1024), mode="bicubic", align_corners=False).clamp(-1, 1)
    prompts = ["a photo of a cat", "a red car", "mountains at dawn", "a bowl of fruit"]
    j = torch.arange(n, device=dev) % 4
    ref = r32.score(imgs, j, r32.prompt_features(prompts))
    out = {"n_images": n}
    for mode in (False, True):
        rw.fp32_residual = mode
        feats = rw.prompt_features(prompts)
        got = rw.score(imgs.to(torch.bfloat16), j, feats)
        torch.cuda.synchronize()
        t = []
        for _ in range(5):
            t0 = time.perf_counter()
            rw.score(imgs.to(torch.bfloat16), j, feats)
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        d = (got["combined"] - ref["combined"]).abs()
        out["fp32_residual" if mode else "bf16"] = {
            "combined_abs_max": float(d.max()), "combined_abs_mean": float(d.mean()),
            "combined_spread": float(ref["combined"].std()), "score_ms": 1e3 * min(t)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
