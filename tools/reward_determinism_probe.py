"""Run-to-run determinism of the reward path on fixed images: CLIP preprocessing, each vision tower,
the combined reward, repeated N times in one process.

    python tools/reward_determinism_probe.py [--small] [--n 128] [--reps 6]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--px", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    from hyperscalees_t2i_amd.rewards import RewardModels, clip_pixels
    dev = torch.device("cuda:0")
    rw = RewardModels.build(dev, tiny=a.small, synthetic=True)
    g = torch.Generator(device=dev).manual_seed(0)
    imgs = (torch.rand(a.n, 3, a.px, a.px, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    feats = rw.prompt_features(["a", "b", "c", "d"])
    j = torch.arange(a.n, device=dev) % 4
    t_clip, t_pick = rw.towers()
    base = None
    res = {"small": a.small, "n": a.n, "reps": []}
    for r in range(a.reps):
        px = clip_pixels(imgs[:16], 0, rw.clip_px.size, rw.clip_px.mean, rw.clip_px.std)
        ec, ep = t_clip(px).clone(), t_pick(px).clone()
        comb = rw.score(imgs, j, feats)["combined"].clone()
        cur = (px, ec, ep, comb)
        if base is None:
            base = cur
            continue
        res["reps"].append({"px": bool(torch.equal(base[0], px)), "clip": bool(torch.equal(base[1], ec)),
                            "pick": bool(torch.equal(base[2], ep)), "combined": bool(torch.equal(base[3], comb)),
                            "rows": [int(i) for i in (base[3] != comb).nonzero().flatten()][:16]})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
