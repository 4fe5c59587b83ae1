"""Where the reward phase's time goes (bench N=1: 128 images of 1024^2 per epoch).

    python tools/reward_probe.py [--n 128] [--iters 5]
HIP-event times: the torch restatement of the CLIP preprocessing vs the HIP eggroll_clip_preprocess,
transformers' towers vs the fused CLIPVisionTower (head dim padded / not), whole RewardModels.score.
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from hyperscalees_t2i_amd.clip_tower import CLIPVisionTower
    from hyperscalees_t2i_amd.rewards import (RewardModels, _image_features, clip_pixels, clip_preprocess,
                                              postprocess_uint8)
    dev = torch.device("cuda:0")
    rm = RewardModels.build(dev, synthetic=True)
    g = torch.Generator(device=dev).manual_seed(0)
    imgs = (torch.rand((a.n, 3, 1024, 1024), generator=g, device=dev) * 2.2 - 1.1).to(torch.bfloat16)
    imgs = imgs.contiguous(memory_format=torch.channels_last)
    feats = rm.prompt_features(["a", "b", "c", "d"])
    idx = torch.arange(a.n, device=dev) % 4
    px = clip_pixels(imgs, 0)
    tb, th = CLIPVisionTower(rm.clip), CLIPVisionTower(rm.pick)
    thn = CLIPVisionTower(rm.pick, pad_head_dim=True)
    res = {
        "n_images": a.n,
        "preprocess_torch_ms": timeit(lambda: clip_preprocess(postprocess_uint8(imgs)), a.iters),
        "preprocess_hip_ms": timeit(lambda: clip_pixels(imgs, 0), a.iters),
        "clip_b32_hf_ms": timeit(lambda: _image_features(rm.clip, px), a.iters),
        "clip_b32_tower_ms": timeit(lambda: tb(px), a.iters),
        "clip_h14_hf_ms": timeit(lambda: _image_features(rm.pick, px), a.iters),
        "clip_h14_tower_ms": timeit(lambda: th(px), a.iters),
        "clip_h14_tower_pad128_ms": timeit(lambda: thn(px), a.iters),
        "score_ms_total": timeit(lambda: rm.score(imgs, idx, feats), a.iters),
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
