"""Is a member's evaluation independent of how many members share its batch?  (configs[2]: 8 members per
GPU vs one process with all 64.)  Runs generate_population + rewards for `pop` members in one batch and
again in chunks of `chunk`, and compares every member's outputs bitwise: per module (first differing
module in execution order, --small only), transformer output, image, rewards.

    python tools/batch_invariance_probe.py [--small] [--pop 16] [--chunk 8]
"""
import argparse
import json
import sys
from pathlib import Path
from types import SimpleNamespace

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--pop", type=int, default=16)
    ap.add_argument("--chunk", type=int, default=8)
    ap.add_argument("--benchmark", type=int, default=1, help="torch.backends.cudnn.benchmark (bench.py: 1)")
    a = ap.parse_args()
    import bench
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    dev = torch.device("cuda:0")
    be, eng, nz, theta, _ = bench.build(SimpleNamespace(workload="sana", small=a.small, pop_per_gpu=a.pop, latent=32),
                                        1, 0, dev)
    rewards = eng.rewards
    seed, gs = 3, be.cfg.guidance_scale
    fac = nz.sample_factors(a.pop, dev, seed=seed)
    tp = nz.perturb(theta, fac, a.pop, 0, a.pop)
    info = be.step_sampling_info(seed)
    flat = info["flat_ids"]
    B = len(flat)
    mods = [(n, m) for n, m in list(be.es_model.transformer.named_modules()) + [("vae", be.es_model.vae)]
            if n] if a.small else [("transformer", be.es_model.transformer)]

    def run(t):
        outs = {}
        hooks = [m.register_forward_hook(lambda _m, _i, o, n=n: outs.setdefault(n, []).append(
            o.detach().clone() if torch.is_tensor(o) else None)) for n, m in mods]
        try:
            imgs = be.generate_population(flat, seed, gs, t)
        finally:
            for h in hooks:
                h.remove()
        j_of = torch.tensor([info["pid_to_j"][p] for p in flat], device=dev).repeat(t.shape[0])
        rew = rewards.score(imgs, j_of, rewards.prompt_features(info["unique_texts"]))
        return outs, imgs, rew["combined"]

    for _ in range(2 if a.benchmark else 1):   # warm MIOpen Find for both batch sizes
        full = run(tp)
        parts = [run(tp[i:i + a.chunk]) for i in range(0, a.pop, a.chunk)]
    torch.cuda.synchronize()
    img_c = torch.cat([p[1] for p in parts])
    rew_c = torch.cat([p[2] for p in parts])
    res = {"pop": a.pop, "chunk": a.chunk, "small": a.small, "benchmark": a.benchmark,
           "images_equal": bool(torch.equal(full[1], img_c)), "rewards_equal": bool(torch.equal(full[2], rew_c)),
           "image_max_abs": float((full[1].float() - img_c.float()).abs().max()),
           "reward_max_abs": float((full[2] - rew_c).abs().max())}
    first = []
    for n, _ in mods:
        fo = full[0].get(n)
        if not fo or fo[0] is None:
            continue
        if any(len(p[0].get(n, [])) != len(fo) for p in parts):
            first.append({"module": n, "calls_differ": [len(fo)] + [len(p[0].get(n, [])) for p in parts]})
            continue
        for ci, t in enumerate(fo):
            if t is None:
                continue
            pc = [p[0][n][ci] for p in parts]
            if t.shape[0] % a.pop == 0 and all(x.shape[0] * (a.pop // a.chunk) == t.shape[0] for x in pc):
                cat = torch.cat(pc)
            else:
                cat = None
            if cat is not None and not torch.equal(t, cat):
                first.append({"module": n, "call": ci, "shape": list(t.shape),
                              "max_abs": float((t.float() - cat.float()).abs().max())})
    res["differing_modules"] = first[:40]
    res["n_differing"] = len(first)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
