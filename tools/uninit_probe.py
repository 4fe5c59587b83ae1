"""Does any kernel read memory it did not write?  Every torch.empty / empty_like / new_empty made from
Python (kernel outputs and workspaces in kernels.py, model buffers) is filled with a poison value; the
member-eval is run under two poisons and each module's output (execution order) is compared.  A
module whose output depends on the poison reads uninitialised memory.

    python tools/uninit_probe.py [--small] [--pop 8]
"""
import argparse
import json
import sys
from pathlib import Path
from types import SimpleNamespace

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

_orig = {"empty": torch.empty, "empty_like": torch.empty_like}
_orig_new_empty = torch.Tensor.new_empty


def _fill(t, val):
    if t.is_floating_point():
        t.fill_(val)
    elif t.dtype in (torch.int32, torch.int64, torch.int16):
        t.fill_(-7 if val != val else 12345)   # noqa: PLR0124 (nan test)
    elif t.dtype == torch.uint8:
        t.fill_(0xA5 if val != val else 0x3C)  # noqa: PLR0124
    return t


def poison(val):
    torch.empty = lambda *a, **k: _fill(_orig["empty"](*a, **k), val)
    torch.empty_like = lambda *a, **k: _fill(_orig["empty_like"](*a, **k), val)
    torch.Tensor.new_empty = lambda self, *a, **k: _fill(_orig_new_empty(self, *a, **k), val)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--pop", type=int, default=8)
    a = ap.parse_args()
    import bench
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda:0")
    be, eng, nz, theta, _ = bench.build(SimpleNamespace(workload="sana", small=a.small, pop_per_gpu=a.pop, latent=32),
                                        1, 0, dev)
    gs, seed = be.cfg.guidance_scale, 1
    info = be.step_sampling_info(seed)
    mods = [(n, m) for n, m in be.es_model.transformer.named_modules() if n]
    mods += [("vae." + n if n else "vae", m) for n, m in be.es_model.vae.named_modules()]
    order = []

    def run(val):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        poison(val)
        outs = {}
        def hook(_m, _i, o, n):
            if n not in outs:
                order.append(n)
            outs.setdefault(n, []).append(o.detach().clone() if torch.is_tensor(o) else None)
        hooks = [m.register_forward_hook(lambda _m, _i, o, n=n: hook(_m, _i, o, n)) for n, m in mods]
        try:
            fac = nz.sample_factors(a.pop, dev, seed=seed)
            tp = nz.perturb(theta, fac, a.pop, 0, a.pop)
            imgs = be.generate_population(info["flat_ids"], seed, gs, tp)
            j = torch.tensor([info["pid_to_j"][p] for p in info["flat_ids"]], device=dev).repeat(a.pop)
            comb = eng.rewards.score(imgs, j, eng.rewards.prompt_features(info["unique_texts"]))["combined"]
            torch.cuda.synchronize()
        finally:
            for h in hooks:
                h.remove()
            torch.empty, torch.empty_like = _orig["empty"], _orig["empty_like"]
            torch.Tensor.new_empty = _orig_new_empty
        return outs, tp.clone(), imgs.clone(), comb.clone()

    A = run(0.0)
    order_a = list(dict.fromkeys(order))
    B = run(float("nan"))
    C = run(1e4)
    res = {"tp_equal": [bool(torch.equal(A[1], X[1])) for X in (B, C)],
           "images_equal": [bool(torch.equal(A[2], X[2])) for X in (B, C)],
           "rewards_equal": [bool(torch.equal(A[3], X[3])) for X in (B, C)],
           "images_nan": bool(torch.isnan(B[2]).any()), "first": []}
    for n in order_a:
        for X, tag in ((B, "nan"), (C, "1e4")):
            for ci, (x, y) in enumerate(zip(A[0].get(n, []), X[0].get(n, []))):
                if x is not None and y is not None and not torch.equal(x, y):
                    res["first"].append({"module": n, "call": ci, "poison": tag, "nan": bool(torch.isnan(y).any()),
                                         "max_abs": float((x.float() - y.float()).abs().nan_to_num(1e30).max())})
                    break
        if len(res["first"]) >= 8:
            break
    print(json.dumps(res))


if __name__ == "__main__":
    main()
