"""In ONE process: a rank's S rows (ESEngine.evaluate_local with DistInfo(rank, 8)) vs the same members
inside a single-process pop-64 evaluation (8 passes of 8), and the pop-64 evaluation repeated.
Separates in-process effects (workspace reuse, run-to-run nondeterminism) from cross-process ones.

    python tools/pass_invariance_probe.py [--small]
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
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import bench
    from hyperscalees_t2i_amd.es_step import DistInfo, ESEngine
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda:0")
    be, eng, nz, theta, pop = bench.build(SimpleNamespace(workload="sana", small=a.small, pop_per_gpu=64, latent=32),
                                          1, 0, dev)
    gs = be.cfg.guidance_scale
    rec = {"gen": [], "score": [], "feats": []}
    g0, s0, f0 = be.generate_population, eng.rewards.score, eng.rewards.prompt_features

    def gen(*x, **k):
        out = g0(*x, **k)
        rec["gen"].append(out.clone())
        return out

    def sc(imgs, *x, **k):
        out = s0(imgs, *x, **k)
        rec["score"].append(out["combined"].clone())
        return out

    def pf(*x, **k):
        out = f0(*x, **k)
        rec["feats"].append({kk: v.clone() for kk, v in out.items()})
        return out
    be.generate_population, eng.rewards.score, eng.rewards.prompt_features = gen, sc, pf
    S64 = eng.evaluate_local(theta, a.seed, gs)[0].clone()
    S64b = eng.evaluate_local(theta, a.seed, gs)[0].clone()
    n = len(rec["gen"]) // 2
    res0 = {"passes": n,
            "gen_equal": [bool(torch.equal(rec["gen"][i], rec["gen"][n + i])) for i in range(n)],
            "score_equal": [bool(torch.equal(rec["score"][i], rec["score"][n + i])) for i in range(n)],
            "feats_equal": all(torch.equal(rec["feats"][0][k], rec["feats"][1][k]) for k in rec["feats"][0])}
    be.generate_population, eng.rewards.score, eng.rewards.prompt_features = g0, s0, f0
    # score the recorded images of eval 1 again, pass by pass
    j = torch.tensor([be.step_sampling_info(a.seed)["pid_to_j"][p] for p in be.step_sampling_info(a.seed)["flat_ids"]],
                     device=dev)
    res0["rescore_equal"] = [bool(torch.equal(s0(rec["gen"][i], j.repeat(8), rec["feats"][0])["combined"], rec["score"][i]))
                             for i in range(n)]
    print(json.dumps(res0), flush=True)
    res = {"repeat_equal": bool(torch.equal(S64, S64b)), "ranks": []}
    for r in range(8):
        e = ESEngine(be, eng.rewards, nz, eng.cfg, dev, DistInfo(r, 8, None))
        Sr = e.evaluate_local(theta, a.seed, gs)[0]
        res["ranks"].append({"rank": r, "equal": bool(torch.equal(Sr, S64[8 * r:8 * r + 8])),
                             "max_abs": float((Sr - S64[8 * r:8 * r + 8]).abs().max())})
    S64c = eng.evaluate_local(theta, a.seed, gs)[0]
    res["repeat_after_ranks_equal"] = bool(torch.equal(S64, S64c))
    res["repeat_rows_differ"] = [int(i) for i in (S64 != S64b).any(1).nonzero().flatten()]
    # one pass evaluated repeatedly: first module (registration order) whose output changes
    tp = nz.perturb(theta, nz.sample_factors(64, dev, seed=a.seed), 64, 0, 64)
    info = be.step_sampling_info(a.seed)
    mods = [(n, m) for n, m in be.es_model.transformer.named_modules() if n] + [("vae", be.es_model.vae)]

    def run(t):
        outs = {}
        hooks = [m.register_forward_hook(lambda _m, _i, o, n=n: outs.setdefault(n, []).append(
            o.detach().clone() if torch.is_tensor(o) else None)) for n, m in mods]
        try:
            imgs = be.generate_population(info["flat_ids"], a.seed, gs, t)
        finally:
            for h in hooks:
                h.remove()
        return outs, imgs
    runs = [run(tp[32:40]), run(tp[32:40].clone()), run(tp[32:40])]
    for i in (1, 2):
        diff = []
        for n, _ in mods:
            for ci, (x, y) in enumerate(zip(runs[0][0].get(n, []), runs[i][0].get(n, []))):
                if x is not None and not torch.equal(x, y):
                    diff.append({"module": n, "call": ci, "max_abs": float((x.float() - y.float()).abs().max())})
        res[f"pass_repeat{i}"] = {"images_equal": bool(torch.equal(runs[0][1], runs[i][1])), "first_diffs": diff[:12]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
