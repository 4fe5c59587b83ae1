"""ESEngine.evaluate_local twice on the same theta / seed in one process: the first module (execution
order) of pass `--pass-index` whose output differs between the two evaluations.

    python tools/eval_repeat_probe.py [--small] [--pop 64] [--pass-index 0]
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
    ap.add_argument("--pop", type=int, default=64)
    ap.add_argument("--pass-index", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--light", action="store_true", help="hook only the transformer and decoder outputs")
    a = ap.parse_args()
    import bench
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda:0")
    be, eng, nz, theta, _ = bench.build(SimpleNamespace(workload="sana", small=a.small, pop_per_gpu=a.pop, latent=32),
                                        1, 0, dev)
    gs = be.cfg.guidance_scale
    mods = [("tr." + n, m) for n, m in be.es_model.transformer.named_modules() if n]
    mods += [("tr", be.es_model.transformer), ("vae", be.es_model.vae)]
    if a.light:
        mods = [(n, m) for n, m in mods if n in ("tr", "vae")]
    elif a.pass_index < 0:   # every pass, transformer-level modules + the decoder output only
        from hyperscalees_t2i_amd.lora import LoRALinear
        mods = [(n, m) for n, m in mods if n.count(".") <= 2 or isinstance(m, LoRALinear)]
    state = {"eval": 0, "pass": -1, "rec": {}, "diffs": [], "cnt": {}}
    g0 = be.generate_population

    def gen(*x, **k):
        state["pass"] += 1
        return g0(*x, **k)
    be.generate_population = gen

    def hook(_m, _i, o, n):
        if (a.pass_index >= 0 and state["pass"] != a.pass_index) or not torch.is_tensor(o):
            return
        ck = (state["pass"], n)
        c = state["cnt"].get(ck, 0)
        state["cnt"][ck] = c + 1
        key = (state["pass"], n, c)
        if state["eval"] == 0:
            state["rec"][key] = o.detach().clone()
        else:
            ref = state["rec"].get(key)
            if ref is not None and not torch.equal(ref, o) and len(state["diffs"]) < 40:
                d = (ref.float() - o.float()).abs().nan_to_num(1e30)
                rows = d.reshape(d.shape[0], -1).amax(1).nonzero().flatten().tolist() if d.dim() > 1 else []
                state["diffs"].append({"pass": state["pass"], "module": n, "call": c, "max_abs": float(d.max()),
                                       "shape": list(o.shape), "rows": rows[:8], "n_rows": len(rows)})
    hooks = [m.register_forward_hook(lambda _m, _i, o, n=n: hook(_m, _i, o, n)) for n, m in mods]
    S1 = eng.evaluate_local(theta, a.seed, gs)[0].clone()
    state.update(eval=1, **{"pass": -1}, cnt={})
    S2 = eng.evaluate_local(theta, a.seed, gs)[0].clone()
    for h in hooks:
        h.remove()
    print(json.dumps({"S_equal": bool(torch.equal(S1, S2)),
                      "rows_differ": [int(i) for i in (S1 != S2).any(1).nonzero().flatten()],
                      "pass": a.pass_index, "first_diffs": state["diffs"]}))


if __name__ == "__main__":
    main()
