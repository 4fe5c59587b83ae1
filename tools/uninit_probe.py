"""Does any op of the full-size member-eval read memory it did not write?  The caching allocator is emptied and
one huge block is allocated, filled with a byte pattern and freed again, so every allocation of the next
member-eval is carved from pattern-filled memory; the eval's outputs (transformer output, images, S) are
compared with a reference eval across patterns 0x00 / 0xFF (NaN in fp32 and bf16) / 0x7F (huge).  An op that
reads unwritten bytes shows up as a pattern-dependent result.
usage: python tools/uninit_probe.py [GiB]"""
import hashlib
import json
import sys
from pathlib import Path
from types import SimpleNamespace

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def digest(t):
    return hashlib.sha256(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12]


def main(gib=150):
    import bench
    from hyperscalees_t2i_amd.es_step import aggregate_member_rewards
    from hyperscalees_t2i_amd.lora import LoRALinear
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = False
    args = SimpleNamespace(workload="sana", small=False, pop_per_gpu=8, latent=32)
    be, engine, noiser, theta, pop = bench.build(args, 1, 0, dev)
    rewards = engine.rewards
    seed, gs = 0, be.cfg.guidance_scale
    info = be.step_sampling_info(seed)
    flat, m = info["flat_ids"], info["m"]
    j_of = torch.tensor([info["pid_to_j"][p] for p in flat], device=dev).repeat(pop)
    caps = {}
    hooks = []
    for name, mod in be.es_model.transformer.named_modules():
        if isinstance(mod, LoRALinear) and name.startswith(("transformer_blocks.0.", "transformer_blocks.19.")):
            hooks.append(mod.register_forward_hook(lambda _m, _i, o, n=name: caps.setdefault(n, []).append(digest(o))))
    be.es_model.transformer.register_forward_hook(lambda _m, _i, o: caps.setdefault("transformer", []).append(digest(o)))

    def one():
        caps.clear()
        with torch.no_grad():
            fac = noiser.epoch_noise(pop, seed=seed)
            tp = noiser.perturb(theta, fac, pop, 0, pop, out=engine.theta_pop[:pop])
            feats = rewards.prompt_features(info["unique_texts"])
            imgs = be.generate_population(flat, seed, gs, tp)
            rw = rewards.score(imgs, j_of, feats)
            S = aggregate_member_rewards(rw, flat, info["pid_to_j"], pop, m)[0]
        torch.cuda.synchronize()
        return {"caps": {k: list(v) for k, v in caps.items()}, "img": digest(imgs), "S": digest(S),
                "S_rows": [digest(S[k]) for k in range(pop)], "img_per_member": [digest(imgs[k * len(flat):(k + 1) * len(flat)]) for k in range(pop)],
                "feats": {k: digest(v) for k, v in feats.items()}}

    ref = one()
    res = []
    for pat in (0x00, 0xFF, 0x7F, 0x00, 0xFF):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        free = torch.cuda.mem_get_info(dev)[0]
        n = min(int(gib) << 30, free - (8 << 30))
        big = torch.empty(n, dtype=torch.uint8, device=dev)
        big.fill_(pat)
        del big       # stays in the caching allocator: the next allocations are split from it
        r = one()
        d = {"pattern": hex(pat), "filled_GiB": round(n / 2 ** 30, 1), "S_equal": r["S"] == ref["S"],
             "img_equal": r["img"] == ref["img"], "feats_equal": r["feats"] == ref["feats"],
             "rows_differ": [k for k in range(pop) if r["S_rows"][k] != ref["S_rows"][k]],
             "img_members_differ": [k for k in range(pop) if r["img_per_member"][k] != ref["img_per_member"][k]],
             "caps_differ": sorted(k for k in ref["caps"] if r["caps"].get(k) != ref["caps"][k])[:20]}
        res.append(d)
        print(json.dumps(d), flush=True)
    out = ROOT / "gpurun_out" / "uninit_probe.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 150)
