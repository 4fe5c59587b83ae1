"""Which bf16 rounding points in the Sana transformer cost fitness-rank fidelity at sigma = 1e-2:
the fp32 restatement (oracle/member_eval_fp32.py) with bf16 rounding injected at one class of points
at a time (then combinations), fp32 DC-AE and towers, vs the pure-fp32 member-eval — pooled
discordant member pairs over the 12 seeds of tests/test_gpu_parity_fp32.py::test_rank_fidelity_over_seeds
(same tiny stack, reference noise g10).  Also the build's own transformer (bf16 kernels) for scale.
usage: python tools/drift_probe.py [out.json]"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig  # noqa: E402
from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params  # noqa: E402
from hyperscalees_t2i_amd.es_step import aggregate_member_rewards  # noqa: E402
from hyperscalees_t2i_amd.rewards import RewardModels  # noqa: E402
from hyperscalees_t2i_amd.sana import SanaArch  # noqa: E402
from oracle import eggroll_oracle as O  # noqa: E402
from oracle import member_eval_fp32 as R  # noqa: E402

dev = torch.device("cuda:0")
TINY = SanaArch(num_attention_heads=4, attention_head_dim=32, num_layers=2, num_cross_attention_heads=2,
                cross_attention_head_dim=64, caption_channels=2304)
be = SanaBackend(str(dev), SanaConfig(synthetic_weights=True, width_latent=4, height_latent=4, batches_per_gen=2,
                                      arch=TINY, vae_widths=(16, 32, 32, 64, 64, 64), vae_layers=(1, 1, 1, 1, 1, 1)))
be.init_and_attach_lora()
rewards = RewardModels.build(dev, tiny=True)
rw32 = R.Rewards32(rewards)
g = np.load(ROOT / "tests" / "golden" / "g10_member_eval_injection.npz")
params, shapes = be.collect_lora_params()
sigma, pop = float(g["s0/sigma"]), 8
theta = flatten_params(params).to(dev)
noiser = EggRollNoiser(shapes, sigma=sigma, lr_scale=0.1, rank=1, use_antithetic=True)
eps_ref = torch.from_numpy(g["s0/eps"]).to(dev)
fac = torch.from_numpy(noiser.layout.pack_factors(g["s0/factors"])).to(dev)
tp = noiser.perturb(theta, fac, pop, 0, pop)
ALL = ("x", "lin_in", "lin_out", "norm", "attn", "out", "mods", "temb")
# (transformer classes rounded, DC-AE classes rounded); towers fp32 throughout
DALL = ("dx", "dact")
T_FIX = tuple(c for c in ALL if c not in ("temb", "x", "mods"))   # transformer after the planned fp32 fixes
VARIANTS = [((), ()), (T_FIX, ()), (T_FIX, DALL), (T_FIX, ("dact",)), (T_FIX, ("dact", "dx_vit", "dx_up")),
            (T_FIX, ("dact", "dx_res", "dx_up")), (T_FIX, ("dact", "dx_res", "dx_vit")), (T_FIX, ("dact", "dx_up"))]


def tau_disc(a, b):
    n, d = len(a), 0
    for i in range(n):
        for j in range(i + 1, n):
            d += np.sign(a[i] - a[j]) * np.sign(b[i] - b[j]) < 0
    return int(d)


def name_of(v):
    t, d = v
    tn = "T:fp32" if not t else ("T:all" if t == ALL else "T:all-" + "-".join(c for c in ALL if c not in t))
    return tn + " D:" + ("+".join(d) or "fp32")
res = {name_of(v): {"disc": 0, "S_abs": 0.0, "S_sq": 0.0, "n": 0} for v in VARIANTS}
res["build_transformer"] = {"disc": 0, "S_abs": 0.0, "S_sq": 0.0, "n": 0}
res["fp32"] = {"disc": 0, "S_abs": 0.0, "S_sq": 0.0, "n": 0}
res["build_transformer+dcae"] = {"disc": 0, "S_abs": 0.0, "S_sq": 0.0, "n": 0}
with torch.no_grad():
    for seed in range(5, 17):
        info = be.step_sampling_info(seed)
        flat, m = info["flat_ids"], info["m"]
        B = len(flat)
        pe, am = be._gather(flat)
        lat = be.es_model._latents(B, seed, 4, 4)
        j_of = torch.tensor([info["pid_to_j"][p] for p in flat], device=dev)
        feats32 = rw32.prompt_features(info["unique_texts"])
        agg = lambda rw: aggregate_member_rewards(rw, flat, info["pid_to_j"], 1, m)[0][0]  # noqa: E731
        tr_out = []
        hook = be.es_model.transformer.register_forward_hook(lambda _m, _i, o: tr_out.append(o))
        imgs = be.generate_population(flat, seed, 4.5, tp)
        hook.remove()
        S = {}
        for v in VARIANTS:
            S[name_of(v)] = torch.stack([agg(rw32.score(R.generate_fp32(
                be.es_model, theta + sigma * eps_ref[k], pe, am, lat, 4.5, rnd=v[0], drnd=v[1])[1], j_of, feats32))
                for k in range(pop)])
        S["build_transformer"] = torch.stack([agg(rw32.score(R.decode_fp32(be.es_model, tr_out[0][k * B:(k + 1) * B], lat),
                                                              j_of, feats32)) for k in range(pop)])
        S["build_transformer+dcae"] = torch.stack([agg(rw32.score(imgs[k * B:(k + 1) * B].float(), j_of, feats32))
                                                   for k in range(pop)])
        S["fp32"] = S["T:fp32 D:fp32"]
        sc32 = O.ref_promptnorm(S["fp32"].cpu().numpy())[0]
        for name, Sx in S.items():
            sc = O.ref_promptnorm(Sx.cpu().numpy())[0]
            res[name]["disc"] += tau_disc(sc, sc32)
            res[name]["S_abs"] = max(res[name]["S_abs"], float((Sx - S["fp32"]).abs().max()))
            res[name]["S_sq"] += float(((Sx - S["fp32"]) ** 2).sum())
            res[name]["n"] += Sx.numel()
for v in res.values():
    v["S_abs"] = round(v["S_abs"], 6)
    v["S_rms"] = round((v.pop("S_sq") / v.pop("n")) ** 0.5, 6)
print(json.dumps(res, indent=1))
if len(sys.argv) > 1:
    Path(sys.argv[1]).write_text(json.dumps(res, indent=1))
