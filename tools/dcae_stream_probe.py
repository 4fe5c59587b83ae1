"""How many DC-AE stages (lowest resolution first) should carry the fp32 residual stream: rank fidelity
vs cost.  (1) Fidelity: the product path (bf16 kernels, fused epilogues) with vae.fp32_stages = k vs
the fp32 restatement, pooled over the 12 seeds of tests/test_gpu_parity_fp32.py::
test_rank_fidelity_over_seeds (same tiny stack, reference noise g10): discordant pairs, best / worst
agreement, max |dS|.  (2) Cost: the full-size decoder (Sana DC-AE f32c32, 8 images of 1024 px per
call = the pipeline's vae_chunk) timed per k.
usage: python tools/dcae_stream_probe.py [out.json]"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig  # noqa: E402
from hyperscalees_t2i_amd.dcae import DCAEDecoder  # noqa: E402
from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params  # noqa: E402
from hyperscalees_t2i_amd.es_step import aggregate_member_rewards  # noqa: E402
from hyperscalees_t2i_amd.rewards import RewardModels  # noqa: E402
from hyperscalees_t2i_amd.sana import SanaArch  # noqa: E402
from oracle import eggroll_oracle as O  # noqa: E402
from oracle import member_eval_fp32 as R  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402

dev = torch.device("cuda:0")
KS = (0, 2, 3, 4, 5, 6)
out = {"fidelity": {}, "decode_ms_8x1024px": {}}

# ---- (2) cost at full size first (the tiny stack's allocations come after)
with torch.no_grad():
    vae = DCAEDecoder().to(dev)
    vae.init_weights(1)
    z = torch.randn(8, 32, 32, 32, device=dev)
    for k in KS:
        vae.fp32_stages = k
        out["decode_ms_8x1024px"][k] = round(min(bench(lambda: vae(z), it=3) for _ in range(3)), 2)
    print(json.dumps(out["decode_ms_8x1024px"]), flush=True)
    del vae, z
    torch.cuda.empty_cache()

# ---- (1) fidelity on the tiny stack
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
tp = noiser.perturb(theta, torch.from_numpy(noiser.layout.pack_factors(g["s0/factors"])).to(dev), pop, 0, pop)
vae = be.es_model.vae
res = {k: {"disc": 0, "best": 0, "worst": 0, "S_abs": 0.0} for k in KS}


def disc(a, b):
    return int(sum(np.sign(a[i] - a[j]) * np.sign(b[i] - b[j]) < 0 for i in range(len(a)) for j in range(i + 1, len(a))))


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
        S32 = torch.stack([agg(rw32.score(R.generate_fp32(be.es_model, theta + sigma * eps_ref[k], pe, am, lat, 4.5)[1],
                                          j_of, feats32)) for k in range(pop)])
        sc32 = O.ref_promptnorm(S32.cpu().numpy())[0]
        o32 = np.argsort(sc32, kind="stable")
        feats = rewards.prompt_features(info["unique_texts"])
        for k in KS:
            vae.fp32_stages = k
            imgs = be.generate_population(flat, seed, 4.5, tp)
            S = aggregate_member_rewards(rewards.score(imgs, j_of.repeat(pop), feats), flat, info["pid_to_j"], pop, m)[0]
            sc = K.fitness(S, True)["scores"].cpu().numpy()
            o = np.argsort(sc, kind="stable")
            d = res[k]
            d["disc"] += disc(sc, sc32)
            d["best"] += int(o[-1] == o32[-1])
            d["worst"] += int(o[0] == o32[0])
            d["S_abs"] = max(d["S_abs"], float((S - S32).abs().max()))
        print(seed, json.dumps({k: v["disc"] for k, v in res.items()}), flush=True)
vae.fp32_stages = len(vae.stages)
for d in res.values():
    d["pooled_tau"] = round(1 - 2 * d["disc"] / (12 * pop * (pop - 1) // 2), 4)
    d["S_abs"] = round(d["S_abs"], 6)
out["fidelity"] = res
print(json.dumps(out), flush=True)
if len(sys.argv) > 1:
    Path(sys.argv[1]).write_text(json.dumps(out, indent=1))
