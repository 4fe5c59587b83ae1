"""Child process of tests/test_gpu_dist_engine.py (not collected by pytest): one rank of a
world-size-N ES epoch on cuda:0 over the gloo backend, running the REAL sharded ESEngine.step
(member shard -> S all-gather -> fitness -> update -> verify_theta_replicas).

    python tests/dist_engine_worker.py RANK WORLD PORT OUT.pt [POP]
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def build_tiny(dev):
    """The tiny Sana / DC-AE / CLIP stack of tests/test_gpu_engine.py (same seeds in every process)."""
    from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig
    from hyperscalees_t2i_amd.rewards import RewardModels
    from hyperscalees_t2i_amd.sana import SanaArch
    arch = SanaArch(num_attention_heads=4, attention_head_dim=32, num_layers=2, num_cross_attention_heads=2,
                    cross_attention_head_dim=64, caption_channels=2304)
    cfg = SanaConfig(synthetic_weights=True, width_latent=4, height_latent=4, batches_per_gen=2, arch=arch,
                     vae_widths=(16, 32, 32, 64, 64, 64), vae_layers=(1, 1, 1, 1, 1, 1))
    be = SanaBackend(str(dev), cfg)
    be.init_and_attach_lora()
    return be, RewardModels.build(dev, tiny=True)


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    pop = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    import torch
    import torch.distributed as dist
    from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params
    from hyperscalees_t2i_amd.es_step import DistInfo, ESConfig, ESEngine

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    be, rewards = build_tiny(dev)
    params, shapes = be.collect_lora_params()
    theta = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=1, use_antithetic=True)
    cfg = ESConfig(pop_size=pop, theta_max_norm=40.0, verify_replicas=True)
    eng = ESEngine(be, rewards, noiser, cfg, dev, DistInfo(rank, world))
    new, st = eng.step(theta, seed=3, guidance_scale=4.5)
    torch.cuda.synchronize()
    torch.save({"theta0": theta.cpu(), "theta": new.cpu(), "S": st["_S"], "shard": (eng.lo, eng.hi),
                "order": st["_fitness"]["order"], "fitness": st["_fitness"]["fitness"]}, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
