"""Same-process interleaved A/B of one build knob on the bench epoch (N=1, pop 8).

    python tools/fuse_ab.py [--rounds 4] [--knob fuse|xattn]
fuse: lora.FUSE_EPILOGUES (GEMM-epilogue fusions); xattn: Sana attn2 on eggroll_cross_attention vs
SDPA; chunk: DC-AE decode chunk size ("fused" arm = the first of --chunks); sharedproj:
lora.SHARED_PROJECTION (one X pass for attn1 q/k/v and attn2 k/v LoRA projections); towers32: reward
towers with the fp32 residual stream vs plain bf16.  2 timed epochs per arm per round (box-to-box spread is +-3 %, so only same-process interleaved
arms are compared)."""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--knob", choices=("fuse", "xattn", "chunk", "sharedproj", "towers32"), default="fuse")
    ap.add_argument("--chunks", type=str, default="8,16", help="knob chunk: the two DC-AE decode chunk sizes")
    a = ap.parse_args()
    import bench
    from hyperscalees_t2i_amd import lora
    args = argparse.Namespace(latent=32, small=False, pop_per_gpu=8, workload="sana")
    backend, engine, noiser, theta, pop = bench.build(args, 1, 0, torch.device("cuda:0"))
    g = backend.cfg.guidance_scale
    for w in range(2):
        theta, _ = engine.step(theta, seed=w, guidance_scale=g)
    res = {"fused": [], "unfused": []}
    seed = 10
    blocks = backend.es_model.transformer.transformer_blocks

    ca, cb = (int(c) for c in a.chunks.split(","))

    def set_arm(on):
        if a.knob == "chunk":
            backend.es_model.vae_chunk = ca if on else cb
        elif a.knob == "fuse":
            lora.FUSE_EPILOGUES = on
        elif a.knob == "sharedproj":
            lora.SHARED_PROJECTION = on
        elif a.knob == "towers32":
            engine.rewards.fp32_residual = on
        else:
            for blk in blocks:
                blk.attn2.use_kernel = on

    for r in range(a.rounds):
        for arm in ("fused", "unfused"):
            set_arm(arm == "fused")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2):
                theta, _ = engine.step(theta, seed=seed, guidance_scale=g)
                seed += 1
            torch.cuda.synchronize()
            res[arm].append(1e3 * (time.perf_counter() - t0) / 2)
            print(arm, round(res[arm][-1], 1), flush=True)
    set_arm(True)
    out = {k: sorted(v) for k, v in res.items()}
    out["knob"] = a.knob
    out["median_ms"] = {k: v[len(v) // 2] for k, v in out.items() if k != "knob"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
