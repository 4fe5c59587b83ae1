"""hipBLASLt (F.linear) vs the 8-phase LoRA GEMM (r = 0, automatic / 256x256 / 256x320 tile) at the
DC-AE decoder's 1x1-conv shapes and the Sana FFN point conv, per vae_chunk (images per decoder call):
EfficientViT stages at 32^2 / 64^2 (1024 ch) and 128^2 (512 ch): qkv, attention out, GLU inverted and
point convs.  Interleaved rounds in one process; bf16 outputs compared (max |diff| / max |y|).
usage: python tools/dcae_gemm_probe.py [rounds] [out.json] [sana|clip]"""
import json
import statistics
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import kernels as K  # noqa: E402
from tools.gemm_probe_util import bench  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")


def shapes():
    if len(sys.argv) > 3 and sys.argv[3] == "clip":   # the reward towers' linears, 128 images per epoch
        M = 128 * 257                                 # CLIP-H/14 vision: 257 tokens, width 1280, MLP 5120
        yield from (("cliph_qkv", M, 3840, 1280), ("cliph_out", M, 1280, 1280), ("cliph_fc1", M, 5120, 1280),
                    ("cliph_fc2", M, 1280, 5120))
        M = 128 * 50                                  # CLIP-B/32 vision: 50 tokens, width 768, MLP 3072
        yield from (("clipb_qkv", M, 2304, 768), ("clipb_out", M, 768, 768), ("clipb_fc1", M, 3072, 768),
                    ("clipb_fc2", M, 768, 3072))
        return
    if len(sys.argv) > 3 and sys.argv[3] == "sana":   # the Sana linears (no LoRA term: the plain GEMM)
        yield from (("sana_attn", 131072, 2240, 2240), ("sana_ff_inv", 131072, 11200, 2240),
                    ("sana_ff_point_5632", 131072, 2240, 5632), ("sana_attn2_kv", 9600, 2240, 2240))
        return
    for chunk in (8, 16, 32):
        for hw, C in ((32 * 32, 1024), (64 * 64, 1024), (128 * 128, 512)):
            M = chunk * hw
            for name, N, Kd in (("qkv", 3 * C, C), ("attn_out", C, 2 * C), ("glu_inv", 8 * C, C),
                                ("glu_point", C, 4 * C)):
                if M * max(Kd, N) * 2 < (1 << 31):
                    yield f"dcae{chunk}_{int(hw ** 0.5)}sq_{name}", M, N, Kd
    yield "sana_ff_point_5632", 131072, 2240, 5632


rows = []
for name, M, N, Kd in shapes():
    g = torch.Generator(device=dev).manual_seed(M + N + Kd)
    x = (torch.rand((M, Kd), generator=g, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand((N, Kd), generator=g, device=dev) * 2 - 1) * Kd ** -0.5).bfloat16()
    outs = {k: torch.empty((M, N), device=dev, dtype=torch.bfloat16) for k in (0, 8, 10)}
    fns = {"hipblaslt": lambda: F.linear(x, W)}
    for k in (0, 8, 10):
        fns[f"k{k}"] = (lambda k=k: K.lora_linear_pop(x, W, None, None, 0, 0, 0, 0.0, M, out=outs[k], kernel=k))
    ref = fns["hipblaslt"]().float()
    err = {k: float((fns[k]().float() - ref).abs().max() / ref.abs().max()) for k in fns if k != "hipblaslt"}
    t = {k: [] for k in fns}
    for _ in range(rounds):
        for k, fn in fns.items():
            t[k].append(bench(fn))
    fl = 2.0 * M * N * Kd
    row = {"name": name, "M": M, "N": N, "K": Kd, "auto_tile": K.gemm_tile_for(M, N, 0, M)}
    for k in fns:
        row[f"{k}_ms"] = round(min(t[k]), 4)
        row[f"{k}_tflops"] = round(fl / min(t[k]) / 1e9, 1)
    row["rel_err"] = err
    row["best"] = min(fns, key=lambda k: min(t[k]))
    rows.append(row)
    print(json.dumps(row), flush=True)
    del x, W, outs
if len(sys.argv) > 2:
    Path(sys.argv[2]).write_text(json.dumps(rows, indent=1))
