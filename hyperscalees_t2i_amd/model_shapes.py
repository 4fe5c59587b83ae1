"""LoRA theta layouts of the reference's other backends (BASELINE configs[0], [3], [4]).

theta = the trainable LoRA parameters in module.parameters() order (utills.py:141-152): for every
PEFT target linear, lora_A [r, in] then lora_B [out, r] (get_peft_model suffix matching of the
target list, es_backend.py:334-341 / 587-608 / 832-838).  The ES kernels are shape-generic; these
lists drive them at each config's real sizes.

  var_d16_lora_shapes      VAR-d16 (es_backend.py:299-450, unifed_es.py:403-406: r 4, alpha 16,
                           targets mat_qkv,proj,fc1,fc2,ada_lin.1,head_nm.ada_lin.1,head).  PINNED:
                           equals the layout make_golden.py derives from the reference's own
                           VAR_models module tree (tests/golden/g8_var.npz; 82 targets, D = 1,540,096).
  zimage_turbo_lora_shapes Z-Image-Turbo (es_backend.py:457-678, unifed_es.py:482-485: r 2, targets
                           to_q,to_k,to_v,linear,w1,w2,w3) from the published ZImageTransformer2DModel
                           config (dim 3840, 30 layers + 2 noise-refiner + 2 context-refiner blocks,
                           FFN 10240, final_layer.linear -> 2*2*16); the restated host is zimage.py.
                           UNPINNED: diffusers is absent, so its module tree cannot be walked here.
  infinity_lora_shapes     Infinity (es_backend.py:680-1023, unifed_es.py:469-472: r 2, targets fc1)
                           from models/Infinity.py:164-181 (depth / embed_dim / mlp_ratio per variant)
                           and the Infinity repo's FFN naming (fc1: C -> 4C).  UNPINNED: the Infinity
                           repo is not vendored (models/Infinity.py:19-21).
"""
from __future__ import annotations

from typing import List, Tuple

Shape = Tuple[int, int]


def _lora(pairs, r: int) -> List[Shape]:
    out: List[Shape] = []
    for fin, fout in pairs:
        out += [(r, fin), (fout, r)]
    return out


def var_d16_lora_shapes(r: int = 4, depth: int = 16, vocab: int = 4096) -> List[Shape]:
    """VAR(depth d): width C = 64 d, mlp_ratio 4, AdaLNSelfAttn.ada_lin = (SiLU, Linear(C, 6C)),
    AdaLNBeforeHead.ada_lin = (SiLU, Linear(C, 2C)), head Linear(C, V); module order per block:
    attn.mat_qkv, attn.proj, ffn.fc1, ffn.fc2, ada_lin.1 (VAR_models/basic_var.py registration)."""
    C = 64 * depth
    pairs = []
    for _ in range(depth):
        pairs += [(C, 3 * C), (C, C), (C, 4 * C), (4 * C, C), (C, 6 * C)]
    pairs += [(C, 2 * C), (C, vocab)]
    return _lora(pairs, r)


def zimage_turbo_lora_shapes(r: int = 2, dim: int = 3840, layers: int = 30, refiner_layers: int = 2,
                             ffn: int = 10240, out_ch: int = 64) -> List[Shape]:
    """all_final_layer.*.linear (dim -> patch^2 * C_out) first — diffusers registers the final layer with
    the x embedder, before the blocks — then per transformer block (noise refiner, context refiner, main
    stack): attention.to_q/k/v (dim -> dim) and feed_forward.w1 (dim -> ffn), w2 (ffn -> dim), w3
    (dim -> ffn).  Equal to zimage.zimage_lora_shapes() (the restated module tree, tests/test_zimage.py)."""
    pairs = [(dim, out_ch)]
    for _ in range(2 * refiner_layers + layers):
        pairs += [(dim, dim)] * 3 + [(dim, ffn), (ffn, dim), (dim, ffn)]
    return _lora(pairs, r)


INFINITY_MODELS = {  # models/Infinity.py:164-181
    "infinity_2b": (32, 2048), "infinity_8b": (40, 3584), "infinity_layer12": (12, 768),
    "infinity_layer16": (16, 1152), "infinity_layer24": (24, 1536), "infinity_layer32": (32, 2080),
    "infinity_layer40": (40, 2688), "infinity_layer48": (48, 3360),
}


def infinity_lora_shapes(model_type: str = "infinity_8b", r: int = 2, mlp_ratio: int = 4) -> List[Shape]:
    """One fc1 (C -> mlp_ratio * C) per block."""
    depth, C = INFINITY_MODELS[model_type]
    return _lora([(C, round(C * mlp_ratio))] * depth, r)
