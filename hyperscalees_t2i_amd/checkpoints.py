"""Local diffusers-format checkpoints for the Sana-Sprint host (transformer + DC-AE decoder).

Reference: `SanaTransformer2DModel.from_pretrained(model_name, subfolder="transformer")` and
`AutoencoderDC.from_pretrained(model_name, subfolder="vae")` (models/SanaSprint.py:35-49).  There is
no hub access here, so `model_name` must be a LOCAL directory laid out as diffusers writes it:

    <model_name>/transformer/config.json + diffusion_pytorch_model[-0000k-of-0000n].safetensors
    <model_name>/vae/config.json         + diffusion_pytorch_model[...].safetensors

This module maps diffusers' state-dict keys onto the build's modules (sana.py / dcae.py keep the
diffusers module names for everything on the LoRA path, so PEFT adapter keys match; the convs that
run as libeggroll kernels keep their weights in kernel layouts and are converted here):

  transformer  patch_embed.proj.weight [D, C, 1, 1]          -> patch_w [D, C]
               transformer_blocks.i.ff.conv_inverted [2h,D,1,1] -> ff.w_inv [2h, D] (+ b_inv)
               transformer_blocks.i.ff.conv_depth [2h,1,3,3]    -> ff.w_dw [9, 2h] ([tap][channel]) (+ b_dw)
               transformer_blocks.i.ff.conv_point [D,h,1,1]     -> ff.w_point [D, h]
               every other key                                  -> the same name
  vae          decoder.up_blocks.i.j.*  -> stages.(S-1-i).j.*   (the build lists stages lowest resolution first)
               attn.to_q / to_k / to_v  -> attn.w_qkv = cat(q, k, v) [3C, C]
               attn.to_qkv_multiscale.s.proj_in  [3C,1,k,k]  -> attn.ms_dw.s [k*k, 3C]
               attn.to_qkv_multiscale.s.proj_out [3C,32,1,1] -> attn.ms_pw.s [3C/32, 32, 32] ([group][out][in])
               attn.to_out.weight       -> attn.w_out;  conv_out.conv_inverted / conv_depth / conv_point as above
               encoder.*                -> ignored (decode only)

The key names and layouts are those of diffusers' sana_transformer.py / autoencoder_dc.py as
published; diffusers is not importable in this container and no real checkpoint exists offline, so
the mapping is pinned only by round trips through `save_sana_diffusers` (tests/test_checkpoint_load.py)
— PARITY WITH REAL DIFFUSERS FILES IS UNPINNED.  Loading is strict: a missing key, an unexpected key
(outside encoder.*) or a shape mismatch raises ValueError; a configuration this build does not
implement raises NotImplementedError.  Weights are cast to bf16 (the build's compute dtype).
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
from torch import nn

from .sana import SanaArch

SANA_CLASS = "SanaTransformer2DModel"
DCAE_CLASS = "AutoencoderDC"
WEIGHTS_NAME = "diffusion_pytorch_model.safetensors"
WEIGHTS_INDEX = "diffusion_pytorch_model.safetensors.index.json"


# ---------------------------------------------------------------------------------------
# safetensors directories
# ---------------------------------------------------------------------------------------


def read_state_dir(d: Path) -> Dict[str, torch.Tensor]:
    """All tensors of a diffusers weights directory (single file, or sharded with an index)."""
    from safetensors.torch import load_file
    d = Path(d)
    if (d / WEIGHTS_NAME).is_file():
        return load_file(str(d / WEIGHTS_NAME))
    if (d / WEIGHTS_INDEX).is_file():
        index = json.loads((d / WEIGHTS_INDEX).read_text())
        out: Dict[str, torch.Tensor] = {}
        for shard in sorted(set(index["weight_map"].values())):
            out.update(load_file(str(d / shard)))
        missing = set(index["weight_map"]) - set(out)
        if missing:
            raise ValueError(f"{d}: index names tensors absent from its shards: {sorted(missing)[:3]}")
        return out
    files = sorted(d.glob("*.safetensors"))
    if len(files) == 1:
        return load_file(str(files[0]))
    raise FileNotFoundError(f"{d}: no {WEIGHTS_NAME} (or index) found")


def write_state_dir(d: Path, state: Dict[str, torch.Tensor], config: dict) -> None:
    from safetensors.torch import save_file
    d = Path(d)
    d.mkdir(parents=True, exist_ok=True)
    save_file({k: v.detach().cpu().contiguous() for k, v in state.items()}, str(d / WEIGHTS_NAME))
    (d / "config.json").write_text(json.dumps(config, indent=2))


def read_config(d: Path) -> dict:
    p = Path(d) / "config.json"
    if not p.is_file():
        raise FileNotFoundError(f"{p} not found")
    return json.loads(p.read_text())


# ---------------------------------------------------------------------------------------
# key rules: build parameter <- diffusers tensors
# ---------------------------------------------------------------------------------------

Rule = Tuple[str, List[str], Callable[[List[torch.Tensor]], torch.Tensor], Callable[[torch.Tensor], List[torch.Tensor]]]


def _same(name: str, dkey: Optional[str] = None) -> Rule:
    return (name, [dkey or name], lambda ts: ts[0], lambda t: [t])


def _conv1x1(name: str, dkey: str) -> Rule:
    return (name, [dkey], lambda ts: ts[0].reshape(ts[0].shape[0], -1),
            lambda t: [t.reshape(t.shape[0], t.shape[1], 1, 1)])


def _depthwise(name: str, dkey: str) -> Rule:
    """[C, 1, k, k] depthwise conv weight <-> the build's [k*k, C] ([tap][channel])."""
    def to_b(ts):
        w = ts[0]
        return w.reshape(w.shape[0], -1).t()

    def from_b(t):
        k2, C = t.shape
        k = int(round(k2 ** 0.5))
        return [t.t().reshape(C, 1, k, k)]
    return (name, [dkey], to_b, from_b)


def _grouped32(name: str, dkey: str) -> Rule:
    """[3C, 32, 1, 1] grouped 1x1 conv (groups of 32) <-> the build's [3C/32, 32 out, 32 in]."""
    return (name, [dkey], lambda ts: ts[0].reshape(-1, 32, 32),
            lambda t: [t.reshape(-1, 32, 1, 1)])


def _qkv(name: str, prefix: str) -> Rule:
    keys = [f"{prefix}.to_q.weight", f"{prefix}.to_k.weight", f"{prefix}.to_v.weight"]
    return (name, keys, lambda ts: torch.cat(ts, 0), lambda t: list(t.chunk(3, 0)))


def _frozen_params(model: nn.Module) -> Dict[str, nn.Parameter]:
    return {n: p for n, p in model.named_parameters() if not p.requires_grad}


def sana_rules(model: nn.Module) -> List[Rule]:
    rules: List[Rule] = []
    for n in _frozen_params(model):
        if n == "patch_w":
            rules.append(_conv1x1(n, "patch_embed.proj.weight"))
        elif n == "patch_b":
            rules.append(_same(n, "patch_embed.proj.bias"))
        elif ".ff." in n:
            pre, leaf = n.rsplit(".", 1)
            rules.append({"w_inv": lambda: _conv1x1(n, f"{pre}.conv_inverted.weight"),
                          "b_inv": lambda: _same(n, f"{pre}.conv_inverted.bias"),
                          "w_dw": lambda: _depthwise(n, f"{pre}.conv_depth.weight"),
                          "b_dw": lambda: _same(n, f"{pre}.conv_depth.bias"),
                          "w_point": lambda: _conv1x1(n, f"{pre}.conv_point.weight")}[leaf]())
        else:
            rules.append(_same(n))
    return rules


def dcae_rules(vae: nn.Module) -> List[Rule]:
    S = len(vae.stages)
    rules: List[Rule] = []
    for n in _frozen_params(vae):
        if n.startswith("stages."):
            _, s, rest = n.split(".", 2)
            dn = f"decoder.up_blocks.{S - 1 - int(s)}.{rest}"
        else:
            dn = f"decoder.{n}"
        blk, _, leaf = dn.rpartition(".")
        if blk.endswith(".attn") and leaf == "w_qkv":
            rules.append(_qkv(n, blk))
        elif blk.endswith(".attn") and leaf == "w_out":
            rules.append(_same(n, f"{blk}.to_out.weight"))
        elif ".attn.ms_dw." in dn:
            pre, s_ = dn.split(".ms_dw.")
            rules.append(_depthwise(n, f"{pre}.to_qkv_multiscale.{s_}.proj_in.weight"))
        elif ".attn.ms_pw." in dn:
            pre, s_ = dn.split(".ms_pw.")
            rules.append(_grouped32(n, f"{pre}.to_qkv_multiscale.{s_}.proj_out.weight"))
        elif blk.endswith(".conv_out") and leaf in ("w_inv", "b_inv", "w_dw", "b_dw", "w_point"):
            rules.append({"w_inv": lambda: _conv1x1(n, f"{blk}.conv_inverted.weight"),
                          "b_inv": lambda: _same(n, f"{blk}.conv_inverted.bias"),
                          "w_dw": lambda: _depthwise(n, f"{blk}.conv_depth.weight"),
                          "b_dw": lambda: _same(n, f"{blk}.conv_depth.bias"),
                          "w_point": lambda: _conv1x1(n, f"{blk}.conv_point.weight")}[leaf]())
        else:
            rules.append(_same(n, dn))
    return rules


def state_from_build(model: nn.Module, rules: Sequence[Rule]) -> Dict[str, torch.Tensor]:
    params = _frozen_params(model)
    out: Dict[str, torch.Tensor] = {}
    for name, dkeys, _, from_b in rules:
        for k, t in zip(dkeys, from_b(params[name].detach())):
            out[k] = t.contiguous()
    return out


@torch.no_grad()
def load_into(model: nn.Module, rules: Sequence[Rule], state: Dict[str, torch.Tensor], what: str,
              ignore_prefixes: Sequence[str] = ()) -> None:
    """Strict: every build parameter from its diffusers tensors (shape-checked, cast to the
    parameter's dtype); any checkpoint key no rule reads raises (except ignore_prefixes)."""
    params = _frozen_params(model)
    used = set()
    missing = [k for _, dk, _, _ in rules for k in dk if k not in state]
    if missing:
        raise ValueError(f"{what}: checkpoint lacks {len(missing)} keys, e.g. {missing[:4]}")
    for name, dkeys, to_b, _ in rules:
        t = to_b([state[k] for k in dkeys])
        p = params[name]
        if tuple(t.shape) != tuple(p.shape):
            raise ValueError(f"{what}: {dkeys[0]} gives {tuple(t.shape)} for {name} {tuple(p.shape)}")
        p.copy_(t.to(device=p.device, dtype=p.dtype))
        used.update(dkeys)
    extra = sorted(k for k in state if k not in used and not k.startswith(tuple(ignore_prefixes)))
    if extra:
        raise ValueError(f"{what}: {len(extra)} checkpoint keys are not used by this build, e.g. {extra[:4]}")


# ---------------------------------------------------------------------------------------
# configs
# ---------------------------------------------------------------------------------------


def sana_arch_from_config(cfg: dict) -> SanaArch:
    """diffusers SanaTransformer2DModel config.json -> SanaArch; refuses what sana.py does not build."""
    if cfg.get("_class_name", SANA_CLASS) != SANA_CLASS:
        raise NotImplementedError(f"transformer class {cfg.get('_class_name')!r} (expected {SANA_CLASS})")
    need = {"patch_size": 1, "guidance_embeds": True, "qk_norm": "rms_norm_across_heads", "attention_bias": False,
            "norm_elementwise_affine": False, "interpolation_scale": None}
    for k, v in need.items():
        if k in cfg and cfg[k] != v:
            raise NotImplementedError(f"transformer config {k}={cfg[k]!r}: this build implements {v!r}")
    if float(cfg.get("timestep_scale", 1.0) or 1.0) != 1.0 or float(cfg.get("dropout", 0.0) or 0.0) != 0.0:
        raise NotImplementedError("transformer config: timestep_scale != 1 / dropout != 0 are not implemented")
    a = SanaArch(in_channels=int(cfg.get("in_channels", 32)),
                 out_channels=int(cfg.get("out_channels") or cfg.get("in_channels", 32)),
                 num_attention_heads=int(cfg.get("num_attention_heads", 70)),
                 attention_head_dim=int(cfg.get("attention_head_dim", 32)),
                 num_layers=int(cfg.get("num_layers", 20)),
                 num_cross_attention_heads=int(cfg.get("num_cross_attention_heads", 20)),
                 cross_attention_head_dim=int(cfg.get("cross_attention_head_dim", 112)),
                 caption_channels=int(cfg.get("caption_channels", 2304)),
                 mlp_ratio=float(cfg.get("mlp_ratio", 2.5)),
                 norm_eps=float(cfg.get("norm_eps", 1e-6)),
                 guidance_embeds_scale=float(cfg.get("guidance_embeds_scale", 0.1)),
                 sample_size=int(cfg.get("sample_size", 32)))
    if int(cfg.get("cross_attention_dim", a.inner_dim)) != a.inner_dim:
        raise NotImplementedError("transformer config: cross_attention_dim != inner dim")
    return a


def sana_config_from_arch(a: SanaArch) -> dict:
    return {"_class_name": SANA_CLASS, "in_channels": a.in_channels, "out_channels": a.out_channels,
            "num_attention_heads": a.num_attention_heads, "attention_head_dim": a.attention_head_dim,
            "num_layers": a.num_layers, "num_cross_attention_heads": a.num_cross_attention_heads,
            "cross_attention_head_dim": a.cross_attention_head_dim, "cross_attention_dim": a.inner_dim,
            "caption_channels": a.caption_channels, "mlp_ratio": a.mlp_ratio, "dropout": 0.0,
            "attention_bias": False, "sample_size": a.sample_size, "patch_size": 1,
            "norm_elementwise_affine": False, "norm_eps": a.norm_eps, "interpolation_scale": None,
            "guidance_embeds": True, "guidance_embeds_scale": a.guidance_embeds_scale,
            "qk_norm": "rms_norm_across_heads", "timestep_scale": 1.0}


def dcae_build_kwargs(cfg: dict) -> dict:
    """diffusers AutoencoderDC config.json -> DCAEDecoder kwargs (decoder side only)."""
    if cfg.get("_class_name", DCAE_CLASS) != DCAE_CLASS:
        raise NotImplementedError(f"vae class {cfg.get('_class_name')!r} (expected {DCAE_CLASS})")
    widths = [int(w) for w in cfg["decoder_block_out_channels"]]
    layers = [int(x) for x in cfg["decoder_layers_per_block"]]
    n = len(widths)

    def per_stage(v, default):
        v = cfg.get(v, default)
        return [v] * n if isinstance(v, str) or not isinstance(v, (list, tuple)) else list(v)
    types = per_stage("decoder_block_types", "ResBlock")
    norms = per_stage("decoder_norm_types", "rms_norm")
    acts = per_stage("decoder_act_fns", "silu")
    ms = cfg.get("decoder_qkv_multiscales", [[]] * n)
    vit_from = next((i for i, t in enumerate(types) if t == "EfficientViTBlock"), n)
    ok = (all(t == ("ResBlock" if i < vit_from else "EfficientViTBlock") for i, t in enumerate(types))
          and all(x == "rms_norm" for x in norms) and all(x == "silu" for x in acts[:vit_from])
          and all(list(ms[i]) == ([5] if i >= vit_from else []) for i in range(n))
          and cfg.get("upsample_block_type", "interpolate") == "interpolate"
          and int(cfg.get("attention_head_dim", 32)) == 32 and int(cfg.get("in_channels", 3)) == 3
          and layers[0] > 0 and all(x > 0 for x in layers))
    if not ok:
        raise NotImplementedError("vae config: this build implements the DC-AE f32c32 decoder family only "
                                  "(ResBlocks then EfficientViT blocks with multiscale (5,), rms_norm, silu, "
                                  "interpolate up-blocks, head dim 32)")
    return dict(latent_channels=int(cfg.get("latent_channels", 32)), widths=tuple(widths), layers=tuple(layers),
                vit_from=vit_from, scaling_factor=float(cfg.get("scaling_factor", 0.41407)))


def dcae_config_from_build(vae: nn.Module) -> dict:
    widths, layers, vit_from = vae.widths, vae.layers, vae.vit_from
    n = len(widths)
    return {"_class_name": DCAE_CLASS, "in_channels": 3, "latent_channels": vae.latent_channels,
            "attention_head_dim": 32, "decoder_block_out_channels": list(widths),
            "decoder_layers_per_block": list(layers),
            "decoder_block_types": ["ResBlock" if i < vit_from else "EfficientViTBlock" for i in range(n)],
            "decoder_norm_types": "rms_norm", "decoder_act_fns": "silu",
            "decoder_qkv_multiscales": [[] if i < vit_from else [5] for i in range(n)],
            "upsample_block_type": "interpolate", "scaling_factor": vae.scaling_factor}


# ---------------------------------------------------------------------------------------
# whole-model load / save
# ---------------------------------------------------------------------------------------


def is_local_model_dir(model_name: str) -> bool:
    p = Path(model_name)
    return p.is_dir() and (p / "transformer").is_dir() and (p / "vae").is_dir()


def load_sana_transformer(model, d: Path) -> None:
    load_into(model, sana_rules(model), read_state_dir(d), f"{d} (transformer)")


def load_dcae_decoder(vae, d: Path) -> None:
    load_into(vae, dcae_rules(vae), read_state_dir(d), f"{d} (vae)", ignore_prefixes=("encoder.",))
    refresh_dcae_caches(vae)


def refresh_dcae_caches(vae) -> None:
    """The kernel-layout copies the decoder derives from its 3x3 weights (phase / packed weights)."""
    from .dcae import ResBlock, UpBlock
    for m in vae.modules():
        if isinstance(m, UpBlock):
            m.refresh_phase_weights()
        if isinstance(m, ResBlock):
            m.refresh_packed_weights()


def save_sana_diffusers(transformer, vae, out_dir: Path) -> None:
    """Write the build's frozen weights as a diffusers model directory (transformer/ + vae/, decoder
    keys only): the inverse of the loader, used by the round-trip tests and for exporting."""
    out = Path(out_dir)
    write_state_dir(out / "transformer", state_from_build(transformer, sana_rules(transformer)),
                    sana_config_from_arch(transformer.config))
    write_state_dir(out / "vae", state_from_build(vae, dcae_rules(vae)), dcae_config_from_build(vae))


# ---------------------------------------------------------------------------------------
# Z-Image-Turbo (BASELINE configs[3]): diffusers ZImageTransformer2DModel + FLUX AutoencoderKL
# ---------------------------------------------------------------------------------------
# Reference: ZImagePipeline.from_pretrained(model_name) (models/zImageTurbo.py:97-125).  zimage.py keeps
# diffusers' module names (all_x_embedder."2-1", all_final_layer."2-1", noise_refiner / context_refiner /
# layers .attention.to_q|to_k|to_v|to_out.0 / norm_q|norm_k, .feed_forward.w1|w2|w3, attention_norm1|2,
# ffn_norm1|2, adaLN_modulation.0, t_embedder.mlp.0|2, cap_embedder.0|1, x_pad_token, cap_pad_token), so the
# transformer maps key for key; flux_vae.py lists the decoder as conv_in / mid.0-2 / up_blocks.i.resnets.j /
# up_blocks.i.upsample / conv_norm_out / conv_out, mapped to diffusers' decoder.* names below.  Like the Sana
# loader, the key names follow the published diffusers modules and are UNPINNED here (no diffusers, no weights).

ZIMAGE_CLASS = "ZImageTransformer2DModel"
AUTOENCODER_KL_CLASS = "AutoencoderKL"


def zimage_rules(model: nn.Module) -> List[Rule]:
    return [_same(n) for n in _frozen_params(model)]


def flux_decoder_name(n: str) -> str:
    """A flux_vae.py parameter name -> the diffusers `Decoder` module's own name for it (relative to
    vae.decoder): mid.0 / mid.1 / mid.2 -> mid_block.resnets.0 / mid_block.attentions.0 /
    mid_block.resnets.1, up_blocks.i.upsample.* -> up_blocks.i.upsamplers.0.conv.*, the rest as is."""
    head, _, rest = n.partition(".")
    if head == "mid":
        i, _, leaf = rest.partition(".")
        return {"0": "mid_block.resnets.0.", "2": "mid_block.resnets.1.", "1": "mid_block.attentions.0."}[i] + leaf
    if head == "up_blocks" and ".upsample." in n:
        i = rest.split(".")[0]
        return f"up_blocks.{i}.upsamplers.0.conv.{n.rsplit('.', 1)[1]}"
    return n


def flux_vae_rules(vae: nn.Module) -> List[Rule]:
    return [_same(n, "decoder." + flux_decoder_name(n)) for n in _frozen_params(vae)]


def zimage_arch_from_config(cfg: dict):
    """diffusers ZImageTransformer2DModel config.json -> ZImageArch; refuses what zimage.py does not build."""
    from .zimage import ZImageArch
    if cfg.get("_class_name", ZIMAGE_CLASS) != ZIMAGE_CLASS:
        raise NotImplementedError(f"transformer class {cfg.get('_class_name')!r} (expected {ZIMAGE_CLASS})")
    ps, fps = list(cfg.get("all_patch_size", [2])), list(cfg.get("all_f_patch_size", [1]))
    if len(ps) != 1 or len(fps) != 1 or int(fps[0]) != 1:
        raise NotImplementedError(f"transformer config: patch sizes {ps} / {fps} (this build: one patch size, f 1)")
    heads = int(cfg.get("n_heads", 30))
    if int(cfg.get("n_kv_heads", heads)) != heads or not bool(cfg.get("qk_norm", True)):
        raise NotImplementedError("transformer config: grouped kv heads / no qk_norm are not implemented")
    dim = int(cfg.get("dim", 3840))
    return ZImageArch(in_channels=int(cfg.get("in_channels", 16)), patch=int(ps[0]), dim=dim,
                      n_layers=int(cfg.get("n_layers", 30)), n_refiner_layers=int(cfg.get("n_refiner_layers", 2)),
                      n_heads=heads, ffn=int(dim / 3 * 8), norm_eps=float(cfg.get("norm_eps", 1e-5)),
                      cap_feat_dim=int(cfg.get("cap_feat_dim", 2560)), adaln_dim=min(dim, 256),
                      t_scale=float(cfg.get("t_scale", 1000.0)), rope_theta=float(cfg.get("rope_theta", 256.0)),
                      axes_dims=tuple(int(x) for x in cfg.get("axes_dims", (32, 48, 48))))


def zimage_config_from_arch(a) -> dict:
    return {"_class_name": ZIMAGE_CLASS, "all_patch_size": [a.patch], "all_f_patch_size": [1],
            "in_channels": a.in_channels, "dim": a.dim, "n_layers": a.n_layers, "n_refiner_layers": a.n_refiner_layers,
            "n_heads": a.n_heads, "n_kv_heads": a.n_heads, "norm_eps": a.norm_eps, "qk_norm": True,
            "cap_feat_dim": a.cap_feat_dim, "rope_theta": a.rope_theta, "t_scale": a.t_scale,
            "axes_dims": list(a.axes_dims), "axes_lens": [1024, 512, 512]}


def flux_vae_kwargs(cfg: dict) -> dict:
    """diffusers AutoencoderKL config.json -> FluxVAEDecoder kwargs (decoder side)."""
    if cfg.get("_class_name", AUTOENCODER_KL_CLASS) != AUTOENCODER_KL_CLASS:
        raise NotImplementedError(f"vae class {cfg.get('_class_name')!r} (expected {AUTOENCODER_KL_CLASS})")
    if cfg.get("use_post_quant_conv", False) or int(cfg.get("norm_num_groups", 32)) != 32 or \
            cfg.get("act_fn", "silu") != "silu" or not cfg.get("mid_block_add_attention", True) or \
            int(cfg.get("out_channels", 3)) != 3:
        raise NotImplementedError("vae config: this build implements the FLUX AutoencoderKL decoder only (no post-quant "
                                  "conv, GroupNorm(32), SiLU, mid-block attention, 3 output channels)")
    return dict(latent_channels=int(cfg.get("latent_channels", 16)),
                widths=tuple(int(w) for w in cfg.get("block_out_channels", (128, 256, 512, 512))),
                layers=int(cfg.get("layers_per_block", 2)),
                scaling_factor=float(cfg.get("scaling_factor", 0.3611)),
                shift_factor=float(cfg.get("shift_factor", 0.1159) or 0.0))


def flux_vae_config_from_build(vae: nn.Module) -> dict:
    widths = [int(vae.conv_norm_out.weight.shape[0])] + [int(b.resnets[-1].conv2.weight.shape[0])
                                                          for b in reversed(list(vae.up_blocks))][1:]
    return {"_class_name": AUTOENCODER_KL_CLASS, "in_channels": 3, "out_channels": 3,
            "latent_channels": int(vae.conv_in.weight.shape[1]), "block_out_channels": widths,
            "layers_per_block": len(vae.up_blocks[0].resnets) - 1, "norm_num_groups": 32, "act_fn": "silu",
            "scaling_factor": vae.scaling_factor, "shift_factor": vae.shift_factor, "use_quant_conv": False,
            "use_post_quant_conv": False, "mid_block_add_attention": True}


def load_zimage_transformer(model, d: Path) -> None:
    load_into(model, zimage_rules(model), read_state_dir(d), f"{d} (transformer)")


def load_flux_vae_decoder(vae, d: Path) -> None:
    load_into(vae, flux_vae_rules(vae), read_state_dir(d), f"{d} (vae)",
              ignore_prefixes=("encoder.", "quant_conv."))


def save_zimage_diffusers(transformer, vae, out_dir: Path) -> None:
    """The build's frozen Z-Image weights as a diffusers directory (transformer/ + vae/ decoder keys)."""
    out = Path(out_dir)
    write_state_dir(out / "transformer", state_from_build(transformer, zimage_rules(transformer)),
                    zimage_config_from_arch(transformer.config))
    write_state_dir(out / "vae", state_from_build(vae, flux_vae_rules(vae)), flux_vae_config_from_build(vae))


# ---------------------------------------------------------------------------------------
# Infinity (BASELINE configs[4]): the Infinity repo's state dicts
# ---------------------------------------------------------------------------------------
# Reference: InfinityES._load_infinity (models/Infinity.py:183-235) builds `Infinity(...)` and loads
# checkpoint_type "torch" (one .pth: torch.load + load_state_dict) or "torch_shard" (a directory with an
# index, transformers.load_sharded_checkpoint(strict=False)); the BSQ-VAE comes from vae_path (a .pth).
# infinity.py keeps the repo's module names where it can (block_chunks.i.module.j.{sa,ca,ffn,ca_norm,ada_gss},
# shared_ada_lin.1, head_nm.ada_lin.1, head, word_embed, text_norm, text_proj_for_ca.0|2, cfg_uncond, pos_start)
# and folds the repo's separate bias vectors into its linears' biases:
#   sa.q_bias, sa.v_bias (+ the zero_k_bias buffer)        -> sa.mat_qkv.bias = [q_bias | 0 | v_bias]
#   ca.v_bias (+ zero_k_bias)                              -> ca.mat_kv.bias  = [0 | v_bias]
#   sa.scale_mul_1H11 [1, 1, H, 1] (flash) or [1, H, 1, 1] -> [1, H, 1, 1]
#   lvl_embed.weight (nn.Embedding)                        -> lvl_embed
#   text_proj_for_sos.ca.{mat_q [1, 1, C], mat_kv.weight, v_bias, proj.*} -> text_proj_for_sos.{query, mat_kv, proj}
# The BSQ-VAE decoder follows the LDM / FLUX autoencoder naming (decoder.conv_in, decoder.mid.block_1 / attn_1 /
# block_2, decoder.up.L.block.j.{norm1,conv1,norm2,conv2,nin_shortcut}, decoder.up.L.upsample.conv with L = 0
# the full-resolution level, decoder.norm_out, decoder.conv_out; 1x1-conv q / k / v / proj_out).  The Infinity
# repo is not vendored: these names are UNPINNED against real files; the loader is strict (the reference's
# shard path is strict=False — here a missing or unused tensor raises rather than leaving random weights).

INFINITY_SHARD_INDEX = ("pytorch_model.bin.index.json", "model.safetensors.index.json")
# persistent buffers of the Infinity modules that carry no learned value in this build
INFINITY_BUFFER_SUFFIXES = ("zero_k_bias", "lvl_1L", "attn_bias_for_masking")


def _fold_bias(name: str, keys: List[str], layout: str, C: int) -> Rule:
    """layout "q0v": [q | 0 | v] from (q_bias, v_bias); "0v": [0 | v] from (v_bias,)."""
    if layout == "q0v":
        return (name, keys, lambda ts: torch.cat([ts[0], torch.zeros_like(ts[0]), ts[1]]),
                lambda t: [t[:C], t[2 * C:]])
    return (name, keys, lambda ts: torch.cat([torch.zeros_like(ts[0]), ts[0]]), lambda t: [t[C:]])


def infinity_rules(model: nn.Module) -> List[Rule]:
    C = model.arch.C
    H = model.arch.num_heads
    rules: List[Rule] = []
    for n in _frozen_params(model):
        if n.endswith(".sa.mat_qkv.bias"):
            p = n[: -len(".mat_qkv.bias")]
            rules.append(_fold_bias(n, [f"{p}.q_bias", f"{p}.v_bias"], "q0v", C))
        elif n.endswith(".ca.mat_kv.bias"):
            p = n[: -len(".mat_kv.bias")]
            rules.append(_fold_bias(n, [f"{p}.v_bias"], "0v", C))
        elif n.endswith(".sa.scale_mul_1H11"):
            rules.append((n, [n], lambda ts: ts[0].reshape(1, H, 1, 1), lambda t: [t.reshape(1, H, 1, 1)]))
        elif n == "lvl_embed":
            rules.append(_same(n, "lvl_embed.weight"))
        elif n == "text_proj_for_sos.query":
            rules.append((n, ["text_proj_for_sos.ca.mat_q"], lambda ts: ts[0].reshape(-1),
                          lambda t: [t.reshape(1, 1, -1)]))
        elif n == "text_proj_for_sos.mat_kv.bias":
            rules.append(_fold_bias(n, ["text_proj_for_sos.ca.v_bias"], "0v", C))
        elif n.startswith("text_proj_for_sos."):
            rules.append(_same(n, "text_proj_for_sos.ca." + n[len("text_proj_for_sos."):]))
        else:
            rules.append(_same(n))
    return rules


def bsq_vae_rules(vae: nn.Module) -> List[Rule]:
    """FluxVAEDecoder (up_blocks listed lowest resolution first) <- LDM decoder keys (up.L, L = 0 the full
    resolution level)."""
    n_up = len(vae.up_blocks)
    rules: List[Rule] = []
    for n in _frozen_params(vae):
        parts = n.split(".")
        if parts[0] == "mid":
            sub = {"0": "block_1", "1": "attn_1", "2": "block_2"}[parts[1]]
            leaf = ".".join(parts[2:])
            if sub == "attn_1":
                lin, _, wb = leaf.rpartition(".")
                if lin in ("to_q", "to_k", "to_v", "to_out.0"):
                    dk = f"decoder.mid.attn_1.{ {'to_q': 'q', 'to_k': 'k', 'to_v': 'v', 'to_out.0': 'proj_out'}[lin] }.{wb}"
                    rules.append(_conv1x1(n, dk) if wb == "weight" else _same(n, dk))
                    continue
                leaf = leaf.replace("group_norm", "norm")
            rules.append(_same(n, f"decoder.mid.{sub}.{leaf}"))
        elif parts[0] == "up_blocks":
            lvl = n_up - 1 - int(parts[1])
            if parts[2] == "upsample":
                rules.append(_same(n, f"decoder.up.{lvl}.upsample.conv.{parts[3]}"))
            else:   # resnets.j.<m>.<w|b>
                m = "nin_shortcut" if parts[4] == "conv_shortcut" else parts[4]
                rules.append(_same(n, f"decoder.up.{lvl}.block.{parts[3]}.{m}.{parts[5]}"))
        elif parts[0] == "conv_norm_out":
            rules.append(_same(n, f"decoder.norm_out.{parts[1]}"))
        else:
            rules.append(_same(n, f"decoder.{n}"))
    return rules


def _torch_state(path: Path) -> Dict[str, torch.Tensor]:
    """A torch-saved state dict, loaded with weights_only=True (no code from the file runs); a dict whose
    tensors sit under one of the usual wrapper keys is unwrapped."""
    sd = torch.load(str(path), map_location="cpu", weights_only=True)
    for k in ("state_dict", "model", "vae", "module"):
        if isinstance(sd, dict) and k in sd and isinstance(sd[k], dict) and not torch.is_tensor(sd[k]):
            sd = sd[k]
            break
    if not isinstance(sd, dict) or not all(torch.is_tensor(v) for v in sd.values()):
        raise ValueError(f"{path}: not a state dict of tensors")
    return dict(sd)


def read_infinity_state(model_path: Path, checkpoint_type: str) -> Dict[str, torch.Tensor]:
    """checkpoint_type "torch": one .pth file; "torch_shard": a directory with pytorch_model.bin.index.json
    (or model.safetensors.index.json) naming its shards."""
    p = Path(model_path)
    if checkpoint_type == "torch":
        if not p.is_file():
            raise FileNotFoundError(f"{p}: Infinity checkpoint file not found")
        return _torch_state(p)
    if checkpoint_type != "torch_shard":
        raise ValueError(f"checkpoint_type must be 'torch' or 'torch_shard', got {checkpoint_type}")
    idx = next((p / n for n in INFINITY_SHARD_INDEX if (p / n).is_file()), None) if p.is_dir() else None
    if idx is None:
        raise FileNotFoundError(f"{p}: no shard index ({' / '.join(INFINITY_SHARD_INDEX)})")
    wmap = json.loads(idx.read_text())["weight_map"]
    out: Dict[str, torch.Tensor] = {}
    for shard in sorted(set(wmap.values())):
        if shard.endswith(".safetensors"):
            from safetensors.torch import load_file
            out.update(load_file(str(p / shard)))
        else:
            out.update(_torch_state(p / shard))
    missing = set(wmap) - set(out)
    if missing:
        raise ValueError(f"{p}: index names tensors absent from its shards: {sorted(missing)[:3]}")
    return out


def _strip_buffers(state: Dict[str, torch.Tensor], what: str) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in state.items():
        if k.endswith(INFINITY_BUFFER_SUFFIXES):
            if k.endswith("zero_k_bias") and bool(v.float().abs().max() > 0):
                raise ValueError(f"{what}: {k} is not zero (the build folds a zero k bias)")
            continue
        out[k] = v
    return out


def load_infinity_transformer(model, model_path: Path, checkpoint_type: str) -> None:
    what = f"{model_path} (Infinity)"
    load_into(model, infinity_rules(model), _strip_buffers(read_infinity_state(model_path, checkpoint_type), what),
              what, ignore_prefixes=("vae_local.",))


def load_bsq_vae_decoder(vae, vae_path: Path) -> None:
    p = Path(vae_path)
    if not p.is_file():
        raise FileNotFoundError(f"{p}: BSQ-VAE checkpoint not found")
    load_into(vae, bsq_vae_rules(vae), _torch_state(p), f"{p} (vae)",
              ignore_prefixes=("encoder.", "quantizer.", "quantize.", "quant_conv.", "post_quant_conv."))


def save_infinity_checkpoint(model, vae, model_path: Path, vae_path: Path, shards: int = 0) -> None:
    """The build's frozen Infinity weights in the repo's layout (zero_k_bias buffers included): one .pth
    (shards 0) or a shard directory with pytorch_model.bin.index.json; the VAE decoder as a .pth."""
    st = state_from_build(model, infinity_rules(model))
    C = model.arch.C
    for blk in [f"block_chunks.{i}.module.{j}" for i, ch in enumerate(model.block_chunks) for j in range(len(ch.module))]:
        st[f"{blk}.sa.zero_k_bias"] = torch.zeros(C, dtype=torch.bfloat16)
        st[f"{blk}.ca.zero_k_bias"] = torch.zeros(C, dtype=torch.bfloat16)
    st["text_proj_for_sos.ca.zero_k_bias"] = torch.zeros(C, dtype=torch.bfloat16)
    st = {k: v.detach().cpu().contiguous() for k, v in st.items()}
    mp = Path(model_path)
    if shards <= 0:
        mp.parent.mkdir(parents=True, exist_ok=True)
        torch.save(st, str(mp))
    else:
        mp.mkdir(parents=True, exist_ok=True)
        keys = sorted(st)
        wmap = {}
        for s in range(shards):
            part = {k: st[k] for k in keys[s::shards]}
            fn = f"pytorch_model-{s + 1:05d}-of-{shards:05d}.bin"
            torch.save(part, str(mp / fn))
            wmap.update({k: fn for k in part})
        (mp / INFINITY_SHARD_INDEX[0]).write_text(json.dumps({"metadata": {}, "weight_map": wmap}, indent=1))
    vp = Path(vae_path)
    vp.parent.mkdir(parents=True, exist_ok=True)
    torch.save({k: v.detach().cpu().contiguous() for k, v in state_from_build(vae, bsq_vae_rules(vae)).items()}, str(vp))
