"""Checkpoint format (es_backend.py:1025-1054) and reward preprocessing (rewards.py:86-90,133-147)
parity, CPU.

* save_latest_checkpoint writes theta into the LoRA params, a PEFT-style adapter dir
  (adapter_model.safetensors with keys base_model.model.<module>.lora_{A,B}.weight + adapter_config.json)
  and the meta .pt with theta_latest; theta_latest loads with torch.load(weights_only=True) and the
  adapter reproduces theta through the reference's unflatten order; load_lora / load_latest_checkpoint
  resume it.
* clip_preprocess(postprocess_uint8(x)) vs transformers' CLIPImageProcessor on the PIL images the
  reference builds (PixArtImageProcessor.postprocess -> PIL).  torchvision is absent in this image, so
  transformers runs its PIL backend (CLIPImageProcessorPil): Pillow BICUBIC resize of the short edge
  to 224, center crop 224, /255, CLIP mean/std.  The build restates Pillow's fixed-point separable
  resampling on the device (rewards.pil_bicubic_resize): BIT-EXACT, square and non-square sizes.
"""
import json

import numpy as np
import pytest
import torch

from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig
from hyperscalees_t2i_amd.es import flatten_params
from hyperscalees_t2i_amd.es_step import load_latest_checkpoint, save_latest_checkpoint
from hyperscalees_t2i_amd.pipeline import to_pil
from hyperscalees_t2i_amd.rewards import clip_preprocess, postprocess_uint8
from hyperscalees_t2i_amd.sana import SanaArch

TINY = SanaArch(num_attention_heads=4, attention_head_dim=32, num_layers=2, num_cross_attention_heads=2,
                cross_attention_head_dim=64, caption_channels=2304)


@pytest.fixture(scope="module")
def backend_cpu():
    cfg = SanaConfig(synthetic_weights=True, width_latent=4, height_latent=4, arch=TINY, vae_widths=(16, 32, 32, 64, 64, 64),
                     vae_layers=(1, 1, 1, 1, 1, 1))
    be = SanaBackend("cpu", cfg)
    be.init_and_attach_lora()
    return be


def test_checkpoint_roundtrip_peft_format(backend_cpu, tmp_path):
    from safetensors.torch import load_file
    be = backend_cpu
    params, shapes = be.collect_lora_params()
    theta = torch.randn(sum(p.numel() for p in params), generator=torch.Generator().manual_seed(3))
    save_latest_checkpoint(theta=theta, backend=be, lora_params=params, lora_shapes=shapes,
                           save_dir=tmp_path / "lora_latest", meta_path=tmp_path / "latest_lora_meta.pt", epoch=7,
                           stats={"summary/mean_reward": 0.25}, extra_meta={"run_name": "r", "wandb_project": "p"})
    ad = load_file(str(tmp_path / "lora_latest" / "adapter_model.safetensors"))
    names = [n for n, p in be.es_model.transformer.named_parameters() if p.requires_grad]
    assert list(ad) and set(ad) == {f"base_model.model.{n}" for n in names}
    assert all(k.endswith((".lora_A.weight", ".lora_B.weight")) for k in ad)
    # the adapter tensors, flattened in parameter order, ARE theta (utills.py:141-162 layout)
    assert torch.equal(torch.cat([ad[f"base_model.model.{n}"].reshape(-1) for n in names]), theta)
    cfg = json.loads((tmp_path / "lora_latest" / "adapter_config.json").read_text())
    assert cfg["peft_type"] == "LORA" and cfg["r"] == 2 and cfg["lora_alpha"] == 8
    assert cfg["target_modules"] == be.cfg.lora_target_modules
    th, meta = load_latest_checkpoint(tmp_path / "latest_lora_meta.pt")
    assert torch.equal(th, theta) and meta["epoch"] == 7 and meta["backend"] == be.name
    assert meta["summary_mean_reward"] == 0.25 and meta["run_name"] == "r"
    # resume: scramble the params, reload the adapter dir -> theta again
    with torch.no_grad():
        for p in params:
            p.zero_()
    be.load_lora(tmp_path / "lora_latest")
    assert torch.equal(flatten_params(params), theta)


def test_load_lora_rejects_foreign_adapter(backend_cpu, tmp_path):
    from safetensors.torch import save_file
    (tmp_path / "x").mkdir()
    save_file({"base_model.model.nope.lora_A.weight": torch.zeros(2, 2)}, str(tmp_path / "x" / "adapter_model.safetensors"))
    with pytest.raises(ValueError):
        backend_cpu.load_lora(tmp_path / "x")


def _images(n, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    base = torch.nn.functional.interpolate(torch.rand(n, 3, max(2, H // 16), max(2, W // 16), generator=g) * 2 - 1,
                                           size=(H, W), mode="bilinear", align_corners=False)
    return (base + 0.15 * torch.randn(n, 3, H, W, generator=g)).clamp(-1.1, 1.1)


@pytest.mark.parametrize("H,W", [(128, 128), (256, 256), (512, 512), (224, 336), (300, 200), (97, 301)])
def test_clip_preprocess_matches_transformers_processor(H, W):
    from transformers import CLIPImageProcessorPil
    proc = CLIPImageProcessorPil()
    x = _images(3, H, W, H * 7 + W)
    ours = clip_preprocess(postprocess_uint8(x)).numpy()
    ref = proc(images=to_pil(x), return_tensors="pt")["pixel_values"].numpy()
    assert ours.shape == ref.shape == (3, 3, 224, 224)
    assert np.array_equal(ours, ref), (H, W, float(np.abs(ours - ref).max()))


@pytest.mark.gpu
def test_clip_preprocess_on_device_1024(dev):
    """The on-device path at the benchmark resolution (1024 px): the 8-bit resampled pixels are
    bit-exact vs Pillow; the float normalisation ((x/255 - mean) / std) runs in device fp32
    arithmetic, within 1 ulp-scale of the processor's numpy fp32."""
    from PIL import Image
    from transformers import CLIPImageProcessorPil
    from hyperscalees_t2i_amd.rewards import pil_bicubic_resize
    x = _images(4, 1024, 1024, 11).to(torch.bfloat16).float()
    pils = to_pil(x)
    u8_dev = pil_bicubic_resize(postprocess_uint8(x.to(dev)), 224, 224).cpu().numpy()
    u8_pil = np.stack([np.asarray(im.resize((224, 224), Image.BICUBIC)) for im in pils]).transpose(0, 3, 1, 2)
    assert np.array_equal(u8_dev, u8_pil.astype(np.float64))
    ours = clip_preprocess(postprocess_uint8(x.to(dev))).cpu().numpy()
    ref = CLIPImageProcessorPil()(images=pils, return_tensors="pt")["pixel_values"].numpy()
    assert np.abs(ours - ref).max() <= 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("H,W", [(1024, 1024), (256, 256), (224, 336), (300, 200), (97, 301)])
def test_clip_pixels_hip_bitexact(dev, H, W):
    """eggroll_clip_preprocess (one HIP pass per resize direction, int32 Pillow taps, fused uint8
    conversion and normalisation) == the torch restatement on the CPU, which
    test_clip_preprocess_matches_transformers_processor pins to transformers bit for bit; both PIL
    conversions (0: PixArt rounding, Sana; 1: fp16 + truncation, VAR; 2: bf16 + truncation, Infinity);
    NHWC-strided input."""
    from hyperscalees_t2i_amd.rewards import clip_pixels
    from hyperscalees_t2i_amd.var import quantize_uint8_var
    x = _images(3, H, W, H * 3 + W).to(torch.bfloat16)
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    from hyperscalees_t2i_amd.infinity_pipeline import images_to_uint8
    for mode, to_u8 in ((0, lambda t: postprocess_uint8(t)), (1, quantize_uint8_var), (2, images_to_uint8)):
        ref = clip_preprocess(to_u8(x)).numpy()
        ours = clip_pixels(xd, mode).cpu().numpy()
        assert ours.shape == ref.shape == (3, 3, 224, 224)
        assert np.array_equal(ours, ref), (mode, float(np.abs(ours - ref).max()))


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["tiny", "b32", "h14"])
def test_clip_vision_tower_matches_transformers(dev, which):
    """The fused reward tower (one qkv GEMM, unfold patch GEMM, [CLS]-only last layer, padded SDPA
    head dim) vs transformers' CLIPModel.get_image_features on the same bf16 weights and pixels."""
    from hyperscalees_t2i_amd.clip_tower import CLIPVisionTower
    from hyperscalees_t2i_amd.rewards import CLIP_B32, CLIP_H14, CLIP_TINY, _image_features, build_clip
    model = build_clip({"tiny": CLIP_TINY, "b32": CLIP_B32, "h14": CLIP_H14}[which], dev, seed=5)
    g = torch.Generator(device=dev).manual_seed(1)
    px = torch.randn((6, 3, 224, 224), generator=g, device=dev)
    ref = _image_features(model, px)
    ours = CLIPVisionTower(model)(px)
    rel = float((ours - ref).norm() / ref.norm())
    cos = float(torch.nn.functional.cosine_similarity(ours, ref, dim=-1).min())
    print(f"[clip tower {which}] rel {rel:.2e} min cos {cos:.6f}")
    assert rel < 2e-2 and cos > 0.9995


@pytest.mark.gpu
def test_clip_h14_tower_fused_gelu_bitexact(dev):
    """CLIP-H/14 at the epoch's batch (64 images: the 8-phase fc1 path): exact GELU in fc1's GEMM epilogue
    gives the same image embeddings, bit for bit, as fc1 followed by torch's F.gelu (the default, which
    measured faster)."""
    from hyperscalees_t2i_amd.clip_tower import CLIPVisionTower
    from hyperscalees_t2i_amd.rewards import CLIP_H14, build_clip
    model = build_clip(CLIP_H14, dev, seed=7)
    g = torch.Generator(device=dev).manual_seed(3)
    px = torch.randn((64, 3, 224, 224), generator=g, device=dev)
    fused, plain = CLIPVisionTower(model, fused_gelu=True), CLIPVisionTower(model, fused_gelu=False)
    assert fused.fused_gelu and not plain.fused_gelu
    assert torch.equal(fused(px), plain(px))


def test_var_checkpoint_roundtrip(tmp_path):
    """VarBackend save_lora / load_lora (shared adapter helpers) on CPU at a tiny VAR: the adapter holds
    every theta entry in parameter order — the mat_qkv LoRA entries the reference's F.linear bypasses
    included — and resume restores theta exactly."""
    from safetensors.torch import load_file
    from hyperscalees_t2i_amd.backend import VarBackend, VarConfig
    from hyperscalees_t2i_amd.var import VARArch
    be = VarBackend("cpu", VarConfig(arch=VARArch(depth=2, vae_ch=32), ckpt_dir="/nonexistent", synthetic_if_missing=True))
    be.init_and_attach_lora()
    params, shapes = be.collect_lora_params()
    theta = torch.randn(sum(p.numel() for p in params), generator=torch.Generator().manual_seed(5))
    save_latest_checkpoint(theta=theta, backend=be, lora_params=params, lora_shapes=shapes,
                           save_dir=tmp_path / "var_lora", meta_path=tmp_path / "var_meta.pt", epoch=2, stats={},
                           extra_meta={})
    ad = load_file(str(tmp_path / "var_lora" / "adapter_model.safetensors"))
    names = [n for n, p in be.es_model.transformer.named_parameters() if p.requires_grad]
    assert any(".mat_qkv.lora_A" in n for n in names)
    assert torch.equal(torch.cat([ad[f"base_model.model.{n}"].reshape(-1) for n in names]), theta)
    cfg = json.loads((tmp_path / "var_lora" / "adapter_config.json").read_text())
    assert cfg["r"] == 4 and cfg["lora_alpha"] == 16
    with torch.no_grad():
        for p in params:
            p.zero_()
    be.load_lora(tmp_path / "var_lora")
    assert torch.equal(flatten_params(params), theta)
    th, meta = load_latest_checkpoint(tmp_path / "var_meta.pt")
    assert torch.equal(th, theta) and meta["backend"] == be.name
