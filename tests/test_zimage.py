"""Z-Image-Turbo host (BASELINE configs[3]) on CPU: the LoRA theta layout, the restated scheduler,
token geometry, RoPE tables, the backend's prompt sampling and the fp32 restatement itself (no GPU).
The architecture and scheduler are restatements of diffusers' (absent here): UNPINNED."""
import math

import numpy as np
import pytest
import torch

from hyperscalees_t2i_amd.backend import ZImageBackend, ZImageConfig, synthetic_zimage_prompt_data
from hyperscalees_t2i_amd.es import repeat_batches, sample_indices_unique
from hyperscalees_t2i_amd.model_shapes import zimage_turbo_lora_shapes
from hyperscalees_t2i_amd.sana import attach_lora
from hyperscalees_t2i_amd.zimage import (ZIMAGE_LORA_TARGETS, ZImageArch, ZImageTransformer2DModel, rope_tables,
                                         zimage_lora_shapes)
from hyperscalees_t2i_amd.zimage_pipeline import flow_sigmas

TINY = ZImageArch(dim=256, n_layers=2, n_refiner_layers=1, n_heads=2, ffn=512, cap_feat_dim=256, t_mid=256,
                  seq_multiple=16)


def test_theta_layout_matches_model_shapes():
    s = zimage_lora_shapes()
    assert s == zimage_turbo_lora_shapes()
    assert len(s) == 2 * (34 * 6 + 1) and sum(math.prod(x) for x in s) == 4_446_848
    assert s[:2] == [(2, 3840), (64, 2)]          # all_final_layer.*.linear first (registration order)
    assert s[2:4] == [(2, 3840), (3840, 2)]       # noise_refiner.0.attention.to_q


def test_lora_targets_by_name():
    with torch.device("meta"):
        m = ZImageTransformer2DModel(TINY)
        n = attach_lora(m, 2, 8.0, ZIMAGE_LORA_TARGETS)
    names = [k for k, p in m.named_parameters() if p.requires_grad]
    assert n == 4 * 6 + 1 and len(names) == 2 * n
    assert names[0] == "all_final_layer.2-1.linear.lora_A.weight"
    assert not any("to_out" in k or "adaLN" in k or "embedder" in k for k in names)


def test_flow_sigmas():
    """ZImagePipeline sets scheduler.sigma_min = 0.0 before set_timesteps: shift(linspace(1, 0, steps))
    then a final 0, so the last Euler step has dt = 0.  sigma_min=None: the scheduler's own default."""
    s = flow_sigmas(7)
    sh = lambda v: 3 * v / (1 + 2 * v)  # noqa: E731
    assert len(s) == 8 and s[0] == 1.0 and s[-2] == 0.0 and s[-1] == 0.0
    assert all(a > b for a, b in zip(s[:-1], s[1:-1]))
    assert s[1] == pytest.approx(sh(1.0 - 1.0 / 6))
    assert s[3] == pytest.approx(sh(0.5))
    d = flow_sigmas(7, sigma_min=None)
    smin = sh(1e-3)
    assert d[-2] == pytest.approx(sh(smin)) and d[-1] == 0.0
    assert d[1] == pytest.approx(sh(1.0 - (1.0 - smin) / 6))


def test_patchify_roundtrip_and_positions():
    with torch.device("meta"):
        m = ZImageTransformer2DModel(TINY)
    m.config = TINY
    lat = torch.randn(3, 16, 8, 12)
    tok = ZImageTransformer2DModel.patchify(m, lat)
    assert tok.shape == (3, 24, 64)
    assert torch.equal(tok[1, 11], lat[1, :, 2:4, 10:12].permute(1, 2, 0).reshape(-1))   # patch (1, 5)
    assert torch.equal(ZImageTransformer2DModel.unpatchify(m, tok, 8, 12), lat)
    img, cap = ZImageTransformer2DModel.positions(m, torch.tensor([32, 64]), 64, 4, 6)
    assert img.shape == (2, 24, 3) and cap.shape == (64, 3)
    assert img[1, 7].tolist() == [65, 1, 1] and img[0, 0].tolist() == [33, 0, 0]
    assert cap[0].tolist() == [1, 0, 0] and cap[63].tolist() == [64, 0, 0]


def test_rope_tables_are_rotations():
    pos = torch.tensor([[3, 5, 7], [0, 0, 0]])
    c, s = rope_tables(TINY, pos)
    assert c.shape == (2, 64)
    assert torch.allclose(c * c + s * s, torch.ones_like(c), atol=1e-6)
    assert torch.equal(c[1], torch.ones(64)) and torch.equal(s[1], torch.zeros(64))
    # axis 0 uses the first 16 pairs with theta^(-2i/32)
    assert c[0, 1].item() == pytest.approx(math.cos(3 * 256 ** (-2 / 32)), rel=1e-6)


def test_backend_sampling_info_matches_reference_functions():
    be = ZImageBackend("cpu", ZImageConfig(synthetic_weights=True, synthetic_prompts=6))
    be.prompt_data = synthetic_zimage_prompt_data(6)
    be.base_prompt_embeds = be.prompt_data["prompt_embeds"]
    be.prompts_list = be.prompt_data["prompts"]
    info = be.step_sampling_info(7)
    uid = sample_indices_unique(seed=7, total=6, k=4)
    assert info["unique_ids"] == uid and info["flat_ids"] == repeat_batches(uid, repeats=4)
    assert info["m"] == 4 and info["total_imgs_per_indiv"] == 16
    assert all(isinstance(e, torch.Tensor) and e.shape[1] == 2560 and 16 <= e.shape[0] <= 100
               for e in be.base_prompt_embeds)


def test_backend_requires_explicit_synthetic_flag():
    be = ZImageBackend("cpu", ZImageConfig())
    with pytest.raises(FileNotFoundError, match="synthetic_weights=True"):
        be.init_and_attach_lora()


def test_fp32_restatement_runs_on_cpu():
    """The oracle's fp32 transformer on a tiny model (CPU): shape, finiteness, and that a member's LoRA
    factors change the velocity."""
    from oracle import zimage_fp32 as Z
    torch.manual_seed(0)
    m = ZImageTransformer2DModel(TINY)
    m.init_weights(0)
    attach_lora(m, 2, 8.0, ZIMAGE_LORA_TARGETS)
    D = sum(p.numel() for p in m.parameters() if p.requires_grad)
    lat = torch.randn(2, 16, 8, 8)
    cap = torch.randn(2, 64, 256)
    lens = torch.tensor([32, 64])
    idx = torch.tensor([1, 0])
    t = torch.tensor([0.3])
    v0 = Z.transformer_fp32(m, lat, t, cap, lens, idx, torch.zeros(D))
    v1 = Z.transformer_fp32(m, lat, t, cap, lens, idx, torch.randn(D) * 0.1)
    assert v0.shape == lat.shape and torch.isfinite(v0).all()
    assert (v0 - v1).abs().max() > 0


def test_unpadded_image_token_count_raises():
    """diffusers pads the image tokens to a multiple of seq_multiple with x_pad_token; the build does not
    restate that padding and refuses such sizes instead of running a different sequence."""
    with torch.device("meta"):
        m = ZImageTransformer2DModel(TINY)
        lat = torch.empty(1, 16, 10, 10)          # 5 x 5 = 25 image tokens, seq_multiple 16
        with pytest.raises(NotImplementedError, match="seq_multiple"):
            m(lat, torch.zeros(1), torch.empty(1, 16, 256), torch.zeros(1, dtype=torch.long),
              torch.zeros(1, dtype=torch.long))
