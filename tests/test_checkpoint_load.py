"""Real-checkpoint drop-in (models/SanaSprint.py:35-49, rewards.py:32-60, es_backend.py:172-200):
local diffusers-format Sana-Sprint directories and local transformers CLIP / PickScore directories.

* The Sana transformer / DC-AE decoder key mapping (hyperscalees_t2i_amd/checkpoints.py) follows
  diffusers' published module names; diffusers is not importable here and no real checkpoint exists,
  so the names are UNPINNED against real files.  What is pinned: a save -> load round trip through
  the diffusers layout reproduces every frozen parameter bit for bit (and the kernel-layout copies the
  decoder derives from them), the diffusers shapes of the converted tensors (1x1 / depthwise /
  grouped convs, fused q|k|v), strictness (missing / unexpected / mis-shaped keys raise), and the
  no-silent-substitution rule (a model_name that is not a local directory raises FileNotFoundError
  unless synthetic weights are asked for explicitly).
* The reward towers load through transformers itself (CLIPModel.save_pretrained / from_pretrained,
  the CLIP BPE tokenizer, the CLIPImageProcessor config) — that path is real transformers code, so
  the text features are compared with CLIPModel.get_text_features on the same weights.
"""
import json

import pytest
import torch

from hyperscalees_t2i_amd import checkpoints as C
from hyperscalees_t2i_amd.dcae import DCAEDecoder
from hyperscalees_t2i_amd.sana import SanaArch, SanaTransformer2DModel

TINY = SanaArch(num_attention_heads=4, attention_head_dim=32, num_layers=2, num_cross_attention_heads=2,
                cross_attention_head_dim=64, caption_channels=128)   # K % 64 == 0 for the GEMM
VAE_W, VAE_L = (16, 32, 32, 64, 64, 64), (1, 1, 1, 1, 1, 2)


def _make_models(seed=3):
    tr = SanaTransformer2DModel(TINY)
    tr.init_weights(seed)
    vae = DCAEDecoder(32, widths=VAE_W, layers=VAE_L)
    vae.init_weights(seed + 1)
    return tr, vae


@pytest.fixture(scope="module")
def saved(tmp_path_factory):
    d = tmp_path_factory.mktemp("sana_local")
    tr, vae = _make_models()
    C.save_sana_diffusers(tr, vae, d)
    return d, tr, vae


def _frozen(m):
    return {n: p for n, p in m.named_parameters() if not p.requires_grad}


def test_diffusers_layout_keys_and_shapes(saved):
    from safetensors.torch import load_file
    d, tr, vae = saved
    st = load_file(str(d / "transformer" / C.WEIGHTS_NAME))
    D, h2 = TINY.inner_dim, 2 * int(TINY.mlp_ratio * TINY.inner_dim)
    want = {"patch_embed.proj.weight": (D, 32, 1, 1), "patch_embed.proj.bias": (D,),
            "time_embed.timestep_embedder.linear_1.weight": (D, 256), "time_embed.linear.weight": (6 * D, D),
            "caption_projection.linear_1.weight": (D, 128), "caption_norm.weight": (D,),
            "transformer_blocks.0.attn1.to_q.weight": (D, D), "transformer_blocks.0.attn1.norm_q.weight": (D,),
            "transformer_blocks.0.attn1.to_out.0.bias": (D,), "transformer_blocks.1.attn2.to_k.bias": (D,),
            "transformer_blocks.1.ff.conv_inverted.weight": (h2, D, 1, 1),
            "transformer_blocks.1.ff.conv_depth.weight": (h2, 1, 3, 3),
            "transformer_blocks.1.ff.conv_point.weight": (D, h2 // 2, 1, 1),
            "transformer_blocks.0.scale_shift_table": (6, D), "scale_shift_table": (2, D), "proj_out.weight": (32, D)}
    for k, shp in want.items():
        assert tuple(st[k].shape) == shp, k
    assert "transformer_blocks.0.attn1.to_q.bias" not in st        # attention_bias=False for attn1 q/k/v
    assert not any("lora" in k for k in st)                          # the base checkpoint holds no adapter
    sv = load_file(str(d / "vae" / C.WEIGHTS_NAME))
    assert all(k.startswith("decoder.") for k in sv)
    # up_blocks are indexed highest resolution first (diffusers), stage 5 (64 ch, 2 layers) has no up block
    assert tuple(sv["decoder.up_blocks.5.1.attn.to_q.weight"].shape) == (64, 64)
    assert tuple(sv["decoder.up_blocks.5.0.attn.to_qkv_multiscale.0.proj_in.weight"].shape) == (192, 1, 5, 5)
    assert tuple(sv["decoder.up_blocks.5.0.attn.to_qkv_multiscale.0.proj_out.weight"].shape) == (192, 32, 1, 1)
    assert tuple(sv["decoder.up_blocks.4.0.conv.weight"].shape) == (64, 64, 3, 3)      # DCUpBlock2d 64 -> 64
    assert tuple(sv["decoder.up_blocks.0.1.conv1.weight"].shape) == (16, 16, 3, 3)     # ResBlock after the up block
    assert tuple(sv["decoder.up_blocks.3.1.conv_out.conv_depth.weight"].shape) == (512, 1, 3, 3)   # 2 x 4 x 64
    assert {"decoder.conv_in.weight", "decoder.norm_out.bias", "decoder.conv_out.weight"} <= set(sv)
    cfg = json.loads((d / "vae" / "config.json").read_text())
    assert cfg["decoder_block_types"][:3] == ["ResBlock"] * 3 and cfg["upsample_block_type"] == "interpolate"


def test_roundtrip_bitexact_and_kernel_layouts(saved):
    d, tr, vae = saved
    tr2 = SanaTransformer2DModel(C.sana_arch_from_config(C.read_config(d / "transformer")))
    assert tr2.config == TINY
    C.load_sana_transformer(tr2, d / "transformer")
    a, b = _frozen(tr), _frozen(tr2)
    assert list(a) == list(b) and all(torch.equal(a[n], b[n]) for n in a)
    vae2 = DCAEDecoder(**C.dcae_build_kwargs(C.read_config(d / "vae")))
    C.load_dcae_decoder(vae2, d / "vae")
    a, b = _frozen(vae), _frozen(vae2)
    assert list(a) == list(b) and all(torch.equal(a[n], b[n]) for n in a)
    assert vae2.scaling_factor == vae.scaling_factor
    from hyperscalees_t2i_amd.dcae import ResBlock, UpBlock
    for m1, m2 in zip(vae.modules(), vae2.modules()):
        if isinstance(m1, ResBlock) and m1.packed is not None:
            assert all(torch.equal(x, y) for x, y in zip(m1.packed, m2.packed))
        if isinstance(m1, UpBlock):
            assert torch.equal(m1.w4, m2.w4)


def test_loader_is_strict(saved, tmp_path):
    from safetensors.torch import load_file, save_file
    d, tr, vae = saved
    st = load_file(str(d / "transformer" / C.WEIGHTS_NAME))
    for mutate, match in ((lambda s: s.pop("transformer_blocks.1.ff.conv_point.weight"), "lacks"),
                          (lambda s: s.__setitem__("transformer_blocks.0.extra.weight", torch.zeros(1)), "not used"),
                          (lambda s: s.__setitem__("proj_out.weight", torch.zeros(31, TINY.inner_dim)), "gives")):
        s = dict(st)
        mutate(s)
        (tmp_path / "t").mkdir(exist_ok=True)
        save_file(s, str(tmp_path / "t" / C.WEIGHTS_NAME))
        with pytest.raises(ValueError, match=match):
            C.load_sana_transformer(SanaTransformer2DModel(TINY), tmp_path / "t")
    # the encoder half of an AutoencoderDC checkpoint is ignored (decode only)
    sv = load_file(str(d / "vae" / C.WEIGHTS_NAME))
    sv["encoder.conv_in.weight"] = torch.zeros(2)
    (tmp_path / "v").mkdir()
    save_file(sv, str(tmp_path / "v" / C.WEIGHTS_NAME))
    C.load_dcae_decoder(DCAEDecoder(32, widths=VAE_W, layers=VAE_L), tmp_path / "v")


def test_unsupported_configs_refused(saved):
    d, _, _ = saved
    cfg = C.read_config(d / "transformer")
    for k, v in (("qk_norm", None), ("patch_size", 2), ("guidance_embeds", False)):
        with pytest.raises(NotImplementedError):
            C.sana_arch_from_config(dict(cfg, **{k: v}))
    vcfg = C.read_config(d / "vae")
    for k, v in (("upsample_block_type", "pixel_shuffle"), ("decoder_norm_types", "batch_norm")):
        with pytest.raises(NotImplementedError):
            C.dcae_build_kwargs(dict(vcfg, **{k: v}))


def test_model_name_never_silently_synthetic(tmp_path):
    from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig
    for name in ("Efficient-Large-Model/Sana_Sprint_1.6B_1024px_diffusers", str(tmp_path / "missing"), str(tmp_path)):
        be = SanaBackend("cpu", SanaConfig(model_name=name, width_latent=4, height_latent=4, arch=TINY,
                                           vae_widths=VAE_W, vae_layers=VAE_L))
        with pytest.raises(FileNotFoundError):
            be.init_and_attach_lora()


def test_backend_loads_local_directory(saved):
    from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig
    d, tr, vae = saved
    be = SanaBackend("cpu", SanaConfig(model_name=str(d), width_latent=4, height_latent=4, synthetic_prompts=2))
    be.init_and_attach_lora()
    m = be.es_model
    assert m.weights_source == str(d) and m.transformer.config == TINY
    a, b = _frozen(tr), _frozen(m.transformer)
    assert all(torch.equal(a[n], b[n]) for n in a)
    assert all(torch.equal(x, y) for x, y in zip(_frozen(vae).values(), _frozen(m.vae).values()))
    params, shapes = be.collect_lora_params()
    syn = SanaBackend("cpu", SanaConfig(synthetic_weights=True, width_latent=4, height_latent=4, arch=TINY,
                                        vae_widths=VAE_W, vae_layers=VAE_L, synthetic_prompts=2))
    syn.init_and_attach_lora()
    assert shapes == syn.collect_lora_params()[1]     # the same theta layout as the synthetic build


# ---------------------------------------------------------------------------------------
# reward towers from local transformers directories
# ---------------------------------------------------------------------------------------

_WORDS = ["a", "photo", "of", "cat", "dog", "red", "high", "quality", "blurry", "image", "beautiful", "noisy"]


def _write_clip_dir(d, seed, hidden):
    from transformers import CLIPConfig, CLIPImageProcessorPil, CLIPModel, CLIPTokenizer
    d.mkdir(parents=True, exist_ok=True)
    vocab = {"<|startoftext|>": 0, "<|endoftext|>": 1}
    for w in _WORDS:
        vocab[w + "</w>"] = len(vocab)
    (d / "vocab.json").write_text(json.dumps(vocab))
    (d / "merges.txt").write_text("#version: 0.2\n")
    CLIPTokenizer(str(d / "vocab.json"), str(d / "merges.txt")).save_pretrained(str(d))
    CLIPImageProcessorPil().save_pretrained(str(d))
    torch.manual_seed(seed)
    cfg = CLIPConfig(text_config=dict(hidden_size=hidden, intermediate_size=2 * hidden, num_hidden_layers=2,
                                      num_attention_heads=2, max_position_embeddings=77, vocab_size=len(vocab),
                                      eos_token_id=1, bos_token_id=0, pad_token_id=1),
                     vision_config=dict(hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                                        num_attention_heads=2, image_size=224, patch_size=32),
                     projection_dim=24)
    m = CLIPModel(cfg)
    m.save_pretrained(str(d))
    return m


@pytest.fixture(scope="module")
def clip_dirs(tmp_path_factory):
    root = tmp_path_factory.mktemp("clip")
    mc = _write_clip_dir(root / "clip-vit-base-patch32", 11, 32)
    mp = _write_clip_dir(root / "PickScore_v1", 12, 48)
    return root / "clip-vit-base-patch32", root / "PickScore_v1", mc, mp


def test_reward_models_load_local_transformers_dirs(clip_dirs):
    from transformers import AutoTokenizer
    from hyperscalees_t2i_amd.rewards import AESTHETIC_TEXT, NEGATIVE_TEXT, PixelSpec, RewardModels
    cdir, pdir, mc, mp = clip_dirs
    rm = RewardModels.build("cpu", clip_path=str(cdir), pickscore_path=str(pdir))
    assert rm.clip_px == rm.pick_px == PixelSpec() and rm.source.startswith("local(")
    # frozen weights: the checkpoint's, cast to bf16 once
    assert torch.equal(rm.clip.text_model.embeddings.token_embedding.weight,
                       mc.text_model.embeddings.token_embedding.weight.to(torch.bfloat16))
    prompts = ["a photo of a red cat", "a dog"]
    ids_c, mask_c, ids_p, mask_p = rm.tokenize(prompts)
    tok = AutoTokenizer.from_pretrained(str(cdir), local_files_only=True)
    want = tok([AESTHETIC_TEXT, NEGATIVE_TEXT] + prompts, padding="max_length", truncation=True, max_length=77,
               return_tensors="pt")
    assert torch.equal(ids_c, want["input_ids"]) and torch.equal(mask_c, want["attention_mask"])
    assert ids_c.shape == (4, 77) and ids_p.shape == (2, 77)
    feats = rm._text_eager(ids_c, mask_c, ids_p, mask_p)
    # reference call (rewards.py:87-96 / 131-153): fp32 CLIPModel, processor padding=True (to the longest)
    for model, d, texts, keys in ((mc, cdir, [AESTHETIC_TEXT, NEGATIVE_TEXT] + prompts, None), (mp, pdir, prompts, "pick")):
        t = AutoTokenizer.from_pretrained(str(d), local_files_only=True)(texts, padding=True, truncation=True,
                                                                          max_length=77, return_tensors="pt")
        with torch.no_grad():
            ref = model.get_text_features(input_ids=t["input_ids"], attention_mask=t["attention_mask"])
        ref = getattr(ref, "pooler_output", ref)
        ref = ref / ref.norm(dim=-1, keepdim=True)
        got = feats["pick_prompt"] if keys else torch.cat([feats["clip_aes"][None], feats["clip_neg"][None],
                                                             feats["clip_prompt"]])
        assert torch.allclose(got, ref, atol=2e-6, rtol=0), float((got - ref).abs().max())


def test_reward_models_never_silently_synthetic(tmp_path, clip_dirs):
    from hyperscalees_t2i_amd.rewards import RewardModels
    cdir, _, _, _ = clip_dirs
    with pytest.raises(FileNotFoundError):
        RewardModels.build("cpu")
    with pytest.raises(FileNotFoundError):
        RewardModels.build("cpu", clip_path=str(cdir), pickscore_path=str(tmp_path / "missing"))
    with pytest.raises(ValueError):
        RewardModels.build("cpu", clip_path=str(cdir))


def test_processor_spec_refuses_other_pipelines(tmp_path):
    from hyperscalees_t2i_amd.rewards import pixel_spec_from_processor
    base = {"do_resize": True, "size": {"shortest_edge": 224}, "crop_size": {"height": 224, "width": 224},
            "do_center_crop": True, "resample": 3, "do_rescale": True, "rescale_factor": 1 / 255,
            "do_normalize": True, "image_mean": [0.5, 0.5, 0.5], "image_std": [0.5, 0.5, 0.5]}
    (tmp_path / "preprocessor_config.json").write_text(json.dumps(base))
    assert pixel_spec_from_processor(tmp_path).mean == (0.5, 0.5, 0.5)
    for k, v in (("resample", 2), ("crop_size", {"height": 256, "width": 224}), ("do_center_crop", False)):
        (tmp_path / "preprocessor_config.json").write_text(json.dumps(dict(base, **{k: v})))
        with pytest.raises(NotImplementedError):
            pixel_spec_from_processor(tmp_path)


@pytest.mark.gpu
def test_loaded_sana_generates_identically(dev, tmp_path):
    """A synthetic GPU model exported as a diffusers directory and loaded back drives the HIP
    member-eval bit for bit like the original (kernel-layout weights re-derived on load)."""
    from hyperscalees_t2i_amd.pipeline import SanaOneStep
    b = SanaOneStep("synthetic", device=str(dev), arch=TINY, vae_widths=VAE_W, vae_layers=VAE_L, weight_seed=3,
                    synthetic_weights=True)
    C.save_sana_diffusers(b.transformer, b.vae, tmp_path)
    a = SanaOneStep(str(tmp_path), device=str(dev))
    g = torch.Generator().manual_seed(0)
    pe = torch.randn(2, 300, 128, generator=g).to(dev, torch.float16)
    am = torch.ones(2, 300, dtype=torch.int64, device=dev)
    ia, _ = a.generate(pe, am, seed=4, guidance_scale=4.5, width_latent=4, height_latent=4, output_type="pt")
    ib, _ = b.generate(pe, am, seed=4, guidance_scale=4.5, width_latent=4, height_latent=4, output_type="pt")
    assert torch.equal(ia, ib)


@pytest.mark.gpu
def test_loaded_reward_towers_match_transformers(clip_dirs, dev):
    """Image side of the loaded towers on the HIP path vs CLIPModel.get_image_features (fp32) on the
    same checkpoint: bf16 GEMM operands, fp32 residual stream."""
    from hyperscalees_t2i_amd.rewards import RewardModels, clip_pixels
    cdir, pdir, mc, mp = clip_dirs
    rm = RewardModels.build(dev, clip_path=str(cdir), pickscore_path=str(pdir))
    g = torch.Generator().manual_seed(2)
    img = (torch.rand(3, 3, 256, 256, generator=g) * 2 - 1).to(dev, torch.bfloat16)
    px = clip_pixels(img)
    for model, tower in zip((mc, mp), rm.towers()):
        with torch.no_grad():
            ref = model.to(dev).get_image_features(pixel_values=px)
        ref = getattr(ref, "pooler_output", ref).float()
        got = tower(px)
        rel = float((got - ref).norm() / ref.norm())
        assert rel < 2e-2, rel
    feats = rm.prompt_features(["a photo of a cat"])
    s = rm.score(img, torch.zeros(3, dtype=torch.long, device=dev), feats)
    assert all(torch.isfinite(v).all() for v in s.values())
