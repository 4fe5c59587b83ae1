"""Real-checkpoint drop-in for the Z-Image-Turbo and Infinity hosts (BASELINE configs[3] / [4]).

* Z-Image (models/zImageTurbo.py:97-125, ZImagePipeline.from_pretrained): a local diffusers directory —
  transformer/ (ZImageTransformer2DModel) + vae/ (the FLUX AutoencoderKL) — mapped onto zimage.py /
  flux_vae.py by hyperscalees_t2i_amd/checkpoints.py.
* Infinity (models/Infinity.py:183-235, load_state_dict / load_sharded_checkpoint): the Infinity repo's
  state dict (.pth via torch.load(weights_only=True), or a sharded directory with its index) and the
  BSQ-VAE .pth, mapped onto infinity.py.
Neither diffusers nor the Infinity repo nor any weights exist offline, so the key names follow the
published modules and are UNPINNED against real files.  Pinned here: save -> load round trips bit for
bit, the published tensor shapes of the converted entries, strictness (missing / unexpected /
mis-shaped keys raise), configurations the build does not implement raise, and a model path that is not
a local checkpoint raises FileNotFoundError unless synthetic weights are asked for explicitly.  The GPU
tests check that a loaded model drives the population member-eval bit for bit like the original, and
the Z-Image VAE-decoder LoRA (es_backend.py:598-608)."""
import pytest
import torch

from hyperscalees_t2i_amd import checkpoints as C
from hyperscalees_t2i_amd.flux_vae import FluxVAEDecoder
from hyperscalees_t2i_amd.zimage import ZImageArch, ZImageTransformer2DModel

ZTINY = ZImageArch(dim=384, n_layers=2, n_refiner_layers=1, n_heads=3, ffn=1024, cap_feat_dim=256,
                   t_mid=1024, seq_multiple=16)
ZVAE_W = (32, 32, 64, 64)


def _frozen(m):
    return {n: p for n, p in m.named_parameters() if not p.requires_grad}


@pytest.fixture(scope="module")
def zsaved(tmp_path_factory):
    d = tmp_path_factory.mktemp("zimage_local")
    tr = ZImageTransformer2DModel(ZTINY)
    tr.init_weights(5)
    vae = FluxVAEDecoder(widths=ZVAE_W)
    vae.init_weights(6)
    C.save_zimage_diffusers(tr, vae, d)
    return d, tr, vae


def test_zimage_diffusers_layout(zsaved):
    from safetensors.torch import load_file
    d, _, _ = zsaved
    st = load_file(str(d / "transformer" / C.WEIGHTS_NAME))
    D = ZTINY.dim
    want = {"all_x_embedder.2-1.weight": (D, 64), "all_final_layer.2-1.linear.weight": (64, D),
            "layers.1.attention.to_out.0.weight": (D, D), "layers.0.feed_forward.w2.weight": (D, ZTINY.ffn),
            "noise_refiner.0.adaLN_modulation.0.weight": (4 * D, 256), "context_refiner.0.attention.norm_k.weight": (128,),
            "t_embedder.mlp.0.weight": (1024, 256), "cap_embedder.1.weight": (D, 256), "x_pad_token": (1, D)}
    for k, sh in want.items():
        assert tuple(st[k].shape) == sh, k
    sv = load_file(str(d / "vae" / C.WEIGHTS_NAME))
    for k, sh in {"decoder.conv_in.weight": (64, 16, 3, 3), "decoder.mid_block.attentions.0.to_q.weight": (64, 64),
                  "decoder.mid_block.attentions.0.to_out.0.bias": (64,), "decoder.mid_block.resnets.1.conv2.weight":
                  (64, 64, 3, 3), "decoder.up_blocks.0.upsamplers.0.conv.weight": (64, 64, 3, 3),
                  "decoder.up_blocks.2.resnets.0.conv_shortcut.weight": (32, 64, 1, 1),
                  "decoder.conv_norm_out.weight": (32,), "decoder.conv_out.weight": (3, 32, 3, 3)}.items():
        assert tuple(sv[k].shape) == sh, k
    assert not any(k.startswith("decoder.up_blocks.3.upsamplers") for k in sv)   # the last up block has none
    cfg = C.read_config(d / "vae")
    assert cfg["block_out_channels"] == list(ZVAE_W) and cfg["layers_per_block"] == 2


def test_zimage_roundtrip_bitexact(zsaved):
    d, tr, vae = zsaved
    a2 = C.zimage_arch_from_config(C.read_config(d / "transformer"))
    assert (a2.dim, a2.n_layers, a2.n_heads, a2.ffn, a2.cap_feat_dim) == (ZTINY.dim, 2, 3, ZTINY.ffn, 256)
    tr2 = ZImageTransformer2DModel(a2)
    C.load_zimage_transformer(tr2, d / "transformer")
    a, b = _frozen(tr), _frozen(tr2)
    assert list(a) == list(b) and all(torch.equal(a[n], b[n]) for n in a)
    vae2 = FluxVAEDecoder(**C.flux_vae_kwargs(C.read_config(d / "vae")))
    C.load_flux_vae_decoder(vae2, d / "vae")
    a, b = _frozen(vae), _frozen(vae2)
    assert list(a) == list(b) and all(torch.equal(a[n], b[n]) for n in a)
    assert (vae2.scaling_factor, vae2.shift_factor) == (vae.scaling_factor, vae.shift_factor)


def test_zimage_loader_is_strict(zsaved, tmp_path):
    from safetensors.torch import load_file, save_file
    d, _, _ = zsaved
    st = load_file(str(d / "transformer" / C.WEIGHTS_NAME))
    for mutate, match in ((lambda s: s.pop("layers.1.feed_forward.w3.weight"), "lacks"),
                          (lambda s: s.__setitem__("layers.0.extra.weight", torch.zeros(1)), "not used"),
                          (lambda s: s.__setitem__("cap_pad_token", torch.zeros(1, 7)), "gives")):
        s = dict(st)
        mutate(s)
        (tmp_path / "t").mkdir(exist_ok=True)
        save_file(s, str(tmp_path / "t" / C.WEIGHTS_NAME))
        with pytest.raises(ValueError, match=match):
            C.load_zimage_transformer(ZImageTransformer2DModel(ZTINY), tmp_path / "t")
    sv = load_file(str(d / "vae" / C.WEIGHTS_NAME))
    sv["encoder.conv_in.weight"] = torch.zeros(2)               # the encoder half is ignored (decode only)
    (tmp_path / "v").mkdir()
    save_file(sv, str(tmp_path / "v" / C.WEIGHTS_NAME))
    C.load_flux_vae_decoder(FluxVAEDecoder(widths=ZVAE_W), tmp_path / "v")
    sv["post_quant_conv.weight"] = torch.zeros(2)               # a decoder-side tensor the build lacks: refused
    save_file(sv, str(tmp_path / "v" / C.WEIGHTS_NAME))
    with pytest.raises(ValueError, match="not used"):
        C.load_flux_vae_decoder(FluxVAEDecoder(widths=ZVAE_W), tmp_path / "v")


def test_zimage_unsupported_configs_refused(zsaved):
    d, _, _ = zsaved
    cfg = C.read_config(d / "transformer")
    for k, v in (("all_patch_size", [2, 4]), ("all_f_patch_size", [2]), ("n_kv_heads", 1), ("qk_norm", False)):
        with pytest.raises(NotImplementedError):
            C.zimage_arch_from_config(dict(cfg, **{k: v}))
    vcfg = C.read_config(d / "vae")
    for k, v in (("use_post_quant_conv", True), ("norm_num_groups", 16), ("mid_block_add_attention", False)):
        with pytest.raises(NotImplementedError):
            C.flux_vae_kwargs(dict(vcfg, **{k: v}))


def test_zimage_backend_loads_local_directory(zsaved, tmp_path):
    from hyperscalees_t2i_amd.backend import ZImageBackend, ZImageConfig
    d, tr, vae = zsaved
    for name in ("Tongyi-MAI/Z-Image-Turbo", str(tmp_path / "missing"), str(tmp_path)):
        with pytest.raises(FileNotFoundError):
            ZImageBackend("cpu", ZImageConfig(model_name=name, arch=ZTINY, vae_widths=ZVAE_W)).init_and_attach_lora()
    be = ZImageBackend("cpu", ZImageConfig(model_name=str(d), synthetic_prompts=2, synthetic_prompt_lens=(4, 9)))
    be.init_and_attach_lora()
    m = be.es_model
    assert m.weights_source == str(d) and m.arch.dim == ZTINY.dim
    assert all(torch.equal(x, y) for x, y in zip(_frozen(tr).values(), _frozen(m.transformer).values()))
    assert all(torch.equal(x, y) for x, y in zip(_frozen(vae).values(), _frozen(m.vae).values()))


def test_zimage_vae_decoder_lora_theta_layout():
    """use_vae_decoder_lora (es_backend.py:598-618): theta = the transformer's LoRA params, then the decoder's
    mid-block to_q / to_k / to_v / to_out.0 LoRA params (r 2 by default), in PEFT's parameter order; the
    decoder modules' theta offsets start after the transformer's."""
    from hyperscalees_t2i_amd.backend import ZImageBackend, ZImageConfig
    from hyperscalees_t2i_amd.lora import lora_modules
    cfg = dict(synthetic_weights=True, arch=ZTINY, vae_widths=ZVAE_W, synthetic_prompts=2, synthetic_prompt_lens=(4, 9))
    plain = ZImageBackend("cpu", ZImageConfig(**cfg))
    plain.init_and_attach_lora()
    be = ZImageBackend("cpu", ZImageConfig(use_vae_decoder_lora=True, **cfg))
    be.init_and_attach_lora()
    p0, s0 = plain.collect_lora_params()
    p1, s1 = be.collect_lora_params()
    Cv = ZVAE_W[-1]
    assert s1[:len(s0)] == s0 and s1[len(s0):] == [(2, Cv), (Cv, 2)] * 4
    d_tr = sum(p.numel() for p in p0)
    mods = lora_modules(be.es_model.vae)
    assert [m.theta_off_A for m in mods] == [d_tr + i * 4 * Cv for i in range(4)]
    assert [m.theta_off_B for m in mods] == [d_tr + i * 4 * Cv + 2 * Cv for i in range(4)]


def test_zimage_vae_decoder_adapter_keys_are_peft_decoder_names(tmp_path):
    """save_lora's vae_decoder/ adapter carries the keys PEFT's save_pretrained writes for a LoRA'd
    pipe.vae.decoder (es_backend.py:598-619): base_model.model.mid_block.attentions.0.<target>.lora_A|B.weight
    — diffusers' Decoder names, not flux_vae.py's mid.1 — and load_lora reads exactly that key set back."""
    from safetensors.torch import load_file
    from hyperscalees_t2i_amd.backend import ZImageBackend, ZImageConfig
    cfg = dict(synthetic_weights=True, arch=ZTINY, vae_widths=ZVAE_W, synthetic_prompts=2, synthetic_prompt_lens=(4, 9),
               use_vae_decoder_lora=True)
    be = ZImageBackend("cpu", ZImageConfig(**cfg))
    be.init_and_attach_lora()
    be.save_lora(tmp_path)
    keys = set(load_file(str(tmp_path / "vae_decoder" / "adapter_model.safetensors")))
    want = {f"base_model.model.mid_block.attentions.0.{t}.lora_{ab}.weight"
            for t in ("to_q", "to_k", "to_v", "to_out.0") for ab in ("A", "B")}
    assert keys == want
    tr_keys = set(load_file(str(tmp_path / "transformer" / "adapter_model.safetensors")))
    assert all(k.startswith("base_model.model.") and ".lora_" in k for k in tr_keys)
    be2 = ZImageBackend("cpu", ZImageConfig(**cfg))
    be2.init_and_attach_lora()
    for m in lora_modules_of(be2.es_model.vae):
        torch.nn.init.zeros_(m.lora_A.weight)
    be2.load_lora(tmp_path)
    for a, b in zip(lora_modules_of(be.es_model.vae), lora_modules_of(be2.es_model.vae)):
        assert torch.equal(a.lora_A.weight, b.lora_A.weight) and torch.equal(a.lora_B.weight, b.lora_B.weight)
    import safetensors.torch as st                               # a flux_vae.py-named file is refused
    t = load_file(str(tmp_path / "vae_decoder" / "adapter_model.safetensors"))
    st.save_file({k.replace("mid_block.attentions.0", "mid.1"): v for k, v in t.items()},
                 str(tmp_path / "vae_decoder" / "adapter_model.safetensors"))
    with pytest.raises(ValueError, match="adapter keys differ"):
        be2.load_lora(tmp_path)


def lora_modules_of(m):
    from hyperscalees_t2i_amd.lora import lora_modules
    return lora_modules(m)


# ---------------------------------------------------------------------------------------------- Infinity
from hyperscalees_t2i_amd.infinity import InfinityArch, InfinityTransformer, infinity_vae  # noqa: E402

ITINY = InfinityArch(depth=2, embed_dim=256, num_heads=2, block_chunks=2, text_channels=256, codebook_dim=4,
                     spatial_patchify=1, vae_widths=(32, 32, 64, 64))


@pytest.fixture(scope="module")
def isaved(tmp_path_factory):
    d = tmp_path_factory.mktemp("infinity_local")
    tr = InfinityTransformer(ITINY)
    tr.init_weights(3)
    with torch.no_grad():   # nonzero biases everywhere, so the q | 0 | v folding is exercised
        for blk in tr.blocks():
            blk.sa.mat_qkv.bias.normal_()
            blk.sa.mat_qkv.bias[256:512].zero_()
            blk.ca.mat_kv.bias.normal_()
            blk.ca.mat_kv.bias[:256].zero_()
        tr.text_proj_for_sos.mat_kv.bias.normal_()
        tr.text_proj_for_sos.mat_kv.bias[:256].zero_()
    vae = infinity_vae(ITINY)
    vae.init_weights(4)
    C.save_infinity_checkpoint(tr, vae, d / "infinity.pth", d / "vae.pth")
    C.save_infinity_checkpoint(tr, vae, d / "shards", d / "vae2.pth", shards=3)
    return d, tr, vae


def test_infinity_repo_layout(isaved):
    d, _, _ = isaved
    st = torch.load(str(d / "infinity.pth"), weights_only=True)
    Cd = ITINY.C
    for k, sh in {"block_chunks.1.module.0.sa.mat_qkv.weight": (3 * Cd, Cd), "block_chunks.0.module.0.sa.q_bias": (Cd,),
                  "block_chunks.0.module.0.sa.v_bias": (Cd,), "block_chunks.0.module.0.sa.zero_k_bias": (Cd,),
                  "block_chunks.0.module.0.ca.v_bias": (Cd,), "block_chunks.0.module.0.ffn.fc1.weight": (1024, Cd),
                  "block_chunks.0.module.0.ada_gss": (1, 1, 6, Cd), "lvl_embed.weight": (15, Cd),
                  "text_proj_for_sos.ca.mat_q": (1, 1, Cd), "text_proj_for_sos.ca.mat_kv.weight": (2 * Cd, 256),
                  "shared_ada_lin.1.weight": (6 * Cd, Cd), "head_nm.ada_lin.1.weight": (2 * Cd, Cd)}.items():
        assert tuple(st[k].shape) == sh, k
    assert "block_chunks.0.module.0.sa.mat_qkv.bias" not in st and "block_chunks.0.module.0.ca.mat_kv.bias" not in st
    sv = torch.load(str(d / "vae.pth"), weights_only=True)
    for k, sh in {"decoder.mid.attn_1.q.weight": (64, 64, 1, 1), "decoder.mid.attn_1.norm.weight": (64,),
                  "decoder.up.0.block.0.conv1.weight": (32, 32, 3, 3), "decoder.up.3.upsample.conv.weight": (64, 64, 3, 3),
                  "decoder.up.1.block.0.nin_shortcut.weight": (32, 64, 1, 1), "decoder.norm_out.bias": (32,)}.items():
        assert tuple(sv[k].shape) == sh, k
    assert not any(k.startswith("decoder.up.0.upsample") for k in sv)


@pytest.mark.parametrize("kind", ["torch", "torch_shard"])
def test_infinity_roundtrip_bitexact(isaved, kind):
    d, tr, vae = isaved
    tr2 = InfinityTransformer(ITINY)
    C.load_infinity_transformer(tr2, d / ("infinity.pth" if kind == "torch" else "shards"), kind)
    a, b = _frozen(tr), _frozen(tr2)
    assert list(a) == list(b) and all(torch.equal(a[n], b[n]) for n in a)
    vae2 = infinity_vae(ITINY)
    C.load_bsq_vae_decoder(vae2, d / "vae.pth")
    assert all(torch.equal(x, y) for x, y in zip(_frozen(vae).values(), _frozen(vae2).values()))


def test_infinity_loader_is_strict(isaved, tmp_path):
    d, _, _ = isaved
    st = torch.load(str(d / "infinity.pth"), weights_only=True)
    H = ITINY.num_heads
    cases = ((lambda s: s.pop("block_chunks.1.module.0.ffn.fc2.bias"), ValueError, "lacks"),
             (lambda s: s.__setitem__("block_chunks.0.module.0.extra", torch.zeros(1)), ValueError, "not used"),
             (lambda s: s.__setitem__("head.weight", torch.zeros(3, 256)), ValueError, "gives"),
             (lambda s: s.__setitem__("block_chunks.0.module.0.sa.zero_k_bias", torch.ones(256)), ValueError, "not zero"))
    for mutate, exc, match in cases:
        s = dict(st)
        mutate(s)
        torch.save(s, str(tmp_path / "m.pth"))
        with pytest.raises(exc, match=match):
            C.load_infinity_transformer(InfinityTransformer(ITINY), tmp_path / "m.pth", "torch")
    # the flash-attention form of scale_mul_1H11 ([1, 1, H, 1]) and wrapped / buffer-carrying dicts load
    s = dict(st)
    for k in [k for k in s if k.endswith("scale_mul_1H11")]:
        s[k] = s[k].reshape(1, 1, H, 1)
    s["lvl_1L"] = torch.zeros(1, 10)
    torch.save({"state_dict": s}, str(tmp_path / "w.pth"))
    C.load_infinity_transformer(InfinityTransformer(ITINY), tmp_path / "w.pth", "torch")
    with pytest.raises(FileNotFoundError):
        C.load_infinity_transformer(InfinityTransformer(ITINY), tmp_path / "missing.pth", "torch")
    with pytest.raises(FileNotFoundError):
        C.load_infinity_transformer(InfinityTransformer(ITINY), tmp_path, "torch_shard")
    with pytest.raises(ValueError):
        C.read_infinity_state(tmp_path / "w.pth", "safetensors")


def test_infinity_backend_loads_local_files(isaved, tmp_path):
    from hyperscalees_t2i_amd.backend import InfinityBackend, InfinityConfig
    d, tr, vae = isaved
    bad = InfinityBackend("cpu", InfinityConfig(arch=ITINY, model_path=str(tmp_path / "none.pth"), checkpoint_type="torch",
                                                vae_path=str(d / "vae.pth"), pn="0.06M", synthetic_prompt_lens=(5, 9)))
    with pytest.raises(FileNotFoundError):
        bad.init_and_attach_lora()
    be = InfinityBackend("cpu", InfinityConfig(arch=ITINY, model_path=str(d / "shards"), checkpoint_type="torch_shard",
                                               vae_path=str(d / "vae.pth"), pn="0.06M", synthetic_prompt_lens=(5, 9)))
    be.init_and_attach_lora()
    m = be.es_model
    assert m.weights_source == str(d / "shards")
    assert all(torch.equal(x, y) for x, y in zip(_frozen(tr).values(), _frozen(m.transformer).values()))
    assert all(torch.equal(x, y) for x, y in zip(_frozen(vae).values(), _frozen(m.vae).values()))
