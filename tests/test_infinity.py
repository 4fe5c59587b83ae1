"""Infinity host (BASELINE configs[4]) on CPU: the LoRA theta layout at Infinity-8B, the scale schedules,
the reference's cfg / tau list normalisation and compact packing, the bit <-> code geometry, the
sampler's micro-batch generator semantics, the backend's prompt sampling and errors, and the fp32
restatement itself (no GPU).  The architecture restates the Infinity repo (absent here): UNPINNED."""
import math

import pytest
import torch

from hyperscalees_t2i_amd.backend import InfinityBackend, InfinityConfig, synthetic_infinity_prompt_data
from hyperscalees_t2i_amd.es import repeat_batches, sample_indices_unique
from hyperscalees_t2i_amd.infinity import (INFINITY_8B, InfinityArch, InfinityTransformer, arch_for, bits_to_codes,
                                           codes_to_tokens, infinity_lora_shapes_from_model, rope2d_tables,
                                           sample_bits, scale_schedule)
from hyperscalees_t2i_amd.infinity_pipeline import InfinityES, as_schedule_list, images_to_uint8
from hyperscalees_t2i_amd.model_shapes import infinity_lora_shapes
from hyperscalees_t2i_amd.sana import attach_lora

TINY = InfinityArch(depth=2, embed_dim=256, num_heads=2, block_chunks=2, text_channels=256, codebook_dim=4,
                    spatial_patchify=1, vae_widths=(32, 32, 64, 64))


def test_theta_layout_8b():
    s = infinity_lora_shapes_from_model()
    assert s == infinity_lora_shapes("infinity_8b")
    assert len(s) == 80 and sum(math.prod(x) for x in s) == 1_433_600      # configs[4] D
    with torch.device("meta"):
        m = InfinityTransformer(TINY)
        n = attach_lora(m, 2, 8.0, ["fc1"])
    names = [k for k, p in m.named_parameters() if p.requires_grad]
    assert n == 2 and names[0] == "block_chunks.0.module.0.ffn.fc1.lora_A.weight"


def test_arch_variants_and_errors():
    a = arch_for("infinity_8b", 14, 1)
    assert (a.depth, a.C, a.num_heads, a.head_dim, a.ffn, a.d_tok) == (40, 3584, 28, 128, 14336, 56)
    assert arch_for("infinity_2b", 32, 0).d_tok == 32
    with pytest.raises(ValueError, match="vae_type"):
        arch_for("infinity_8b", 15, 1)
    with pytest.raises(ValueError, match="model_type"):
        arch_for("infinity_9b", 14, 1)


def test_scale_schedules():
    s = scale_schedule("0.25M")
    assert s[0] == (1, 1, 1) and s[-1] == (1, 32, 32) and sum(h * w for _, h, w in s) == 2521
    assert scale_schedule("1M")[-1] == (1, 64, 64)
    with pytest.raises(ValueError):
        scale_schedule("2M")


def test_schedule_lists_as_reference():
    assert as_schedule_list(3, "cfg", 3) == [3.0] * 3
    assert as_schedule_list([1, 2], "cfg", 4) == [1.0, 2.0, 2.0, 2.0]
    assert as_schedule_list([1, 2, 3, 4, 5], "cfg", 3) == [1.0, 2.0, 3.0]
    assert as_schedule_list(torch.tensor(2.5), "cfg", 2) == [2.5, 2.5]
    with pytest.raises(ValueError):
        as_schedule_list(None, "cfg", 2)
    with pytest.raises(TypeError):
        as_schedule_list("3", "cfg", 2)


def test_pack_compacts():
    kv = [torch.randn(3, 8), torch.randn(5, 8)]
    cat, lens, cu, Lt = InfinityES._pack_compacts_for_infinity(kv, [3, 5], "cpu", torch.float32)
    assert cat.shape == (8, 8) and lens == [3, 5] and cu.tolist() == [0, 3, 8] and cu.dtype == torch.int32 and Lt == 5
    with pytest.raises(ValueError):
        InfinityES._pack_compacts_for_infinity(kv, [3], "cpu", torch.float32)
    with pytest.raises(ValueError):
        InfinityES._pack_compacts_for_infinity([], [], "cpu", torch.float32)


def test_bits_codes_geometry():
    a = INFINITY_8B
    bits = torch.randint(0, 2, (2, 6 * 6, a.d_tok))
    z = bits_to_codes(bits, a, 6, 6)
    assert z.shape == (2, 14, 12, 12)
    # token (r, c), bit (ch, dy, dx) lands on VAE pixel (2r + dy, 2c + dx) of channel ch
    r, c, ch, dy, dx = 2, 5, 9, 1, 0
    want = (bits[1, r * 6 + c, ch * 4 + dy * 2 + dx].float() * 2 - 1) / math.sqrt(14)
    assert z[1, ch, 2 * r + dy, 2 * c + dx] == want
    assert torch.equal(codes_to_tokens(z, a), (bits.float() * 2 - 1) / math.sqrt(14))


def test_rope2d_tables():
    c, s = rope2d_tables(INFINITY_8B, 4, 4, 32, "cpu")
    assert c.shape == (16, 64) and torch.allclose(c * c + s * s, torch.ones_like(c), atol=1e-6)
    # token (1, 2) of a 4x4 grid sits at (8, 16) of the 32-grid: pair 1 of the row half, pair 32 + 1 of the column
    f1 = 10000.0 ** (-2.0 / 64)
    assert c[6, 1].item() == pytest.approx(math.cos(8 * f1), rel=1e-6)
    assert c[6, 33].item() == pytest.approx(math.cos(16 * f1), rel=1e-6)


def test_sample_bits_top_p_and_chunk_reseeding():
    lg = torch.tensor([[[0.0, 5.0], [5.0, 0.0], [0.0, 0.1]]])          # p_min 0.0067 (removed), 0.0067, 0.475
    outs = set()
    for s in range(20):
        b = sample_bits(lg.clone(), torch.Generator().manual_seed(s), 900, 0.97)
        assert b[0, 0] == 1 and b[0, 1] == 0
        outs.add(int(b[0, 2]))
    assert outs == {0, 1}
    # the reference's micro-batched calls each restart the generator at `seed`: chunk c's draws are the
    # draws a fresh generator makes for that chunk alone
    lg = torch.randn(4, 12, 2)
    g = torch.Generator().manual_seed(7)
    st = g.get_state()
    got = []
    for c0 in (0, 2):
        g.set_state(st)
        got.append(sample_bits(lg[c0:c0 + 2].clone(), g, 900, 0.97))
    for c0, b in zip((0, 2), got):
        assert torch.equal(b, sample_bits(lg[c0:c0 + 2].clone(), torch.Generator().manual_seed(7), 900, 0.97))


@pytest.mark.parametrize("B,mb", [(5, 2), (4, 2), (7, 3), (3, 4)])
def test_chunked_sampler_matches_independent_chunk_calls(B, mb):
    """ChunkedBitSampler over several scales == one fresh generator per (member, chunk) seeded with g_seed
    that sees only its own chunk's logits, scale after scale (the reference's separate chunk calls),
    including a smaller last chunk whose draws advance its generator differently."""
    from hyperscalees_t2i_amd.infinity import ChunkedBitSampler
    n, seed = 2, 11
    g = torch.Generator().manual_seed(123)
    scales = [torch.randn(n, B, ld, 2, generator=g) for ld in (4, 9, 30)]
    sampler = ChunkedBitSampler(torch.Generator().manual_seed(seed), B, mb)
    got = [sampler.sample(lg.clone(), 900, 0.97) for lg in scales]
    for k in range(n):
        for c0 in range(0, B, mb):
            ref = torch.Generator().manual_seed(seed)
            for lg, b in zip(scales, got):
                want = sample_bits(lg[k, c0:c0 + mb].clone(), ref, 900, 0.97)
                assert torch.equal(b[k, c0:c0 + mb], want), (k, c0)


def test_images_to_uint8_truncates():
    x = torch.tensor([-1.0, 0.0, 0.999, 1.0]).view(1, 1, 1, 4).expand(1, 3, 1, 4)
    u = images_to_uint8(x)
    assert u[0, 0, 0].tolist() == [0.0, 127.0, 255.0, 255.0]


def test_backend_sampling_info_and_errors():
    be = InfinityBackend("cpu", InfinityConfig(synthetic_weights=True, synthetic_prompts=6))
    be._load_or_encode_prompts()
    info = be.step_sampling_info(3)
    uid = sample_indices_unique(seed=3, total=6, k=4)
    assert info["unique_ids"] == uid and info["flat_ids"] == repeat_batches(uid, repeats=4)
    assert info["m"] == 4 and info["total_imgs_per_indiv"] == 16
    assert all(kv.shape == (L, 2048) for kv, L in zip(be.kv_compact_list, be.lens_list))
    with pytest.raises(FileNotFoundError, match="synthetic_weights=True"):
        InfinityBackend("cpu", InfinityConfig(arch=TINY)).init_and_attach_lora()
    with pytest.raises(FileNotFoundError):
        InfinityBackend("cpu", InfinityConfig(encoded_prompt_path="/nonexistent/enc.pt"))._load_or_encode_prompts()


def test_fp32_restatement_runs_on_cpu():
    """The oracle's fp32 member pass on a tiny model (CPU, teacher-forced bits): shapes, finiteness, and
    that a member's fc1 factors change the logits."""
    from oracle import infinity_fp32 as O
    m = InfinityTransformer(TINY)
    m.init_weights(0)
    attach_lora(m, 2, 8.0, ["fc1"])
    D = sum(p.numel() for p in m.parameters() if p.requires_grad)
    sched = scale_schedule("0.06M")[:3]
    data = synthetic_infinity_prompt_data(2, (5, 9), TINY.text_channels)
    idx = torch.tensor([1, 0, 1])
    bits = [torch.randint(0, 2, (3, h * w, TINY.d_tok)) for _, h, w in sched]
    l0 = O.member_logits_fp32(m, data["kv_compact_list"], data["lens_list"], idx, torch.zeros(D), sched, [3.0] * 3,
                              [1.0] * 3, bits)
    l1 = O.member_logits_fp32(m, data["kv_compact_list"], data["lens_list"], idx, torch.randn(D) * 0.1, sched, [3.0] * 3,
                              [1.0] * 3, bits)
    assert [t.shape for t in l0] == [(3, h * w * TINY.d_tok, 2) for _, h, w in sched]
    assert all(torch.isfinite(t).all() for t in l0)
    assert (l0[-1] - l1[-1]).abs().max() > 0
