"""Bit-exact pins of the SHIPPED host index path (not the oracle's copy) against fixtures made by
the reference's own utills.py (tests/golden/make_golden.py):
  * es.sample_indices_unique / repeat_batches              vs g5  (utills.py:364-379)
  * SanaBackend.step_sampling_info (every dict field)       vs g5b (es_backend.py:234-263)
  * es.sample_classes_unique (VAR class sampler)            vs g5b (es_backend.py:377-396)
  * es_step.aggregate_member_rewards (S and raw means)      vs g9  (unifed_es.py:165-215)
CPU only: this is integer / host logic; tests/test_gpu_engine.py repeats the aggregation on device."""
import numpy as np
import pytest
import torch

from hyperscalees_t2i_amd import es
from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig
from hyperscalees_t2i_amd.es_step import RAW_KEYS, aggregate_member_rewards


def _groups(npz):
    out = {}
    for k in npz.files:
        if "/" in k:
            g, f = k.split("/", 1)
            out.setdefault(g, {})[f] = npz[k]
    return out


def test_product_sample_indices_match_reference(golden):
    g = golden("g5_indices.npz")
    for key in g.files:
        if not key.startswith("P"):
            continue
        P, k = (int(x[1:]) for x in key.split("_"))
        got = np.array([es.sample_indices_unique(seed, P, k) for seed in range(100)], np.int64)
        assert np.array_equal(got, g[key]), key
    assert es.repeat_batches([3, 1, 2, 0], 3) == g["repeat_4x3"].tolist()


def _backend(P, k, R, L, prompts):
    be = SanaBackend("cpu", SanaConfig(synthetic_weights=True, prompts_per_gen=k, batches_per_gen=R, max_log_batches=L))
    be.base_prompt_embeds = torch.zeros(P, 1, 1)
    be.prompts_list = prompts
    return be


def test_step_sampling_info_matches_reference(golden):
    g = _groups(golden("g5b_sampling_info.npz"))
    n = 0
    for key, d in g.items():
        parts = key.split("_")
        P, k, R, L = (int(x[1:]) for x in parts[:4])
        prompts = [f"prompt text {i}" for i in range(P)] if key.endswith("_named") else None
        be = _backend(P, k, R, L, prompts)
        for seed in range(100):
            info = be.step_sampling_info(seed)
            assert info["unique_ids"] == d["unique_ids"][seed].tolist(), (key, seed)
            assert info["flat_ids"] == d["flat_ids"][seed].tolist(), (key, seed)
            assert sorted(info["pid_to_j"].items()) == [tuple(x) for x in d["pid_to_j"][seed].tolist()]
            assert [info["m"], info["total_imgs_per_indiv"], info["total_imgs_for_logging"],
                    info["log_batches"]] == d["scalars"][seed].tolist(), (key, seed)
            assert "\x1f".join(info["unique_texts"] + info["flat_texts"]) == str(d["texts"][seed]), (key, seed)
            n += 1
    assert n == 48 * 100


def test_var_class_sampler_matches_reference(golden):
    g = golden("g5b_sampling_info.npz")
    for allowed, tag in ((None, "all"), ([3, 3, 17, 999, 1000, -1, 42, 7, 17, 500], "list")):
        for m in (1, 4):
            got = np.array([es.sample_classes_unique(s, allowed, m) for s in range(100)], np.int64)
            assert np.array_equal(got, g[f"var_{tag}_m{m}"]), (tag, m)
    with pytest.raises(ValueError):
        es.sample_classes_unique(0, [1, 2], 3)


def _aggregate_case(d, device):
    flat = d["flat_ids"].tolist()
    unique = d["unique_ids"].tolist()
    pid_to_j = {pid: j for j, pid in enumerate(unique)}
    pop = d["S"].shape[0]
    rew = {k: torch.from_numpy(d[f"rew_{k}"]).reshape(-1).to(device) for k in RAW_KEYS}
    return aggregate_member_rewards(rew, flat, pid_to_j, pop, len(unique))


def test_s_aggregation_matches_reference_loop(golden):
    g = _groups(golden("g9_s_aggregation.npz"))
    assert set(g) >= {"m4_R4", "shuffled", "ragged"}
    for name, d in g.items():
        S, raw = _aggregate_case(d, "cpu")
        np.testing.assert_array_equal(S.numpy(), d["S"], err_msg=name)
        np.testing.assert_array_equal(raw.numpy(), d["raw"], err_msg=name)


def test_mix_weights_forms():
    from hyperscalees_t2i_amd.rewards import split_mix_weights
    assert split_mix_weights((0.3, 0.3, 0.4)) == (0.3, 0.3, 0.4, 0.0)
    assert split_mix_weights([0, 0, 0, 1]) == (0.0, 0.0, 0.0, 1.0)
    with pytest.raises(ValueError):
        split_mix_weights((1.0, 2.0))


def test_var_d16_layout_matches_reference_module_tree(golden):
    """model_shapes.var_d16_lora_shapes == the theta layout make_golden.py walked out of the
    reference's VAR_models (PEFT suffix matching of unifed_es.py:406's targets)."""
    from hyperscalees_t2i_amd.model_shapes import var_d16_lora_shapes
    g8 = golden("g8_var.npz")
    assert [tuple(s) for s in g8["shapes"].tolist()] == var_d16_lora_shapes()
    names = str(g8["names"]).split("\x1f")
    assert len(names) == 82 and names[0] == "blocks.0.attn.mat_qkv" and names[-1] == "head"
    assert sum(a * b for a, b in var_d16_lora_shapes()) == 1_540_096
