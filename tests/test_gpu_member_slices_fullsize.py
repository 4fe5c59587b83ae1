"""BASELINE configs[2]'s partition at the full architecture (Sana-Sprint 1.6B, 1024 px, CLIP-H/14 PickScore +
CLIP-B/32): pop 64 over 8 ranks, 8 members per rank.

The reference evaluates every member on its own (unifed_es.py:159-215: theta_k = theta + sigma * eps[k],
unflatten, generate, score), so a member's reward row cannot depend on which other members share its
process.  The build evaluates members in passes of members_per_pass = 8 (SanaConfig) on global member
boundaries (ESEngine.member_passes): this test evaluates the whole pop-64 epoch in ONE process (8 passes)
and, separately, the member slices [0, 8) and [56, 64) as ranks 0 and 7 of 8 (member_shard; evaluate_local,
no collective), and asserts that the slices' S rows — and their raw reward rows — equal the pop-64 rows
bit for bit.  This is the property the node-level metric (bench.py --gpus 8) rests on: the S all-gather of
8 ranks reassembles exactly the single-process S."""
from types import SimpleNamespace

import pytest
import torch

from hyperscalees_t2i_amd.es_step import DistInfo, ESConfig, ESEngine, member_shard

pytestmark = pytest.mark.gpu
POP, WORLD = 64, 8


@pytest.fixture(scope="module")
def full(dev):
    import bench
    torch.backends.cudnn.benchmark = False          # MIOpen immediate mode: solver chosen by shape only
    args = SimpleNamespace(workload="sana", small=False, pop_per_gpu=POP, latent=32)
    backend, engine, noiser, theta, pop = bench.build(args, 1, 0, dev)
    assert pop == POP and engine.cfg.pop_size == POP
    yield backend, engine, noiser, theta


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", [3])
def test_member_slices_equal_pop64_rows(full, dev, seed):
    backend, engine, noiser, theta = full
    gs = backend.cfg.guidance_scale
    assert backend.members_per_pass() == 8
    assert engine.member_passes() == [(a, a + 8) for a in range(0, POP, 8)]
    S_all, raw_all, _, info = engine.evaluate_local(theta, seed, gs)
    assert S_all.shape == (POP, info["m"]) and torch.isfinite(S_all).all()
    for rank in (0, WORLD - 1):
        lo, hi = member_shard(POP, rank, WORLD)
        assert (lo, hi) == (8 * rank, 8 * rank + 8)
        cfg = ESConfig(**{**engine.cfg.__dict__})
        shard = ESEngine(backend, engine.rewards, noiser, cfg, dev, DistInfo(rank, WORLD, None))
        assert (shard.lo, shard.hi) == (lo, hi) and shard.member_passes() == [(0, 8)]
        S_r, raw_r, _, info_r = shard.evaluate_local(theta, seed, gs)
        assert info_r["flat_ids"] == info["flat_ids"]
        assert torch.equal(S_r, S_all[lo:hi]), (rank, float((S_r - S_all[lo:hi]).abs().max()))
        assert torch.equal(raw_r, raw_all[lo:hi]), rank
    # antithetic partners live in different slices (member k and k + 32): their rows differ
    assert not torch.equal(S_all[0], S_all[POP // 2])
    print(f"[member-slices] pop {POP}: ranks 0 and {WORLD - 1} of {WORLD} reproduce rows [0, 8) and [56, 64) "
          f"bitwise; S spread {float(S_all.std(0).mean()):.4f}")
