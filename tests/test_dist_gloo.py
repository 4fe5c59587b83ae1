"""gloo tests (CPU, no GPU) of the member sharding, the S all-gather and the replica check at world sizes
2, 3 and 8 (BASELINE configs[2]: pop 64 over 8 ranks)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hyperscalees_t2i_amd.es_step import DistInfo, all_gather_members, member_shard, verify_theta_replicas
from oracle import eggroll_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, pop, m, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = member_shard(pop, rank, world)
        g = torch.Generator().manual_seed(0)
        S_full = torch.randn(pop, m, generator=g) + 20
        local = S_full[lo:hi].clone()
        S = all_gather_members(local, pop, DistInfo(rank, world))
        ok = torch.equal(S, S_full)
        # every rank then derives identical fitness / ranks (oracle restatement of kernel 3)
        f = O.dev_fitness(S.numpy(), True)
        q.put((rank, ok, f["order"].tolist(), f["fitness"].tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pop,world", [(8, 2), (7, 2), (5, 3), (64, 8)])
def test_allgather_members_gloo(pop, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pop, 4, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res)
    assert len({(tuple(o), fb) for _, _, o, fb in res}) == 1  # identical on all ranks


def _epoch_worker(rank, world, port, pop, m, q):
    """One configs[2]-shaped ES epoch tail on a rank: its members' S rows (each a function of the member
    index only, as a member's evaluation is), the S all-gather, then fitness -> EGGROLL update -> theta
    cap on the gathered S with the noise regenerated locally from (seed, base sample) (kernel (1)'s
    contract, oracle restatement), and the replica check."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        theta, eps = _epoch_inputs(pop)
        lo, hi = member_shard(pop, rank, world)
        local = torch.stack([_member_scores(k, m) for k in range(lo, hi)])
        S = all_gather_members(local, pop, DistInfo(rank, world))
        after, info = O.ref_es_tail(S.numpy(), eps, theta, promptnorm=True, lr_scale=0.1, sigma=0.01,
                                    max_step_norm=0.0, theta_max_norm=40.0)
        verify_theta_replicas(torch.from_numpy(after), DistInfo(rank, world))
        q.put((rank, hi - lo, after.tobytes(), info["order"].tolist()))
    finally:
        dist.destroy_process_group()


SHAPES_SMALL = [(2, 12), (10, 2), (2, 7), (5, 2)]


def _epoch_inputs(pop):
    lay = O.layout(SHAPES_SMALL, 1)
    fac = O.noise_factors(9, 0, O.n_base_samples(pop, True), lay["factor_len"])
    # the per-matrix [a | b] factor vector with the device layout's 4-float padding removed
    eps = O.dev_eps_rows(_unpad(fac, SHAPES_SMALL), SHAPES_SMALL, pop, 1, True, 0, pop)
    theta = np.random.default_rng(4).standard_normal(eps.shape[1]).astype(np.float32)
    return theta, eps


def _unpad(fac, shapes):
    parts, off = [], 0
    for mm, nn in shapes:
        for n in (mm, nn):
            parts.append(fac[:, off:off + n])
            off += -(-n // 4) * 4
    return np.concatenate(parts, axis=1)


def _member_scores(k, m):
    return torch.randn(m, generator=torch.Generator().manual_seed(1000 + k)) + 20


def test_configs2_eight_rank_epoch_gloo():
    """BASELINE configs[2]'s partition (pop 64 over 8 ranks, 8 members each) on CPU gloo: every rank
    ends with the same theta' (verify_theta_replicas passes on all 8), equal bit for bit to the
    single-process epoch tail over the whole population."""
    pop, world, m = 64, 8, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_epoch_worker, args=(r, world, port, pop, m, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(n for _, n, _, _ in res) == [8] * 8
    theta, eps = _epoch_inputs(pop)
    S = torch.stack([_member_scores(k, m) for k in range(pop)]).numpy()
    after, info = O.ref_es_tail(S, eps, theta, promptnorm=True, lr_scale=0.1, sigma=0.01, max_step_norm=0.0,
                                theta_max_norm=40.0)
    assert {b for _, _, b, _ in res} == {after.tobytes()}
    assert all(o == info["order"].tolist() for _, _, _, o in res)
    assert not np.array_equal(after, theta)


def test_member_shard_partition():
    for pop in range(1, 70):
        for world in range(1, 9):
            spans = [member_shard(pop, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == pop
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_member_passes_on_global_boundaries():
    """ESEngine.member_passes: passes of members_per_pass sit on global member indices.  Every global
    pass is the union of the ranks' passes that overlap it, and with shard boundaries on multiples of
    the pass size (pop 64 / 8 ranks, pop 24 / 3 ranks) each rank's passes ARE the global passes."""
    from types import SimpleNamespace
    from hyperscalees_t2i_amd.es_step import ESEngine

    def passes(pop, rank, world, per):
        e = ESEngine.__new__(ESEngine)
        e.lo, e.hi = member_shard(pop, rank, world)
        e.backend = SimpleNamespace(members_per_pass=lambda: per)
        return [(e.lo + a, e.lo + b) for a, b in e.member_passes()]

    for pop in (1, 7, 8, 24, 64, 65):
        for per in (1, 3, 8):
            single = passes(pop, 0, 1, per)
            assert single == [(a, min(pop, a + per)) for a in range(0, pop, per)]
            for world in (2, 3, 8):
                got = [p for r in range(world) for p in passes(pop, r, world, per)]
                assert got[0][0] == 0 and got[-1][1] == pop and all(a[1] == b[0] for a, b in zip(got, got[1:]))
                assert all(a // per == (b - 1) // per for a, b in got)       # no pass straddles a global one
                if all(member_shard(pop, r, world)[0] % per == 0 for r in range(world)):
                    assert got == single
    assert passes(24, 1, 2, 8) == [(12, 16), (16, 24)]                      # shard starting mid-pass
    e = ESEngine.__new__(ESEngine)
    e.lo, e.hi, e.backend = 3, 9, SimpleNamespace()                          # no pass size: one pass
    assert e.member_passes() == [(0, 6)]


def _verify_worker(rank, world, port, diverge, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        theta = torch.randn(1000, generator=torch.Generator().manual_seed(3))
        if diverge and rank == world - 1:
            theta[517] = torch.nextafter(theta[517], torch.tensor(1e9))  # one ulp on one rank
        try:
            verify_theta_replicas(theta, DistInfo(rank, world))
            q.put((rank, "ok"))
        except RuntimeError as e:
            q.put((rank, "diverged" if "diverged" in str(e) else str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("diverge,world", [(False, 2), (True, 2), (False, 8), (True, 8)])
def test_verify_theta_replicas_gloo(diverge, world):
    """theta checksum all-reduce (SURVEY §8e debug): silent when replicas agree, raises on EVERY rank
    when one rank's theta differs by one ulp in one element."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_verify_worker, args=(r, world, port, diverge, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert set(res.values()) == {"diverged" if diverge else "ok"}
