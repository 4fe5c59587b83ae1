"""World-size-2 gloo tests of the member sharding and the S all-gather (CPU, no GPU)."""
import os
import socket

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


@pytest.mark.parametrize("pop,world", [(8, 2), (7, 2), (5, 3)])
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


def test_member_shard_partition():
    for pop in range(1, 70):
        for world in range(1, 9):
            spans = [member_shard(pop, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == pop
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


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


@pytest.mark.parametrize("diverge", [False, True])
def test_verify_theta_replicas_gloo(diverge):
    """theta checksum all-reduce (SURVEY §8e debug): silent when replicas agree, raises on EVERY rank
    when one rank's theta differs by one ulp in one element."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, world = _free_port(), 2
    procs = [ctx.Process(target=_verify_worker, args=(r, world, port, diverge, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert set(res.values()) == {"diverged" if diverge else "ok"}
