"""The real member-sharded ESEngine.step in two processes: two fresh child processes,
each one rank on cuda:0 with the gloo backend (RCCL refuses two ranks on one device), run the same
epoch on their member shard, all-gather S, then fitness + update + verify_theta_replicas.

Asserted: theta' is bit-identical on both ranks (and verify_theta_replicas stayed silent — it
raises otherwise), the gathered S equals the single-process S of the same epoch up to the bf16
batch-composition drift (a member's rows go through GEMMs of a different M, so library kernels may
pick another tiling), and theta' is the oracle's reference tail (unifed_es.py:227-281) applied to
the gathered S, with ranks equal to the reference argsort."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = Path(__file__).resolve().parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_process_engine_step(dev, tmp_path):
    from oracle import eggroll_oracle as O
    sys.path.insert(0, str(HERE))
    from dist_engine_worker import build_tiny
    from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params
    from hyperscalees_t2i_amd.es_step import ESConfig, ESEngine

    world, pop, port = 2, 4, _free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, str(HERE / "dist_engine_worker.py"), str(r), str(world), str(port),
                               str(tmp_path / f"r{r}.pt"), str(pop)], env=env) for r in range(world)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    res = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    assert [tuple(r["shard"]) for r in res] == [(0, 2), (2, 4)]
    assert torch.equal(res[0]["theta"], res[1]["theta"]), "theta' differs across ranks"
    assert torch.equal(res[0]["S"], res[1]["S"]) and torch.equal(res[0]["order"], res[1]["order"])

    # single-process epoch on the same seeds
    be, rewards = build_tiny(dev)
    params, shapes = be.collect_lora_params()
    theta = flatten_params(params).to(dev)
    assert torch.equal(theta.cpu(), res[0]["theta0"])
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=1, use_antithetic=True)
    eng = ESEngine(be, rewards, noiser, ESConfig(pop_size=pop, theta_max_norm=40.0), dev)
    new1, st1 = eng.step(theta, seed=3, guidance_scale=4.5)
    S2 = res[0]["S"].numpy()
    np.testing.assert_allclose(S2, st1["_S"].numpy(), rtol=2e-2, atol=2e-2)

    eps = noiser.eps_from_factors(noiser.sample_factors(pop, dev, seed=3), pop).cpu().numpy()
    ref, info = O.ref_es_tail(S2, eps, theta.cpu().numpy(), promptnorm=True, lr_scale=1e-1, sigma=1e-2,
                              max_step_norm=0.0, theta_max_norm=40.0)
    np.testing.assert_allclose(res[0]["theta"].numpy(), ref, rtol=1e-5, atol=1e-8)
    assert np.array_equal(res[0]["order"].numpy(), info["order"])
