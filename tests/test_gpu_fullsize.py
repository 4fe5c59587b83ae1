"""BASELINE configs at their FULL architecture sizes in the GPU suite (not only in bench.py): one ES epoch
of each host — Sana-Sprint 1.6B at 1024 px (configs[1]), Z-Image-Turbo 6B (configs[3]), Infinity-8B at
pn 0.25M (configs[4]) — with random-init weights of the real shapes, population 2 (one antithetic
pair), through exactly the builders bench.py times.  Checked: every member's rewards finite, the pair's
rewards differ (the LoRA perturbation reaches the images at full size), and theta' equals the oracle's
epoch tail (promptnorm fitness -> EGGROLL update -> norm cap, oracle/eggroll_oracle.py) on the same S
and the same counter-based noise.  Model-level logits parity is covered at tiny sizes
(test_gpu_{sana,zimage,infinity}.py); the kernels at full sizes in test_gpu_kernels.py."""
import gc
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import eggroll_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("workload", ["sana", "zimage", "infinity"])
def test_full_size_epoch(workload, dev):
    import bench
    torch.backends.cudnn.benchmark = False   # bench.py turns MIOpen Find on; a single epoch does not pay it back
    args = SimpleNamespace(workload=workload, small=False, pop_per_gpu=2, latent=32)
    backend, engine, noiser, theta, pop = bench.build(args, 1, 0, dev)
    try:
        assert pop == 2
        new, st = engine.step(theta, seed=7, guidance_scale=backend.cfg.guidance_scale)
        torch.cuda.synchronize()
        S = st["_S"].numpy()
        assert S.shape[0] == pop and np.isfinite(S).all()
        assert not np.array_equal(S[0], S[1])
        eps = noiser.eps_from_factors(noiser.sample_factors(pop, dev, seed=7), pop).cpu().numpy()
        c = engine.cfg
        ref, _ = O.ref_es_tail(S, eps, theta.cpu().numpy(), promptnorm=c.promptnorm, lr_scale=c.lr_scale,
                               sigma=c.sigma, max_step_norm=c.max_step_norm, theta_max_norm=c.theta_max_norm)
        np.testing.assert_allclose(new.cpu().numpy(), ref, rtol=1e-5, atol=1e-8)
        print(f"[fullsize] {workload}: D {theta.numel()}, S {S.shape}, |dtheta| "
              f"{float(np.linalg.norm(ref - theta.cpu().numpy())):.3e}")
    finally:
        del backend, engine, noiser, theta
        gc.collect()
        torch.cuda.empty_cache()
