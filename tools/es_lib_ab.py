"""A/B of two builds of libeggroll on the ES arithmetic kernels (noise, perturb, update + caps) at the
bench's aux layouts: Sana-Sprint 1.6B (egg rank 1, pop 64, 8 local members) and Z-Image-Turbo
(configs[3]: egg rank 4, pop 128, 16 local members).  Outputs of A and B are compared bitwise, then
each kernel is timed interleaved (median of rounds, HIP events on the launch stream).
Build A first: `python tools/lib_ab.py build-a <rev>`.
usage: python tools/es_lib_ab.py tools/_stamps/libeggroll_a.so hyperscalees_t2i_amd/_build/libeggroll.so"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hyperscalees_t2i_amd import _lib, kernels as K  # noqa: E402
from hyperscalees_t2i_amd.model_shapes import zimage_turbo_lora_shapes  # noqa: E402
from hyperscalees_t2i_amd.sana import sana_lora_shapes  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(str(Path(path).resolve()))
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def timed(fn, it=5):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main(pa, pb, rounds=7):
    libs = [bind(pa), bind(pb)]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for name, shapes, rank, pop, nloc in (("sana_r1_pop64", sana_lora_shapes(), 1, 64, 8),
                                          ("sana_r1_pop8", sana_lora_shapes(), 1, 8, 8),
                                          ("zimage_r4_pop128", zimage_turbo_lora_shapes(), 4, 128, 16)):
        lay = K.ThetaLayout(shapes, rank)
        nb = K.n_base_samples(pop, True)
        mats, tiles = lay.mats_on(dev), lay.tiles_on(dev)
        theta = torch.randn(lay.D, device=dev) * 0.01
        S = torch.randn(pop, 4, device=dev) + 21
        fit = K.fitness(S, True)
        ws = [K.UpdateWorkspace(lay, dev) for _ in libs]
        fac = [torch.empty((nb, lay.factor_ld), device=dev) for _ in libs]
        tp = [torch.empty((nloc, K._pad4(lay.D)), device=dev) for _ in libs]
        upd = [torch.empty_like(theta) for _ in libs]

        def noise(i):
            assert libs[i].eggroll_noise_factors(7, 0, nb, lay.factor_len, lay.factor_ld, fac[i].data_ptr(), st) == 0

        def perturb(i):
            assert libs[i].eggroll_perturb(theta.data_ptr(), fac[i].data_ptr(), fac[i].stride(0), nb, mats.data_ptr(),
                                           tiles.data_ptr(), lay.n_tiles, lay.D, rank, pop, 1, 0, nloc, 1e-2,
                                           tp[i].data_ptr(), tp[i].stride(0), st) == 0

        def update(i):
            assert libs[i].eggroll_update(theta.data_ptr(), fac[i].data_ptr(), fac[i].stride(0), nb,
                                          fit["fitness"].data_ptr(), fit["stats"].data_ptr(), pop, 1, mats.data_ptr(),
                                          tiles.data_ptr(), lay.n_tiles, lay.D, rank, 1e-3, 0.0, 40.0,
                                          ws[i].buf.data_ptr(), upd[i].data_ptr(), st) == 0

        tps = [torch.empty((nloc, K._pad4(lay.D)), device=dev) for _ in libs]
        tpp = [torch.empty((pop, K._pad4(lay.D)), device=dev) for _ in libs]

        def perturb_seeded(i):   # this GPU's members of the node-level population (default engine path)
            assert libs[i].eggroll_perturb_seeded(7, theta.data_ptr(), mats.data_ptr(), tiles.data_ptr(), lay.n_tiles,
                                                  lay.D, rank, pop, 1, 0, nloc, 1e-2, tps[i].data_ptr(),
                                                  tps[i].stride(0), st) == 0

        def perturb_seeded_all(i):   # one process over the whole population (N = 1 at pop = pop)
            assert libs[i].eggroll_perturb_seeded(7, theta.data_ptr(), mats.data_ptr(), tiles.data_ptr(), lay.n_tiles,
                                                  lay.D, rank, pop, 1, 0, pop, 1e-2, tpp[i].data_ptr(),
                                                  tpp[i].stride(0), st) == 0

        res = {}
        for kname, fn, buf in (("noise", noise, fac), ("perturb", perturb, tp), ("update_caps", update, upd),
                               ("perturb_seeded", perturb_seeded, tps),
                               ("perturb_seeded_allpop", perturb_seeded_all, tpp)):
            fn(0)
            fn(1)
            torch.cuda.synchronize()
            same = torch.equal(buf[0], buf[1])
            us = [[], []]
            for _ in range(rounds):
                for i in (0, 1):
                    us[i].append(timed(lambda: fn(i)))
            a, b = statistics.median(us[0]), statistics.median(us[1])
            res[kname] = {"A_us": round(a, 2), "B_us": round(b, 2), "B_vs_A": round(a / b, 4), "bitwise_equal": same}
            print(json.dumps({name: {kname: res[kname]}}), flush=True)
            assert same, (name, kname)
        out[name] = res
        del fac, tp, upd, tps, tpp
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
