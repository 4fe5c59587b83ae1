"""A/B of two builds of libeggroll on the fp32-residual-stream GEMM epilogues (EPI_RES32 / EPI_GATED32,
eggroll_lora_linear_pop_epi_sel) at the Sana shapes: attn1 to_out (gated, LoRA r 2), attn2 to_out
(res, r 2), the FFN point conv (gated, r 0, K 5632).  fp32 residual and bf16 shadow compared bitwise,
then interleaved timing (median of rounds).
usage: python tools/epi32_lib_ab.py <libA.so> <libB.so> [kernelA kernelB]  (8 / 10, default 8 8)"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from es_lib_ab import bind, timed  # noqa: E402
from hyperscalees_t2i_amd import kernels as K  # noqa: E402


def main(pa, pb, ka=8, kb=8, rounds=7):
    libs = [bind(pa), bind(pb)]
    kern = [int(ka), int(kb)]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(3)
    out = {}
    for name, M, N, Kd, r, epi in (("attn1_to_out_gated32", 131072, 2240, 2240, 2, 5),
                                   ("attn2_to_out_res32", 131072, 2240, 2240, 2, 4),
                                   ("ffn_point_gated32", 131072, 2240, 5632, 0, 5)):
        x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
        W = (torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5).bfloat16()
        rpm = 16384
        tp = torch.randn(M // rpm, 2 * Kd + 2 * N + 8, device=dev, generator=g) * 0.05
        ws = torch.empty(K.lora_workspace_numel(M, Kd, max(r, 1), rpm), device=dev)
        gate = torch.randn(M // 1024, N, device=dev, generator=g)
        res0 = torch.randn(M, N, device=dev, generator=g)
        res = [res0.clone() for _ in libs]
        sh = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in libs]

        def run(i, reset=False):
            if reset:
                res[i].copy_(res0)
            rc = libs[i].eggroll_lora_linear_pop_epi_sel(
                x.data_ptr(), Kd, W.data_ptr(), Kd, None, tp.data_ptr() if r else None, tp.stride(0) if r else 0,
                0, r * Kd, r, 4.0, rpm if r else M, M, N, Kd, sh[i].data_ptr(), N, ws.data_ptr() if r else None, epi,
                res[i].data_ptr(), N, gate.data_ptr() if epi == 5 else None, N, 1024, kern[i], st)
            assert rc == 0, rc
        run(0, True)
        run(1, True)
        torch.cuda.synchronize()
        same = bool(torch.equal(res[0], res[1]) and torch.equal(sh[0], sh[1]))
        ta, tb = [], []
        for _ in range(rounds):
            ta.append(timed(lambda: run(0)))
            tb.append(timed(lambda: run(1)))
        a, b = statistics.median(ta), statistics.median(tb)
        out[name] = {"A_us": round(a, 1), "B_us": round(b, 1), "B_vs_A": round(a / b, 4), "bitwise_equal": same}
        print(json.dumps({name: out[name]}), flush=True)
        del x, W, tp, ws, gate, res0, res, sh
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
