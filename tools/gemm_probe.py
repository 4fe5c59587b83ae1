"""Quick A/B of the population LoRA GEMM vs torch (hipBLASLt) at Sana shapes (diagnostic)."""
import sys, time, json
import torch
sys.path.insert(0, '.')
from hyperscalees_t2i_amd import kernels as K

def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it

dev = torch.device('cuda:0')
res = []
for (M, N, Kd, rpm) in [(8*16384, 2240, 2240, 16384), (8*4800, 2240, 2240, 4800), (8*16384, 32, 2240, 16384), (8*16384, 11200, 2240, 16384)]:
    x = torch.randn(M, Kd, device=dev).bfloat16()
    W = (torch.randn(N, Kd, device=dev) * 0.05).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    tp = torch.randn(8, 2*Kd + 2*N + 8, device=dev) * 0.1
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    T = torch.empty(M*2, device=dev)
    from hyperscalees_t2i_amd import _lib
    _lib.call("eggroll_lora_gemm_tile", 128)
    t_128 = bench(lambda: K.lora_linear_pop(x, W, b, tp, 0, 2*Kd, 2, 4.0, rpm, out=y, T_ws=T))
    _lib.call("eggroll_lora_gemm_tile", 256)
    t_256 = bench(lambda: K.lora_linear_pop(x, W, b, tp, 0, 2*Kd, 2, 4.0, rpm, out=y, T_ws=T))
    _lib.call("eggroll_lora_gemm_tile", 0)
    t_ours = bench(lambda: K.lora_linear_pop(x, W, b, tp, 0, 2*Kd, 2, 4.0, rpm, out=y, T_ws=T))
    t_base = bench(lambda: K.lora_linear_pop(x, W, b, None, 0, 0, 0, 0.0, rpm, out=y))
    t_proj = bench(lambda: K.lora_project(x, tp, 0, 2, rpm, out=T.view(M, 2)))
    t_torch = bench(lambda: torch.nn.functional.linear(x, W, b))
    fl = 2 * M * N * Kd
    r = dict(M=M, N=N, K=Kd, tile128_tflops=fl / t_128 / 1e9, tile256_tflops=fl / t_256 / 1e9, ours_ms=t_ours, base_ms=t_base, project_ms=t_proj, torch_ms=t_torch,
             ours_tflops=fl / t_ours / 1e9, base_tflops=fl / t_base / 1e9, torch_tflops=fl / t_torch / 1e9,
             project_GBps=M * Kd * 2 / t_proj / 1e6)
    print(json.dumps(r), flush=True)
