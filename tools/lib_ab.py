"""A/B of two builds of libeggroll on the population LoRA GEMM (eggroll_lora_gemm_sel, 8-phase kernel):
bitwise equality of the outputs on ragged / member-straddling / bias / no-bias cases, then interleaved
timing at the Sana-1.6B shapes (median of rounds, HIP events on the launch stream).
Build A from a committed revision into tools/_stamps/ (`python tools/lib_ab.py build-a <rev>`), then
run `python tools/lib_ab.py tools/_stamps/libeggroll_a.so hyperscalees_t2i_amd/_build/libeggroll.so`."""
import ctypes
import json
import statistics
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SRCS = ["eggroll_es.hip", "eggroll_lora.hip", "eggroll_model.hip"]


def build_a(rev):
    out = ROOT / "tools" / "_stamps" / "libeggroll_a.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        arc = subprocess.run(["git", "archive", rev, "hyperscalees_t2i_amd/csrc", "include"], cwd=ROOT, check=True,
                             capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", td], input=arc, check=True)
        objs = []
        for s in SRCS:
            src = Path(td) / "hyperscalees_t2i_amd" / "csrc" / s
            o = Path(td) / (src.stem + ".o")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                            f"-I{Path(td) / 'include'}", str(src), "-o", str(o)], check=True)
            objs.append(str(o))
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", str(out)],
                       check=True)
    print(out)


def main(pa, pb, kern=8):
    import torch
    libs = [ctypes.CDLL(str(Path(p).resolve())) for p in (pa, pb)]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    vp, i64, i32, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
    g = torch.Generator(device=dev).manual_seed(3)

    def case(M, N, K, rpm, r, bias):
        x = ((torch.rand(M, K, device=dev, generator=g) * 2 - 1)).bfloat16()
        W = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16()
        b = torch.randn(N, device=dev, generator=g).bfloat16() if bias else None
        members = (M + rpm - 1) // rpm
        tp = torch.randn(members, r * (K + N) + 8, device=dev, generator=g) * 0.1
        T = torch.randn(M, max(r, 1), device=dev, generator=g)
        ys = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in libs]

        def run(i):
            rc = libs[i].eggroll_lora_gemm_sel(vp(x.data_ptr()), i64(K), vp(W.data_ptr()), i64(K),
                                               vp(b.data_ptr() if b is not None else 0), vp(T.data_ptr()),
                                               vp(tp.data_ptr()), i64(tp.stride(0)), i64(r * K), i32(r), f32(4.0),
                                               i64(rpm), i64(M), i64(N), i64(K), vp(ys[i].data_ptr()), i64(N), i32(kern),
                                               st)
            assert rc == 0, rc
        return run, ys

    for M, N, K, rpm, r, bias in ((1000, 300, 256, 300, 2, True), (1000, 300, 256, 300, 1, False),
                                  (4096, 512, 512, 256, 2, True), (2560, 1120, 1152, 640, 1, True),
                                  (3000, 700, 320, 1000, 2, False), (8192, 2240, 2240, 2048, 2, True)):
        run, ys = case(M, N, K, rpm, r, bias)
        run(0)
        run(1)
        torch.cuda.synchronize()
        same = torch.equal(ys[0], ys[1])
        print(json.dumps({"case": [M, N, K, rpm, r, bias], "bitwise_equal": same}), flush=True)
        assert same

    res = {}
    for M, N, K in ((131072, 2240, 2240), (131072, 11200, 2240), (131072, 2240, 5632)):
        run, ys = case(M, N, K, 16384, 2, True)
        ms = [[], []]
        for _ in range(5):
            for i in (0, 1):
                run(i)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    run(i)
                e.record()
                torch.cuda.synchronize()
                ms[i].append(s.elapsed_time(e) / 5)
        a, b = statistics.median(ms[0]), statistics.median(ms[1])
        tf = 2 * M * N * K / 1e9
        res[f"{M}x{N}x{K}"] = {"A_ms": round(a, 4), "B_ms": round(b, 4), "A_TF": round(tf / a, 1),
                               "B_TF": round(tf / b, 1), "B_vs_A": round(a / b, 4),
                               "bitwise_equal": torch.equal(ys[0], ys[1])}
        print(json.dumps({f"{M}x{N}x{K}": res[f"{M}x{N}x{K}"]}), flush=True)
        del ys
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "build-a":
        build_a(sys.argv[2] if len(sys.argv) > 2 else "HEAD")
    else:
        main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 8)
