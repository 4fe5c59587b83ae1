"""Where a tile's time goes in the 8-phase kernels: per-workgroup s_memtime stamps from a
diagnostic build of eggroll_lora.hip (-DEGG_STAMPS; tools/_stamps/libeggroll_stamps.so, built
here with `python tools/stamp_probe.py build`, never loaded by the package).

Stamps (wave 0 of each workgroup): 0 start, 1 prologue landed (first barrier), 2 main loop done,
3 ring drained (vmcnt 0 + barrier), 4 epilogue math done (addend / norm), 5 stores drained;
6 / 7 s_memrealtime (100 MHz) at start / end -> clock = d(memtime) / d(realtime) * 100 MHz.
Prints medians of each phase in cycles and us, and how spread the workgroups' start times are
within each round of the grid (lock-step rounds burst their prologue loads / epilogue stores).
usage: python tools/stamp_probe.py [build]"""
import ctypes
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "tools" / "_stamplib" / "libeggroll_stamps.so"  # build only for a stamp run, delete after (13 MB)


def build():
    OUT.parent.mkdir(parents=True, exist_ok=True)
    srcs = ["eggroll_es.hip", "eggroll_lora.hip", "eggroll_model.hip"]
    objs = []
    for s in srcs:
        o = OUT.parent / (Path(s).stem + "_stamps.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                        "-DEGG_STAMPS", f"-I{ROOT / 'include'}", str(ROOT / "hyperscalees_t2i_amd" / "csrc" / s),
                        "-o", str(o)], check=True)
        objs.append(str(o))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", str(OUT)],
                   check=True)
    print(OUT)


def main():
    import numpy as np
    import torch

    sys.path.insert(0, str(ROOT))
    from hyperscalees_t2i_amd import kernels as K

    lib = ctypes.CDLL(str(OUT))
    lib.eggroll_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def report(name, nblocks, launch, reps=3):
        for _ in range(reps):
            launch()
        torch.cuda.synchronize()
        buf = np.zeros(nblocks * 8, dtype=np.uint64)
        assert lib.eggroll_debug_stamps(buf.ctypes.data, buf.size) == 0
        s = buf.reshape(nblocks, 8).astype(np.int64)
        ph = {"prologue": s[:, 1] - s[:, 0], "main": s[:, 2] - s[:, 1], "drain": s[:, 3] - s[:, 2],
              "epi_math": s[:, 4] - s[:, 3], "stores": s[:, 5] - s[:, 4], "total": s[:, 5] - s[:, 0]}
        clk = np.median((s[:, 5] - s[:, 0]) / np.maximum(s[:, 7] - s[:, 6], 1) * 100e6)
        out = {"kernel": name, "blocks": nblocks, "clock_GHz": round(clk / 1e9, 3)}
        for k, v in ph.items():
            out[k + "_cyc"] = int(np.median(v))
            out[k + "_us"] = round(float(np.median(v)) / clk * 1e6, 2)
        # start-time spread inside each round of (up to) 256 concurrently resident workgroups,
        # in dispatch order (realtime stamps, 10 ns)
        t0 = np.sort(s[:, 6])
        spreads = [float(t0[i + 255] - t0[i]) * 10e-3 for i in range(0, len(t0) - 255, 256)]
        out["round_start_spread_us_median"] = round(float(np.median(spreads)), 2) if spreads else None
        out["kernel_wall_us"] = round(float(s[:, 7].max() - s[:, 6].min()) * 10e-3, 1)
        print(json.dumps(out), flush=True)

    # population LoRA GEMM at the Sana attention shape (131072 x 2240 x 2240, r 2)
    M, N, Kd, rpm = 131072, 2240, 2240, 16384
    x = (torch.rand(M, Kd, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand(N, Kd, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    tp = torch.randn(M // rpm, 2 * Kd + 2 * N + 8, device=dev) * 0.1
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    T = torch.randn(M, 2, device=dev)

    def gemm(kern=8):
        rc = lib.eggroll_lora_gemm_sel(ctypes.c_void_p(x.data_ptr()), ctypes.c_int64(Kd), ctypes.c_void_p(W.data_ptr()),
                                       ctypes.c_int64(Kd), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(T.data_ptr()),
                                       ctypes.c_void_p(tp.data_ptr()), ctypes.c_int64(tp.stride(0)),
                                       ctypes.c_int64(2 * Kd), ctypes.c_int32(2), ctypes.c_float(4.0),
                                       ctypes.c_int64(rpm), ctypes.c_int64(M), ctypes.c_int64(N), ctypes.c_int64(Kd),
                                       ctypes.c_void_p(y.data_ptr()), ctypes.c_int64(N), ctypes.c_int32(kern), st)
        assert rc == 0
    report("k_lora_gemm8<2> 131072x2240x2240", 512 * 9, gemm)
    report("k_lora_gemm8n<2> (256x320) 131072x2240x2240", 512 * 7, lambda: gemm(10))
    if len(sys.argv) > 1 and sys.argv[1] == "gemm":
        return
    del x, y

    # DC-AE up-block phase convs with the fused sub-pixel epilogue (eggroll_conv2x2_subpixel_nhwc): the four
    # product shapes (B 8; (H, Cin) -> Cout), bf16 stream
    for H, Cin, Cout in ((512, 256, 128), (256, 512, 256), (128, 512, 512), (64, 1024, 512)):
        xs = torch.randn(8, H, H, Cin, device=dev, dtype=torch.bfloat16)
        w3 = (torch.randn(Cout, Cin, 3, 3, device=dev) / (9 * Cin) ** 0.5)
        from hyperscalees_t2i_amd.dcae import subpixel_phase_weights
        w4 = subpixel_phase_weights(w3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w4p = K.pack_conv3x3_weight(w4, 1)
        bias = torch.randn(Cout, device=dev).bfloat16()
        ys = torch.empty(8, 2 * H, 2 * H, Cout, device=dev, dtype=torch.bfloat16)
        nblk = -(-(8 * (H + 1) * (H + 1)) // 256) * (4 * Cout // 256)

        def up():
            rc = lib.eggroll_conv2x2_subpixel_nhwc(
                ctypes.c_void_p(xs.data_ptr()), ctypes.c_void_p(w4p.data_ptr()), ctypes.c_void_p(bias.data_ptr()),
                ctypes.c_void_p(xs.data_ptr()), ctypes.c_int32(0), ctypes.c_int64(8), ctypes.c_int64(H),
                ctypes.c_int64(H), ctypes.c_int64(Cin), ctypes.c_int64(Cout), ctypes.c_void_p(ys.data_ptr()), None, st)
            assert rc == 0
        report(f"conv2x2_subpixel 8x{H}x{H}x{Cin}->{Cout}", nblk, up)
        del xs, ys
    if len(sys.argv) > 1 and sys.argv[1] == "up":
        return

    # DC-AE ResBlock convs (8 images): 128 ch at 1024^2 (512x128 tile), 256 at 512^2, 512 at 256^2
    for C, hw in ((128, 1024), (256, 512), (512, 256)):
        xc = torch.randn(8, hw, hw, C, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(C, C, 3, 3, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16)
        wp = K.pack_conv3x3_weight(w, 1)
        yc = torch.empty_like(xc)
        bm, bn = (512, 128) if C == 128 else (256, 256)
        nblk = (8 * hw * hw // bm) * (C // bn if C >= bn else 1)

        rs = torch.randn_like(xc)
        nw = torch.randn(C, device=dev).bfloat16()
        nb = torch.randn(C, device=dev).bfloat16()

        def conv(act=0):
            rc = lib.eggroll_conv_nhwc(ctypes.c_void_p(xc.data_ptr()), ctypes.c_void_p(wp.data_ptr()), None,
                                       ctypes.c_int64(8), ctypes.c_int64(hw), ctypes.c_int64(hw), ctypes.c_int64(C),
                                       ctypes.c_int64(C), ctypes.c_int32(3), ctypes.c_int32(1), ctypes.c_int32(act),
                                       ctypes.c_void_p(yc.data_ptr()), st)
            assert rc == 0

        def conv_norm():
            rc = lib.eggroll_conv3x3_rmsnorm_nhwc(
                ctypes.c_void_p(xc.data_ptr()), ctypes.c_void_p(wp.data_ptr()), None, ctypes.c_int64(8),
                ctypes.c_int64(hw), ctypes.c_int64(hw), ctypes.c_int64(C), ctypes.c_int64(C), ctypes.c_int32(1),
                ctypes.c_float(1e-5), ctypes.c_void_p(nw.data_ptr()), ctypes.c_void_p(nb.data_ptr()),
                ctypes.c_void_p(rs.data_ptr()), ctypes.c_void_p(yc.data_ptr()), st)
            assert rc == 0
        report(f"conv3x3 8x{hw}x{hw}x{C}", nblk, conv)
        report(f"conv3x3 8x{hw}x{hw}x{C} silu", nblk, lambda: conv(2))
        if C in (128, 256):
            report(f"conv3x3+rmsnorm 8x{hw}x{hw}x{C}", nblk, conv_norm)
        del xc, yc, rs


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()   # usage: python tools/stamp_probe.py build; then [gemm] on the GPU
    else:
        main()
