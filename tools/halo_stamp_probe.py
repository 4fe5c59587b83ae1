"""Where a multi-tile halo conv workgroup's time goes (kernel 4) vs the one-tile kernel (2): s_memtime
stamps from a -DEGG_STAMPS build (tools/_stamps/libeggroll_stamps.so, `python tools/halo_stamp_probe.py
build`; never loaded by the package).  Kernel 2 stamps: 0 start, 1 prologue landed, 2 main loop done,
3 ring drained, 4 epilogue math, 5 stores drained.  Kernel 4: 0 start, 1 first tile's data landed,
2 tile 0's main loop done, 3 tile 0's epilogue done, 5 all tiles done -> the later tiles' average.
usage: python tools/halo_stamp_probe.py [build]"""
import ctypes
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "tools" / "_ab" / "libeggroll_stamps.so"   # travels to the GPU box (git-ignored)


def build():
    OUT.parent.mkdir(parents=True, exist_ok=True)
    objs = []
    for src in ["eggroll_es.hip", "eggroll_lora.hip", "eggroll_model.hip"]:
        o = OUT.parent / (Path(src).stem + "_stamps.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                        "-DEGG_STAMPS", f"-I{ROOT / 'include'}", str(ROOT / "hyperscalees_t2i_amd" / "csrc" / src),
                        "-o", str(o)], check=True)
        objs.append(str(o))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", str(OUT)], check=True)
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
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    for C, hw in ((128, 1024), (256, 512), (512, 256)):
        x = torch.randn(8, hw, hw, C, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(C, C, 3, 3, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16)
        wp = K.pack_conv3x3_weight(w, 1)
        y = torch.empty_like(x)
        tiles = (8 * hw * hw // 512) if C == 128 else (8 * hw * hw // 256) * (C // 256)
        for kern in (2, 4):
            nblk = tiles if kern == 2 else tiles // 4
            for _ in range(3):
                assert lib.eggroll_conv_nhwc_sel(vp(x.data_ptr()), vp(wp.data_ptr()), None, i64(8), i64(hw), i64(hw),
                                                 i64(C), i64(C), i32(3), i32(1), i32(0), vp(y.data_ptr()), i32(kern),
                                                 st) == 0
            torch.cuda.synchronize()
            buf = np.zeros(nblk * 8, dtype=np.uint64)
            assert lib.eggroll_debug_stamps(buf.ctypes.data, buf.size) == 0
            s = buf.reshape(nblk, 8).astype(np.int64)
            clk = np.median((s[:, 5] - s[:, 0]) / np.maximum(s[:, 7] - s[:, 6], 1) * 100e6)
            med = lambda v: int(np.median(v))  # noqa: E731
            if kern == 2:
                out = {"prologue": med(s[:, 1] - s[:, 0]), "main": med(s[:, 2] - s[:, 1]),
                       "drain": med(s[:, 3] - s[:, 2]), "epilogue": med(s[:, 5] - s[:, 3]),
                       "tile": med(s[:, 5] - s[:, 0])}
            else:
                out = {"tile0_prologue": med(s[:, 1] - s[:, 0]), "tile0_main": med(s[:, 2] - s[:, 1]),
                       "tile0_epilogue": med(s[:, 3] - s[:, 2]), "later_tile_avg": med((s[:, 5] - s[:, 3]) / 3),
                       "workgroup": med(s[:, 5] - s[:, 0])}
            wall = float(s[:, 7].max() - s[:, 6].min()) * 10e-9
            out.update({"kernel": kern, "shape": f"8x{hw}x{hw}x{C}", "clock_GHz": round(clk / 1e9, 3),
                        "wall_us": round(wall * 1e6, 1),
                        # cycles per workgroup a CU delivers (wall x clock x 256 CUs / workgroups): vs the
                        # median workgroup duration, the time lost between workgroups
                        "cu_cycles_per_workgroup": int(wall * clk * 256 / nblk)})
            print(json.dumps(out), flush=True)
        del x, y


if __name__ == "__main__":
    build() if len(sys.argv) > 1 and sys.argv[1] == "build" else main()
