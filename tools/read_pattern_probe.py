"""Strided (64 B per lane, 4 float4 loads) vs coalesced (1 KiB per load instruction) reads of the
rank-4 update's factor stream: 64 rows x 2172 chunks of 16 KiB (the Z-Image layout's 2.28 GB), at
the update kernel's occupancy (5 workgroups per CU via dynamic LDS) and uncapped.
usage: python tools/read_pattern_probe.py [build]"""
import ctypes
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SO = ROOT / "tools" / "_stamps" / "libreadpattern.so"


def build():
    SO.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    str(ROOT / "tools" / "read_pattern_probe.hip"), "-o", str(SO)], check=True)
    print(SO)


def main():
    import statistics
    import torch
    lib = ctypes.CDLL(str(SO))
    lib.rp_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                            ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    nrows, nchunks = 64, 2172
    ld4 = nchunks * 1024 + 64
    f = torch.rand(nrows, ld4 * 4, device=dev)
    sink = torch.empty(nchunks * 256, device=dev)
    nbytes = nrows * nchunks * 16384
    res = {}
    for lds in (32768, 0):
        for co in (0, 1):
            def run():
                assert lib.rp_read(ctypes.c_void_p(f.data_ptr()), ld4, nrows, nchunks, co, lds,
                                   ctypes.c_void_p(sink.data_ptr()), st) == 0
            ts = []
            for _ in range(7):
                run()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(3):
                    run()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) / 3 * 1e3)
            us = statistics.median(ts)
            key = f"{'coalesced' if co else 'strided'}_lds{lds}"
            res[key] = {"us": round(us, 1), "TBps": round(nbytes / us / 1e6, 3)}
            print(json.dumps({key: res[key]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    build() if len(sys.argv) > 1 and sys.argv[1] == "build" else main()
