"""Are the library GEMMs of the member-eval (F.linear -> hipBLASLt: the DC-AE's 1x1 convs, the CLIP towers)
bitwise repeatable while other processes share the GPU?  Each shape's output is computed alone (reference),
then repeatedly while `n` child processes run the same GEMM mix in a loop; every repeat is compared bitwise.
usage: python tools/blas_contention_probe.py [n_children] [reps]"""
import hashlib
import json
import subprocess
import sys
import time

import torch
import torch.nn.functional as F

SHAPES = [((8192, 1024), (3072, 1024)), ((8192, 2048), (1024, 2048)), ((8192, 1024), (8192, 1024)),
          ((8192, 4096), (1024, 4096)), ((32768, 1024), (3072, 1024)), ((32768, 2048), (1024, 2048)),
          ((32768, 1024), (8192, 1024)), ((32768, 4096), (1024, 4096)), ((131072, 1024), (512, 1024)),
          ((131072, 2048), (512, 2048)), ((32896, 1280), (1280, 1280)), ((32896, 5120), (1280, 5120)),
          ((6400, 768), (2304, 768)), ((6400, 768), (768, 768)), ((6400, 768), (3072, 768)), ((6400, 3072), (768, 3072))]

CHILD = """
import sys, time, torch, torch.nn.functional as F
shapes = %r
dev = torch.device('cuda:0')
ops = [(torch.randn(a, device=dev).bfloat16(), torch.randn(w, device=dev).bfloat16()) for a, w in shapes]
print('up', flush=True)
t_end = time.time() + float(sys.argv[1])
while time.time() < t_end:
    for x, w in ops:
        F.linear(x, w)
    torch.cuda.synchronize()
"""


def main(n_children=7, reps=30):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    ops = [(torch.randn(a, device=dev, generator=g).bfloat16(), torch.randn(w, device=dev, generator=g).bfloat16(),
            torch.randn(w[0], device=dev, generator=g).bfloat16()) for a, w in SHAPES]

    def run():
        return [hashlib.sha256(F.linear(x, w, b).view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12]
                for x, w, b in ops]
    ref = run()
    assert run() == ref
    kids = [subprocess.Popen([sys.executable, "-c", CHILD % (SHAPES,), "600"], stdout=subprocess.PIPE, text=True)
            for _ in range(n_children)]
    for k in kids:
        k.stdout.readline()
    diff = {}
    try:
        t0 = time.time()
        for r in range(reps):
            got = run()
            for i, (a, b) in enumerate(zip(got, ref)):
                if a != b:
                    diff.setdefault(str(SHAPES[i]), 0)
                    diff[str(SHAPES[i])] += 1
            if r % 5 == 4:
                print(json.dumps({"rep": r + 1, "elapsed_s": round(time.time() - t0, 1), "differ": diff}), flush=True)
    finally:
        for k in kids:
            k.kill()
            k.wait()
    print(json.dumps({"reps": reps, "children": n_children, "shapes_differing": diff}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 7, int(sys.argv[2]) if len(sys.argv) > 2 else 30)
