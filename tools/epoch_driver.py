"""One full Sana ES epoch (bench.py's configs[1] build: pop 8, 16 images per member, 1024 px) after
one warm-up epoch, for rocprofv3 --pmc / --kernel-trace censuses of every kernel the epoch launches
(tools/pmc_epoch.sh, tools/pmc_epoch_summary.py).  The epoch is bracketed by two marker launches
(tools/trace_window.py's convention) so the census can exclude the build and the warm-up.
usage: python tools/epoch_driver.py   (diagnostic)"""
import sys
from pathlib import Path
from types import SimpleNamespace

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import bench
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda:0")
    be, eng, nz, theta, _ = bench.build(SimpleNamespace(workload="sana", small=False, pop_per_gpu=8, latent=32),
                                        1, 0, dev)
    gs = be.cfg.guidance_scale
    theta = eng.step(theta, 0, gs)[0]
    torch.cuda.synchronize()
    print("warm", flush=True)
    bench.marker()
    theta = eng.step(theta, 1, gs)[0]
    bench.marker()
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
