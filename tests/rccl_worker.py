"""Child process of tests/test_gpu_bench_dist.py::test_rccl_collectives_single_rank: RCCL (torch
backend "nccl") initialised exactly as bench.py's dist_setup does, then the three collective call
sites of the N>1 path on CUDA tensors — es_step.all_gather_members' dist.all_gather, bench.py's
max_over_ranks all-reduce(MAX) and verify_theta_replicas' all-reduce(MIN / MAX) — and a barrier.
One rank: RCCL refuses two ranks on one device, so this is the most of RCCL a 1-GPU box can run."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out = sys.argv[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    import bench
    from hyperscalees_t2i_amd.es_step import DistInfo, theta_checksum
    x = torch.arange(8 * 9, dtype=torch.float32, device="cuda").view(8, 9)
    outs = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, x)
    m = bench.max_over_ranks(3.25, dist.get_world_size())
    th = torch.randn(1000, device="cuda")
    c = theta_checksum(th)
    lo, hi = c.clone(), c.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.barrier()
    res = {"backend": dist.get_backend(), "world": dist.get_world_size(),
           "gather_ok": bool(torch.equal(outs[0], x)), "max_over_ranks": m,
           "checksum_ok": bool(torch.equal(lo, c) and torch.equal(hi, c)),
           "rank": DistInfo.from_env().rank}
    dist.destroy_process_group()
    Path(out).write_text(json.dumps(res))


if __name__ == "__main__":
    main()
