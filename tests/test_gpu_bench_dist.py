"""bench.py's N>1 path end to end, on one GPU: `torch.distributed.run --nproc-per-node 2 bench.py
--gpus 2` started as a fresh child process (no GPU call in the test process before it), with
EGGROLL_DIST_BACKEND=gloo EGGROLL_SAME_DEVICE=1 so both ranks share cuda:0 (RCCL refuses two ranks on
one device).  Runs the exact code the driver's 8-GPU scaling bench runs — dist_setup, the barriers
around the timed region, max_over_ranks, the S all-gather inside ESEngine.step and
verify_theta_replicas — on the tiny architecture."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_same_device(tmp_path):
    env = dict(os.environ, EGGROLL_DIST_BACKEND="gloo", EGGROLL_SAME_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0",
               OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--small", "--no-cpu-baseline", "--pop-per-gpu", "4"]
    out = tmp_path / "bench.out"
    with open(out, "w") as fo, open(tmp_path / "bench.err", "w") as fe:
        rc = subprocess.run(cmd, env=env, stdout=fo, stderr=fe, timeout=400, cwd=str(ROOT)).returncode
    err_tail = (tmp_path / "bench.err").read_text()[-3000:]
    assert rc == 0, err_tail
    lines = [ln for ln in out.read_text().splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, (out.read_text()[-2000:], err_tail)     # rank 0 prints exactly one line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["pop_total"] == 8 and line["config"]["pop_per_gpu"] == 4
    assert line["theta_replicas_identical"] is True
    assert line["value"] > 0 and line["steps"] == 2 and line["warmup"] == 1
    assert line["scaling"] == "weak" and line["cpu_baseline"] is None
    assert "member-shard x2" in line["config"]["parallelism"]


def test_rccl_collectives_single_rank(tmp_path):
    """RCCL itself on the box: a fresh child process inits the "nccl" backend as bench.py does and runs
    the all-gather / all-reduce / barrier call sites of the N>1 path on CUDA tensors (world size 1)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    out = tmp_path / "rccl.json"
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "rccl_worker.py"), str(out)], env=env, timeout=240,
                       capture_output=True, text=True, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["gather_ok"] and res["checksum_ok"] and res["max_over_ranks"] == 3.25
