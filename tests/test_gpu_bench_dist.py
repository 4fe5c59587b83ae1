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
    assert out.read_text().rstrip().splitlines()[-1] == lines[0]     # ... and it is the last stdout line
    assert len(lines[0].encode()) <= 8192, len(lines[0])              # the driver parses the tail of stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["pop_total"] == 8 and line["config"]["pop_per_gpu"] == 4
    assert line["theta_replicas_identical"] is True
    assert line["value"] > 0 and line["steps"] == 2 and line["warmup"] == 1
    assert line["scaling"] == "weak" and line["cpu_baseline"] is None
    assert "member-shard x2" in line["config"]["parallelism"]


def _run_bench(tmp_path, tag, nproc, extra):
    env = dict(os.environ, EGGROLL_DIST_BACKEND="gloo", EGGROLL_SAME_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0",
               OMP_NUM_THREADS="2", EGGROLL_MIOPEN_FIND="0")
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
               "--gpus", str(nproc)]
    else:
        cmd = [sys.executable, str(ROOT / "bench.py")]
    cmd += ["--steps", "1", "--warmup", "1", "--small", "--no-cpu-baseline"] + extra
    out, err = tmp_path / f"{tag}.out", tmp_path / f"{tag}.err"
    with open(out, "w") as fo, open(err, "w") as fe:
        rc = subprocess.run(cmd, env=env, stdout=fo, stderr=fe, timeout=500, cwd=str(ROOT)).returncode
    assert rc == 0, err.read_text()[-3000:]
    lines = [ln for ln in out.read_text().splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, (out.read_text()[-2000:], err.read_text()[-2000:])
    return json.loads(lines[0])


def test_bench_eight_ranks_configs2_partition(tmp_path):
    """BASELINE configs[2]'s partition — pop 64 as 8 ranks x 8 members — through bench.py itself
    (tiny architecture, 8 gloo ranks sharing cuda:0): every rank's theta' identical
    (verify_theta_replicas), and equal bit for bit to ONE process evaluating all 64 members."""
    eight = _run_bench(tmp_path, "ws8", 8, ["--pop-per-gpu", "8"])
    one = _run_bench(tmp_path, "ws1", 1, ["--pop-per-gpu", "64"])
    assert eight["n_gpus"] == 8 and eight["config"]["pop_total"] == 64 and eight["config"]["pop_per_gpu"] == 8
    assert "member-shard x8" in eight["config"]["parallelism"]
    assert eight["theta_replicas_identical"] is True
    assert one["n_gpus"] == 1 and one["config"]["pop_total"] == 64
    assert eight["theta_final_sha16"] == one["theta_final_sha16"], (eight["theta_final_sha16"], one["theta_final_sha16"])
    print(f"[ws8] theta' {eight['theta_final_sha16']} == single-process pop 64; "
          f"{eight['value']:.2f} vs {one['value']:.2f} member-evals/s (tiny arch, shared device)")


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
