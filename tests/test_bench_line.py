"""bench.py's stdout contract on the CPU: the headline line a driver parses from the tail of stdout is
compact (≤ 4 KB), valid JSON, and carries the headline keys, `roofline` and `cpu_baseline`, with the
per-kernel tables moved to the aux record (a 22.6-KB line went unparsed)."""
import importlib.util
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    argv = sys.argv
    try:
        sys.argv = ["bench.py"]
        spec.loader.exec_module(m)
    finally:
        sys.argv = argv
    return m


def test_compact_line_from_full_record():
    b = _bench()
    full = json.loads((ROOT / "profiles" / "r12d_bench_line.json").read_text())   # a full round-5 record
    assert len(json.dumps(full)) > 16000
    full["roofline"]["algorithmic_bytes"] = b.algo_bytes("131072x2240x2240")
    s = json.dumps(b.compact_line(full, "gpurun_out/bench_aux.json"), separators=(",", ":"))
    assert len(s.encode()) <= b.LINE_MAX_BYTES
    c = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in c, k
    r = c["roofline"]
    assert r["kernel"] == "k_lora_gemm8n<2,0>" and r["bound"] == "mfma" and r["unit"] == "TFLOP/s"
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["algorithmic_bytes"] == 2.0 * (131072 * 2240 * 2 + 2240 * 2240)
    assert r["mfma_busy"] is not None and r["traffic"] > r["algorithmic_bytes"]
    cpu = c["cpu_baseline"]
    assert set(cpu) == {"value", "unit", "cores", "kind", "sample"} and cpu["kind"] in ("port", "reference")
    assert "\n" not in cpu["sample"]
    assert "model_kernels" not in c and "aux_kernels" not in c


def test_emit_writes_aux_and_prints_last(tmp_path, capsys):
    b = _bench()
    full = json.loads((ROOT / "profiles" / "r12d_bench_line.json").read_text())

    class A:
        aux_out = str(tmp_path / "aux.json")
    b.emit(full, {"all": {}}, A)
    out = capsys.readouterr().out.strip().splitlines()
    c = json.loads(out[-1])
    assert c["value"] == full["value"]
    rec = json.loads((tmp_path / "aux.json").read_text())
    assert rec["line"]["model_kernels"] == full["model_kernels"]
