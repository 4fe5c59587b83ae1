"""Which GEMMs of a full-size Sana ES epoch still go to the vendor library (hipBLASLt / rocBLAS), and what they cost.

F.linear, torch.matmul, Tensor.__matmul__ and torch.bmm are wrapped for ONE engine.step (after one unwrapped
warm-up step); each call is bracketed with events on the current stream and keyed by (caller file:line, operand
shapes, dtype).  Prints one JSON record per key, sorted by total time, with the achieved TF/s.
usage: python tools/vendor_gemm_census.py  ->  gpurun_out/vendor_gemm_census.json"""
import json
import sys
from collections import defaultdict
from pathlib import Path
from types import SimpleNamespace

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import bench
    dev = torch.device("cuda:0")
    args = SimpleNamespace(workload="sana", small=False, pop_per_gpu=8, latent=32)
    be, engine, noiser, theta, pop = bench.build(args, 1, 0, dev)
    theta, _ = engine.step(theta, seed=0, guidance_scale=be.cfg.guidance_scale)
    torch.cuda.synchronize()

    rec = defaultdict(list)
    orig = {"linear": F.linear, "matmul": torch.matmul, "bmm": torch.bmm, "__matmul__": torch.Tensor.__matmul__}

    def flops(a, b, kind):
        if kind == "linear":           # a [..., K], b [N, K]
            return 2 * a.numel() // a.shape[-1] * a.shape[-1] * b.shape[0]
        if a.dim() >= 2 and b.dim() >= 2:
            batch = max(a.numel() // (a.shape[-1] * a.shape[-2]), b.numel() // (b.shape[-1] * b.shape[-2]))
            return 2 * batch * a.shape[-2] * a.shape[-1] * b.shape[-1]
        return 2 * a.numel() * (b.shape[-1] if b.dim() > 1 else 1)

    def wrap(kind):
        fn = orig[kind]

        def w(a, b, *rest, **kw):
            f = sys._getframe(1)
            key = (kind, f"{Path(f.f_code.co_filename).name}:{f.f_lineno}", tuple(a.shape), tuple(b.shape), str(a.dtype))
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = fn(a, b, *rest, **kw)
            e.record()
            rec[key].append((s, e, flops(a, b, kind)))
            return out
        return w

    F.linear = wrap("linear")
    torch.matmul = wrap("matmul")
    torch.bmm = wrap("bmm")
    torch.Tensor.__matmul__ = wrap("__matmul__")
    try:
        theta, _ = engine.step(theta, seed=1, guidance_scale=be.cfg.guidance_scale)
    finally:
        F.linear, torch.matmul, torch.bmm = orig["linear"], orig["matmul"], orig["bmm"]
        torch.Tensor.__matmul__ = orig["__matmul__"]
    torch.cuda.synchronize()
    rows = []
    for (kind, site, sa, sb, dt), v in rec.items():
        ms = sum(s.elapsed_time(e) for s, e, _ in v)
        fl = sum(x for _, _, x in v)
        rows.append({"site": site, "op": kind, "a": sa, "b": sb, "dtype": dt, "calls": len(v), "ms": round(ms, 3),
                     "TFps": round(fl / ms / 1e9, 1) if ms > 0 else None})
    rows.sort(key=lambda r: -r["ms"])
    tot = sum(r["ms"] for r in rows)
    for r in rows:
        print(json.dumps(r), flush=True)
    print(json.dumps({"total_ms_per_epoch": round(tot, 2), "keys": len(rows)}), flush=True)
    out = ROOT / "gpurun_out" / "vendor_gemm_census.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps({"total_ms_per_epoch": tot, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
