"""Which op of the full-size member-eval changes its bits when another process shares the GPU?

bench.py --gpus 8 with 8 gloo ranks on ONE device (the opt-in tests/test_gpu_bench_dist_fullsize.py) gave
S rows that differed from the single process's for a timing-dependent subset of ranks, while two
single-process runs were bitwise equal (profiles/r13l_*).  This probe evaluates one pass (8 members, the
full Sana-Sprint 1.6B at 1024 px, DC-AE, CLIP-H + CLIP-B) alone, then again while `hammer` child processes
keep the GPU busy, and reports which stage's output moved: the transformer output, the decoded images, the
two towers' image embeddings — and, inside the towers and the DC-AE, every F.linear / F.conv2d call site
(library GEMMs / convs) through a recording wrapper.
usage: python tools/contention_determinism_probe.py [n_hammers]"""
import hashlib
import json
import os
import subprocess
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

HAMMER = """
import sys, time, torch
dev = torch.device('cuda:0')
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16); b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
x = torch.randn(64 << 20, device=dev)
t_end = time.time() + float(sys.argv[1])
print('hammer up', flush=True)
while time.time() < t_end:
    for _ in range(4):
        c = a @ b
    x.mul_(1.0000001)
    torch.cuda.synchronize()
"""


HAMMER_EVAL = """
import sys, time, torch
from types import SimpleNamespace
sys.path.insert(0, %r)
import bench
dev = torch.device('cuda:0')
torch.backends.cudnn.benchmark = False
args = SimpleNamespace(workload='sana', small=False, pop_per_gpu=8, latent=32)
be, engine, noiser, theta, pop = bench.build(args, 1, 0, dev)
print('hammer up', flush=True)
t_end = time.time() + float(sys.argv[1])
s = 100
while time.time() < t_end:
    with torch.no_grad():
        engine.evaluate_local(theta, s, be.cfg.guidance_scale)
    torch.cuda.synchronize()
    s += 1
""" % str(ROOT)


def digest(t):
    return hashlib.sha256(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12]


class Recorder:
    """Wraps F.linear / F.conv2d: every call's output digest, in call order."""

    def __init__(self):
        self.log, self.on = [], False
        self._lin, self._conv = F.linear, F.conv2d

    def __enter__(self):
        rec = self

        def lin(*a, **k):
            y = rec._lin(*a, **k)
            if rec.on:
                rec.log.append(("linear", tuple(a[0].shape), tuple(a[1].shape), digest(y)))
            return y

        def conv(*a, **k):
            y = rec._conv(*a, **k)
            if rec.on:
                rec.log.append(("conv2d", tuple(a[0].shape), tuple(a[1].shape), digest(y)))
            return y
        F.linear, F.conv2d = lin, conv
        return self

    def __exit__(self, *exc):
        F.linear, F.conv2d = self._lin, self._conv


def main(n_hammers=3):
    import bench
    from hyperscalees_t2i_amd.es_step import aggregate_member_rewards
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = False
    args = SimpleNamespace(workload="sana", small=False, pop_per_gpu=8, latent=32)
    be, engine, noiser, theta, pop = bench.build(args, 1, 0, dev)
    rewards = engine.rewards
    seed, gs = 0, be.cfg.guidance_scale
    fac = noiser.epoch_noise(pop, seed=seed)
    tp = noiser.perturb(theta, fac, pop, 0, pop, out=engine.theta_pop[:pop])
    info = be.step_sampling_info(seed)
    flat, m = info["flat_ids"], info["m"]
    j_of = torch.tensor([info["pid_to_j"][p] for p in flat], device=dev).repeat(pop)
    feats = rewards.prompt_features(info["unique_texts"])
    tr_out = []
    be.es_model.transformer.register_forward_hook(lambda _m, _i, o: tr_out.append(digest(o)))
    t_clip, t_pick = rewards.towers()

    def one(rec):
        tr_out.clear()
        rec.log.clear()
        rec.on = True
        with torch.no_grad():
            imgs = be.generate_population(flat, seed, gs, tp)
            rw = rewards.score(imgs, j_of, feats)
        torch.cuda.synchronize()
        rec.on = False
        S = aggregate_member_rewards(rw, flat, info["pid_to_j"], pop, m)[0]
        return {"tr": list(tr_out), "img": digest(imgs), "S": digest(S), "lib": list(rec.log),
                "S_rows": [digest(S[k]) for k in range(pop)]}

    with Recorder() as rec:
        ref = one(rec)
        again = one(rec)
        print(json.dumps({"alone_repeat_equal": again == ref, "lib_calls": len(ref["lib"])}), flush=True)
        src = HAMMER_EVAL if os.environ.get("PROBE_HAMMER", "eval") == "eval" else HAMMER
        procs = [subprocess.Popen([sys.executable, "-c", src, "240"], stdout=subprocess.PIPE, text=True)
                 for _ in range(n_hammers)]
        for p in procs:
            p.stdout.readline()
        time.sleep(2)
        diffs = []
        try:
            for rep in range(int(os.environ.get("PROBE_REPS", "8"))):
                r = one(rec)
                d = {"rep": rep, "S_equal": r["S"] == ref["S"], "img_equal": r["img"] == ref["img"],
                     "tr_equal": r["tr"] == ref["tr"],
                     "rows_differ": [k for k in range(pop) if r["S_rows"][k] != ref["S_rows"][k]],
                     "lib_differ": [(i,) + ref["lib"][i][:3] for i in range(min(len(r["lib"]), len(ref["lib"])))
                                    if r["lib"][i][3] != ref["lib"][i][3]][:12]}
                diffs.append(d)
                print(json.dumps(d), flush=True)
        finally:
            for p in procs:
                p.kill()
                p.wait()
    out = ROOT / "gpurun_out" / "contention_determinism.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps({"ref_lib_calls": ref["lib"], "diffs": diffs}, indent=1, default=str))


def self_check(tag, reps):
    """One of N identical processes started together: each compares its own repeated evals with its first
    (no hammers: the other instances are the load, as 8 gloo ranks sharing one GPU are)."""
    import bench
    from hyperscalees_t2i_amd.es_step import aggregate_member_rewards
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = False
    args = SimpleNamespace(workload="sana", small=False, pop_per_gpu=8, latent=32)
    be, engine, noiser, theta, pop = bench.build(args, 1, 0, dev)
    rewards = engine.rewards
    seed, gs = 1, be.cfg.guidance_scale
    fac = noiser.epoch_noise(pop, seed=seed)
    tp = noiser.perturb(theta, fac, pop, 0, pop, out=engine.theta_pop[:pop])
    info = be.step_sampling_info(seed)
    flat, m = info["flat_ids"], info["m"]
    j_of = torch.tensor([info["pid_to_j"][p] for p in flat], device=dev).repeat(pop)
    feats = rewards.prompt_features(info["unique_texts"])
    B = len(flat)

    def one(rec):
        rec.log.clear()
        rec.on = True
        with torch.no_grad():
            imgs = be.generate_population(flat, seed, gs, tp)
            rw = rewards.score(imgs, j_of, feats)
        torch.cuda.synchronize()
        rec.on = False
        S = aggregate_member_rewards(rw, flat, info["pid_to_j"], pop, m)[0]
        return {"S_rows": [digest(S[k]) for k in range(pop)], "lib": list(rec.log),
                "img": [digest(imgs[k * B:(k + 1) * B]) for k in range(pop)]}
    out = []
    with Recorder() as rec:
        ref = one(rec)
        for rep in range(reps):
            r = one(rec)
            d = {"rep": rep, "rows_differ": [k for k in range(pop) if r["S_rows"][k] != ref["S_rows"][k]],
                 "img_differ": [k for k in range(pop) if r["img"][k] != ref["img"][k]],
                 "lib_differ": [(i,) + tuple(ref["lib"][i][:3]) for i in range(min(len(r["lib"]), len(ref["lib"])))
                                if r["lib"][i][3] != ref["lib"][i][3]][:12]}
            out.append(d)
            print(tag, json.dumps(d), flush=True)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / f"selfcheck_{tag}.json").write_text(json.dumps({"ref_S_rows": ref["S_rows"], "reps": out}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "self":
        self_check(sys.argv[2], int(sys.argv[3]))
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
