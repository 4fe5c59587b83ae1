"""HBM traffic per launch of the population LoRA GEMM from two rocprofv3 --pmc passes.

FETCH_SIZE / WRITE_SIZE are KiB.  gfx950: FETCH_SIZE counts exactly half the bytes of a wide
coalesced stream (16 B/lane global_load / LDS-DMA), so it is doubled (MI355X_MICROARCH.md §HBM);
WRITE_SIZE is exact for 16-B stores.  Algorithmic bytes per launch: X (M*K*2) + W (N*K*2) +
Y (M*N*2) + T (M*r*4).  Writes profiles/pmc_lora_gemm.json.
usage: python tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE [reps]"""
import csv, json, sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tools.sana_layers import sana_lora_layers  # noqa: E402

import argparse  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("fetch_dir")
ap.add_argument("write_dir")
ap.add_argument("reps", type=int, nargs="?", default=2)
ap.add_argument("--l2", default="", help="pass with TCC_HIT_sum / TCC_MISS_sum")
ap.add_argument("--ea", default="", help="pass with TCC_EA0_RDREQ_sum / TCC_EA0_RDREQ_DRAM_sum")
ap.add_argument("--out", default="profiles/pmc_lora_gemm.json")
A = ap.parse_args()
fetch_dir, write_dir, reps = A.fetch_dir, A.write_dir, A.reps


def load(d, name):
    tot, n = 0.0, 0
    for r in csv.DictReader(open(Path(d) / "run_counter_collection.csv")):
        if "k_lora_gemm" in r["Kernel_Name"] and r["Counter_Name"] == name:
            tot += float(r["Counter_Value"])
            n += 1
    return tot, n


f_kib, nf = load(fetch_dir, "FETCH_SIZE")
w_kib, nw = load(write_dir, "WRITE_SIZE")
launches = nf
alg = 0.0
for rows, Kd, N, cnt in sana_lora_layers():
    M = rows * 8
    alg += cnt * (M * Kd * 2 + N * Kd * 2 + M * N * 2 + M * 2 * 4)
alg_per_launch = alg / (launches / reps)
read_b = 2 * f_kib * 1024 / launches
write_b = w_kib * 1024 / launches
out = {"kernel": "k_lora_gemm (population LoRA GEMM)", "launches_profiled": launches,
       "fetch_bytes_per_launch_corrected": read_b, "write_bytes_per_launch": write_b,
       "hbm_bytes_per_launch": read_b + write_b, "algorithmic_bytes_per_launch": alg_per_launch,
       "traffic_over_algorithmic": (read_b + write_b) / alg_per_launch,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, "
                 "--kernel-include-regex k_lora_gemm, tools/lora_epoch_driver.py (one epoch's launch mix x2); "
                 "FETCH_SIZE doubled per the gfx950 note"}
if A.l2:
    hit, _ = load(A.l2, "TCC_HIT_sum")
    miss, _ = load(A.l2, "TCC_MISS_sum")
    out["l2_hit_rate"] = hit / max(hit + miss, 1.0)
    out["l2_requests_per_launch"] = (hit + miss) / launches
if A.ea:
    rd, _ = load(A.ea, "TCC_EA0_RDREQ_sum")
    dram, _ = load(A.ea, "TCC_EA0_RDREQ_DRAM_sum")
    out["ea_rdreq_per_launch"] = rd / launches
    out["ea_rdreq_dram_fraction"] = dram / max(rd, 1.0)
    out["mall_split_note"] = ("rocprofv3 on gfx950 lists no Infinity-Cache (MALL) hit/miss counter; "
                              "TCC_EA0_RDREQ_DRAM counts L2 read requests destined for the memory controller, "
                              "which fronts the MALL, so MALL hits and HBM reads are not separable by counters")
print(json.dumps(out, indent=1))
Path(A.out).parent.mkdir(exist_ok=True)
Path(A.out).write_text(json.dumps(out, indent=1))
