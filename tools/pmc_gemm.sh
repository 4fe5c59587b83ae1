#!/bin/bash
# SQ counter passes over the 8-phase LoRA GEMM (one counter group per pass, kernel-trace only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tile=${1:-9}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "k_lora_gemm" -d gpurun_out/pmcg_${tile}_$i -o run --output-format csv -- python3 tools/gemm_one.py $tile 3 > gpurun_out/pmcg_${tile}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcg_${tile}_$i.log; exit 1; }
done
python3 - "$tile" <<'PY'
import csv, sys, glob, collections
tile = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/pmcg_{tile}_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:32s} n={len(v)} mean={sum(v)/len(v):.4g}")
PY
