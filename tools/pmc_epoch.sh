#!/bin/bash
# Kernel trace + PMC passes over one full Sana ES epoch (tools/epoch_driver.py), each pass its own run
# (rocprofv3 does not split counters).  Summary: python tools/pmc_epoch_summary.py <tag>.
#   usage: bash tools/pmc_epoch.sh <tag>
set -o pipefail
tag=${1:-pmc_epoch}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # run <pass> <rocprofv3 args...>
  local p=$1; shift
  echo "[pmc_epoch] $p $(date +%T)"
  timeout -s KILL 300 rocprofv3 "$@" -d gpurun_out/${tag}_$p -o run --output-format csv \
      -- python3 -u tools/epoch_driver.py > gpurun_out/${tag}_$p.log 2>&1 || { tail -5 gpurun_out/${tag}_$p.log; exit 1; }
}
run tr --kernel-trace
run p1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run p2 --pmc FETCH_SIZE GRBM_GUI_ACTIVE
run p3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
echo ok
