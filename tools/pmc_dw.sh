#!/bin/bash
# PMC passes + one kernel trace on the depthwise conv at its product shapes (tools/dw_driver.py); each
# pass its own run (rocprofv3 does not split counters).  Summary: tools/pmc_dw_summary.py <tag>.
#   usage: bash tools/pmc_dw.sh <tag>
set -o pipefail
tag=${1:-pmc_dw}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # run <pass> <rocprofv3 args...>
  local p=$1; shift
  echo "[pmc_dw] $p $(date +%T)"
  timeout -s KILL 90 rocprofv3 "$@" --kernel-include-regex "k_dwconv" -d gpurun_out/${tag}_$p -o run \
      --output-format csv -- python3 tools/dw_driver.py 3 > gpurun_out/${tag}_$p.log 2>&1 || { tail -5 gpurun_out/${tag}_$p.log; exit 1; }
}
run tr --kernel-trace
run p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE
run p2 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE
run p3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE
run p4 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
echo ok
