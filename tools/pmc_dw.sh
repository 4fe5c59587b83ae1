#!/bin/bash
# PMC passes on the depthwise conv (tools/dw_driver.py): issue mix / busy / wait counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY \
  --kernel-include-regex "k_dwconv" -d gpurun_out/pmc_dw1 -o run --output-format csv -- python3 tools/dw_driver.py 2 > gpurun_out/pmc_dw1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_dwconv" -d gpurun_out/pmc_dw2 -o run --output-format csv -- python3 tools/dw_driver.py 2 > gpurun_out/pmc_dw2.log 2>&1 || exit 1
echo ok
