#!/bin/bash
# Kernel trace + one SQ counter pass over the seeded ES kernels (tools/es_valu_driver.py), each its own run.
# Summary: python tools/es_valu_summary.py gpurun_out/<tag>_p1 gpurun_out/<tag>_tr
#   usage: bash tools/pmc_es_valu.sh <tag>
set -o pipefail
tag=${1:-es_valu}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rx="k_perturb|k_update"
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$rx" -d gpurun_out/${tag}_tr -o run \
    --output-format csv -- python3 -u tools/es_valu_driver.py > gpurun_out/${tag}_tr.log 2>&1 || { tail -5 gpurun_out/${tag}_tr.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$rx" -d gpurun_out/${tag}_p1 -o run \
    --output-format csv -- python3 -u tools/es_valu_driver.py > gpurun_out/${tag}_p1.log 2>&1 || { tail -5 gpurun_out/${tag}_p1.log; exit 1; }
echo ok
