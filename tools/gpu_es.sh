#!/bin/bash
# ES-kernel GPU check: non-LoRA GPU kernel/engine tests, the HBM-kernel roofline probe, and a
# rocprofv3 kernel-trace/stats pass over the same probe (per-kernel durations to cross-check it).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not lora" > gpurun_out/t_es.log 2>&1 || { tail -40 gpurun_out/t_es.log; exit 1; }
tail -2 gpurun_out/t_es.log
timeout -k 10 200 python -u tools/aux_probe.py > gpurun_out/aux_probe.log 2>&1 || { tail -20 gpurun_out/aux_probe.log; exit 1; }
cat gpurun_out/aux_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/aux_prof -o run --output-format csv \
    -- python3 -u tools/aux_probe.py > gpurun_out/aux_prof.log 2>&1 || { tail -20 gpurun_out/aux_prof.log; exit 1; }
find gpurun_out/aux_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/aux_kernel_stats.csv
