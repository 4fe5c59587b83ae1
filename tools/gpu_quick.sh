#!/bin/bash
# Kernel-level GPU check: GPU kernel/engine tests, HBM-kernel roofline probe, GEMM/projection probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { tail -40 gpurun_out/q_tests.log; exit 1; }
tail -2 gpurun_out/q_tests.log
timeout -k 10 200 python -u tools/aux_probe.py || exit 1
timeout -k 10 300 python -u tools/gemm_probe.py 2 || exit 1
