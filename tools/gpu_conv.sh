#!/bin/bash
# Implicit-GEMM conv check: its parity tests, then the throughput probe vs MIOpen.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or resblock or upblock" > gpurun_out/t_conv.log 2>&1 || { tail -40 gpurun_out/t_conv.log; exit 1; }
tail -2 gpurun_out/t_conv.log
timeout -k 10 300 python -u tools/conv_gemm_probe.py > gpurun_out/conv_probe.log 2>&1 || { tail -20 gpurun_out/conv_probe.log; exit 1; }
cat gpurun_out/conv_probe.log
