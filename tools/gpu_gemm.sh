#!/bin/bash
# LoRA GEMM check: its parity tests, then the interleaved A/B probe vs hipBLASLt.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "lora" --timeout 120 --timeout-method thread > gpurun_out/t_lora.log 2>&1 || { tail -40 gpurun_out/t_lora.log; exit 1; }
tail -2 gpurun_out/t_lora.log
timeout -k 10 300 python -u tools/gemm_probe.py ${1:-3}
