#!/bin/bash
# HBM traffic of the population LoRA GEMM: two separate rocprofv3 --pmc passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950), kernel-trace only, no sys/runtime traces.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex "k_lora_gemm" -d gpurun_out/pmc_$c -o run \
      --output-format csv -- python3 tools/lora_epoch_driver.py 2 > gpurun_out/pmc_$c.log 2>&1 || exit $?
done
echo pmc-done
