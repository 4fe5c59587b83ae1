#!/bin/bash
# One round-evidence GPU call (run on the GPU box from the repo root):
#   pytest -m gpu -> smoke -> bench.py (the driver's line) -> rocprofv3 kernel-trace/stats of a short
#   bench -> two PMC passes (FETCH_SIZE, WRITE_SIZE) over the LoRA GEMM launch mix.
# Every GPU step has its own time limit; the first failure ends the call.
# usage: bash tools/gpu_round.sh <tag>     (outputs under gpurun_out/<tag>_*)
set -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { echo "[gpu_round] $1 $(date +%T)"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
step bench
timeout -k 10 600 python -u bench.py --aux-out gpurun_out/${tag}_bench_aux.json > gpurun_out/${tag}_bench.json \
    2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${tag}_bench.json
step rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv \
    -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${tag}_prof.log 2>&1 \
    || { tail -30 gpurun_out/${tag}_prof.log; exit 1; }
tail -1 gpurun_out/${tag}_prof.log | cut -c1-300
for c in FETCH_SIZE WRITE_SIZE; do
  step "pmc $c"
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_lora_gemm" -d gpurun_out/${tag}_pmc_$c -o run \
      --output-format csv -- python3 tools/lora_epoch_driver.py 2 > gpurun_out/${tag}_pmc_$c.log 2>&1 \
      || { tail -20 gpurun_out/${tag}_pmc_$c.log; exit 1; }
done
step done
