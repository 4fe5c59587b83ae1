#!/bin/bash
# Round-evidence GPU call: pytest -m gpu -> smoke -> bench (driver-like line) -> rocprofv3
# kernel-trace/stats of a short bench + timed window -> PMC FETCH_SIZE / WRITE_SIZE passes over the
# LoRA GEMM launch mix (summarised locally by tools/pmc_summary.py) -> SQ counter passes (tile 8).
# Each GPU step has its own limit; the first failure ends the call.  usage: bash tools/gpu_round3.sh <tag>
set -o pipefail
tag=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { echo "[gpu_round3] $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log | cut -c1-200
step bench
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --aux-out gpurun_out/${tag}_bench_aux.json \
    > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${tag}_bench.json
step rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv \
    -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${tag}_prof.log 2>&1 \
    || { tail -30 gpurun_out/${tag}_prof.log; exit 1; }
t=$(find gpurun_out/${tag}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$t" 45 > gpurun_out/${tag}_timed_window.txt && head -6 gpurun_out/${tag}_timed_window.txt | cut -c1-160
for c in FETCH_SIZE WRITE_SIZE; do
  step "pmc $c"
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_lora_gemm" -d gpurun_out/${tag}_pmc_$c -o run \
      --output-format csv -- python3 tools/lora_epoch_driver.py 2 > gpurun_out/${tag}_pmc_$c.log 2>&1 \
      || { tail -20 gpurun_out/${tag}_pmc_$c.log; exit 1; }
done
step "pmc sq"
timeout -k 10 300 bash tools/pmc_gemm.sh 8 > gpurun_out/${tag}_pmc_sq.txt 2>&1 || { tail -20 gpurun_out/${tag}_pmc_sq.txt; exit 1; }
cat gpurun_out/${tag}_pmc_sq.txt
step done
