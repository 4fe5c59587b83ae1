#!/bin/bash
# Round-evidence GPU call: pytest -m gpu -> smoke -> bench (driver's default line) -> rocprofv3
# kernel-trace/stats of a short bench with the timed-window breakdown.  Each GPU step has its own
# limit; the first failure ends the call.   usage: bash tools/gpu_round2.sh <tag>
set -o pipefail
tag=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { echo "[gpu_round2] $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
step bench
timeout -k 10 900 python -u bench.py --steps 10 --warmup 3 --aux-out gpurun_out/${tag}_bench_aux.json \
    > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-700 gpurun_out/${tag}_bench.json
step rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv \
    -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${tag}_prof.log 2>&1 \
    || { tail -30 gpurun_out/${tag}_prof.log; exit 1; }
t=$(find gpurun_out/${tag}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$t" 45 > gpurun_out/${tag}_timed_window.txt && head -50 gpurun_out/${tag}_timed_window.txt | cut -c1-200
step done
