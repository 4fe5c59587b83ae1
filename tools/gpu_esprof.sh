#!/bin/bash
# rocprofv3 kernel-trace stats of tools/es_kernel_probe.py (ES arithmetic kernels only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-es}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv \
    -- python3 -u tools/es_kernel_probe.py 20 > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
f=$(find gpurun_out/${tag}_prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -30
t=$(find gpurun_out/${tag}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/es_prof_summary.py "$t" 20
