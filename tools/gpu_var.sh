#!/bin/bash
# VAR model-level GPU call: the VAR parity tests, then the configs[0] bench line (VAR-d16, pop 4).
# usage: bash tools/gpu_var.sh <tag> [--bench]
set -o pipefail
tag=${1:-var}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "[gpu_var] pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_var_model.py -m gpu -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
grep -E "passed|failed|var parity" gpurun_out/${tag}_pytest.log
if [ "$2" = "--bench" ]; then
    echo "[gpu_var] bench $(date +%T)"
    timeout -k 10 900 python -u bench.py --workload var_d16 --steps 5 --warmup 2 \
        > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
    cut -c1-600 gpurun_out/${tag}_bench.json
fi
echo "[gpu_var] done $(date +%T)"
