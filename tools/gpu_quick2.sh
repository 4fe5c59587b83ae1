#!/bin/bash
# Focused GPU check: selected -m gpu test files, an optional probe, a short bench.
# usage: bash tools/gpu_quick2.sh <tag> "<test files>" [probe.py] [--bench]
set -o pipefail
tag=$1; files=$2; probe=$3; bench=$4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "[quick2] pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest $files -m gpu -q -rf -s --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/${tag}_pytest.log | head -30; tail -5 gpurun_out/${tag}_pytest.log; exit 1; }
grep -E "passed|failed|\[clip tower|\[var parity" gpurun_out/${tag}_pytest.log | tail -8
if [ -n "$probe" ] && [ "$probe" != "-" ]; then
    echo "[quick2] probe $(date +%T)"
    timeout -k 10 600 python -u $probe > gpurun_out/${tag}_probe.json 2> gpurun_out/${tag}_probe.err \
        || { tail -20 gpurun_out/${tag}_probe.err; exit 1; }
    cat gpurun_out/${tag}_probe.json
fi
if [ "$bench" = "--bench" ]; then
    echo "[quick2] bench $(date +%T)"
    timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --aux-out gpurun_out/${tag}_bench_aux.json \
        > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
    cut -c1-400 gpurun_out/${tag}_bench.json
    python -c "import json;l=json.load(open('gpurun_out/${tag}_bench_aux.json'))['line'];print(l['phases_ms'])"
fi
echo "[quick2] done $(date +%T)"
