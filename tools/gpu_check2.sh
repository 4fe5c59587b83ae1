#!/bin/bash
# GPU validation pass (run on the box from the repo root): full `pytest -m gpu` (no -x: every
# failure is listed), smoke, a short bench.  Each step has its own time limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-chk}
mkdir -p gpurun_out
echo "[chk] pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -15 gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[chk] smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
echo "[chk] bench $(date +%T)"
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --aux-out gpurun_out/${tag}_bench_aux.json \
    > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-600 gpurun_out/${tag}_bench.json
exit $rc
