#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (run on the GPU box from the repo root).
# usage: bash tools/prof.sh <outdir-name> [bench args...]
set -o pipefail
name=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/$name -o run --output-format csv -- python3 -u bench.py "$@" > gpurun_out/$name.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/$name.log
exit $rc
