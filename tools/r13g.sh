#!/bin/bash
# round 6 call g: linear-attention fold A/B + tests, up-block conv stamps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "linear_attention" -q --timeout 120 --timeout-method thread > gpurun_out/r13g_la_tests.log 2>&1 || { tail -30 gpurun_out/r13g_la_tests.log; exit 1; }
tail -2 gpurun_out/r13g_la_tests.log
timeout -k 10 300 python -u tools/ops_lib_ab.py tools/_ab/libeggroll_a.so hyperscalees_t2i_amd/_build/libeggroll.so > gpurun_out/r13g_ops_ab.log 2>&1 || { tail -20 gpurun_out/r13g_ops_ab.log; exit 1; }
grep -i "linear" gpurun_out/r13g_ops_ab.log | tail -6 | cut -c1-400
timeout -k 10 300 python -u tools/stamp_probe.py up > gpurun_out/r13f_stamps.txt 2>&1 || { tail -20 gpurun_out/r13f_stamps.txt; exit 1; }
grep kernel gpurun_out/r13f_stamps.txt
