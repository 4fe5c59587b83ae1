#!/bin/bash
# round 6 call b: MFMA shape probe (built on the box), new GPU tests, ES perturb member-split A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out tools/_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/_build/mfma_shape_probe tools/mfma_shape_probe.hip || exit 1
timeout -k 10 240 tools/_build/mfma_shape_probe 1024 4096 20 > gpurun_out/r13b_mfma_shape.jsonl 2>&1 || { cat gpurun_out/r13b_mfma_shape.jsonl; exit 1; }
cat gpurun_out/r13b_mfma_shape.jsonl
timeout -k 10 300 python -u tools/es_lib_ab.py tools/_ab/libeggroll_a.so hyperscalees_t2i_amd/_build/libeggroll.so > gpurun_out/r13b_es_ab.log 2>&1 || { tail -20 gpurun_out/r13b_es_ab.log; exit 1; }
tail -1 gpurun_out/r13b_es_ab.log | cut -c1-1500
timeout -k 10 600 python -u -m pytest tests/test_gpu_member_slices_fullsize.py "tests/test_gpu_kernels.py::test_forward_fp32_any_lora_rank" "tests/test_gpu_kernels.py::test_subpixel_upblock_matches_reference" tests/test_gpu_kernels.py -k "perturb or seeded or member_slices or any_lora_rank or upblock" -v -s --timeout 600 --timeout-method thread > gpurun_out/r13b_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|member-slices|passed|failed" gpurun_out/r13b_tests.log | cut -c1-300 | tail -40
exit $rc
