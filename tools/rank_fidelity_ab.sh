#!/bin/bash
# tests/test_gpu_parity_fp32.py::test_rank_fidelity_over_seeds with forward_fp32's LoRA term on
# eggroll_lora_delta_f32 vs torch bmm (lora.FP32_DELTA_KERNEL), over two seed sets; reports in gpurun_out/<tag>.log
set -o pipefail
tag=${1:-rank_ab}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for seeds in ${RANK_AB_SEEDS:-5:17 17:29}; do
  for kern in 1 0; do
    echo "== seeds $seeds kernel $kern" >> gpurun_out/$tag.log
    EGG_RANK_SEEDS=$seeds timeout -k 10 300 python3 -u -c "
import sys, pytest
import hyperscalees_t2i_amd.lora as L
L.FP32_DELTA_KERNEL = bool($kern)
sys.exit(pytest.main(['-q', '-s', '-p', 'no:cacheprovider', 'tests/test_gpu_parity_fp32.py::test_rank_fidelity_over_seeds']))
" 2>&1 | grep -E "rank fidelity over seeds|passed|failed" >> gpurun_out/$tag.log
    rc=$?
    [ $rc -le 1 ] || exit $rc
  done
done
echo ok
