set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "lora or conv or resblock or upblock" --timeout 120 --timeout-method thread > gpurun_out/t_kern.log 2>&1 || { tail -30 gpurun_out/t_kern.log; exit 1; }
tail -1 gpurun_out/t_kern.log
timeout -k 10 200 python -u tools/stamp_probe.py && timeout -k 10 300 python -u tools/gemm_probe.py 3 && timeout -k 10 300 python -u tools/conv_gemm_probe.py
