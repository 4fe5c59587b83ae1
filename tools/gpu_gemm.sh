set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "lora" --timeout 120 --timeout-method thread > gpurun_out/t_lora.log 2>&1 || { tail -40 gpurun_out/t_lora.log; exit 1; }
tail -2 gpurun_out/t_lora.log
timeout -k 10 200 python -u tools/gemm_probe.py 3
