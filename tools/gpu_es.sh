set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not lora" > gpurun_out/t_es.log 2>&1 || { tail -40 gpurun_out/t_es.log; exit 1; }
tail -2 gpurun_out/t_es.log
timeout -k 10 200 python -u tools/aux_probe.py
