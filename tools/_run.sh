cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "320_tile" --timeout 120 --timeout-method thread > gpurun_out/r04f_pytest.log 2>&1 || { tail -30 gpurun_out/r04f_pytest.log; exit 1; }
tail -1 gpurun_out/r04f_pytest.log
timeout -k 10 300 python -u tools/stamp_probe.py gemm > gpurun_out/r04f_stamps.txt 2>&1 || { tail -20 gpurun_out/r04f_stamps.txt; exit 1; }
grep kernel gpurun_out/r04f_stamps.txt | cut -c1-400
timeout -k 10 300 python -u tools/gemm10_probe.py 5 gpurun_out/r04f_gemm10.json 2>&1 | grep M
