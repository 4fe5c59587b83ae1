cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -q -x -rf --timeout 240 --timeout-method thread > gpurun_out/r02b_pytest.log 2>&1; rc=$?; tail -12 gpurun_out/r02b_pytest.log; \
[ $rc -le 1 ] && timeout -k 10 300 python -u tools/aux_probe.py > gpurun_out/r02b_aux.log 2>&1; cat gpurun_out/r02b_aux.log | cut -c1-900; exit $rc
