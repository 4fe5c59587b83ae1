set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --aux-out gpurun_out/bench_aux.json > gpurun_out/bench.out 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.out; grep "bench +" gpurun_out/bench.err | grep -v heartbeat
MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_nonaive.out 2> gpurun_out/bench_nonaive.err || { echo "bench2 rc=$?"; tail -30 gpurun_out/bench_nonaive.err; exit 1; }
cat gpurun_out/bench_nonaive.out | cut -c1-300; grep "bench +" gpurun_out/bench_nonaive.err | grep -v heartbeat
