# rocprofv3 kernel trace of one bench epoch of a workload; keeps only the summaries (the trace CSV is large)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=$1; wl=$2
timeout -k 10 800 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 -u bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { tail -30 gpurun_out/${tag}_prof.log; exit 1; }
t=$(find gpurun_out/${tag}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$t" 45 > gpurun_out/${tag}_timed_window.txt && rm -f "$t" && head -40 gpurun_out/${tag}_timed_window.txt | cut -c1-200
