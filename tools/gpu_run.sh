#!/bin/bash
# One GPU call, steps chosen by name; each GPU step has its own time limit and the first failure ends
# the call (no retries).  Output under gpurun_out/<tag>_*.
#   usage: bash tools/gpu_run.sh <tag> <step> [<step> ...]
#   steps: pytest | pytest:<expr> (pytest -k expr) | smoke | bench | prof (rocprofv3 kernel trace of a
#          short bench + timed window) | probe:<script args...> (python tools/<script>, ',' for spaces)
#          | counters (rocprofv3 -L, the counter list)
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
say() { echo "[gpu_run $tag] $1 $(date +%T)"; }
for st in "$@"; do
  case "$st" in
    pytest)
      say pytest
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
          > gpurun_out/${tag}_pytest.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
      tail -2 gpurun_out/${tag}_pytest.log ;;
    pytest:*)
      say "$st"
      timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -rf --timeout 300 --timeout-method thread -k "${st#pytest:}" \
          > gpurun_out/${tag}_pytestk.log 2>&1 || { tail -40 gpurun_out/${tag}_pytestk.log; exit 1; }
      grep -E "PASS|FAIL|ERROR|fp32-parity|passed|failed" gpurun_out/${tag}_pytestk.log | cut -c1-600 ;;
    smoke)
      say smoke
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
          || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
      tail -1 gpurun_out/${tag}_smoke.log | cut -c1-300 ;;
    bench)
      say bench
      timeout -k 10 900 python -u bench.py --steps 10 --warmup 3 --aux-out gpurun_out/${tag}_bench_aux.json \
          > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
      cut -c1-600 gpurun_out/${tag}_bench.json ;;
    prof)
      say prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv \
          -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${tag}_prof.log 2>&1 \
          || { tail -30 gpurun_out/${tag}_prof.log; exit 1; }
      t=$(find gpurun_out/${tag}_prof -name "*kernel_trace.csv" | head -1)
      python3 tools/trace_window.py "$t" 45 > gpurun_out/${tag}_timed_window.txt && head -30 gpurun_out/${tag}_timed_window.txt | cut -c1-180 ;;
    probe:*)
      args=${st#probe:}; args=${args//,/ }
      say "probe $args"
      timeout -k 10 600 python -u tools/$args > gpurun_out/${tag}_probe_$(echo ${args%% *} | tr -c 'a-z0-9_\n' '_').log 2>&1 \
          || { tail -30 gpurun_out/${tag}_probe_*.log; exit 1; }
      tail -5 gpurun_out/${tag}_probe_$(echo ${args%% *} | tr -c 'a-z0-9_\n' '_').log | cut -c1-1500 ;;
    pmcgemm)
      # LoRA GEMM traffic over one epoch's launch mix x2: FETCH / WRITE bytes, L2 hit rate, and the EA read
      # requests split by destination (DRAM = memory controller, which fronts the Infinity Cache)
      i=0
      for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
        i=$((i+1)); say "pmc pass $i: $grp"
        timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_lora_gemm" -d gpurun_out/${tag}_pmc$i -o run \
            --output-format csv -- python3 tools/lora_epoch_driver.py 2 > gpurun_out/${tag}_pmc$i.log 2>&1 \
            || { tail -20 gpurun_out/${tag}_pmc$i.log; exit 1; }
      done
      python3 tools/pmc_summary.py gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 2 --l2 gpurun_out/${tag}_pmc3 \
          --ea gpurun_out/${tag}_pmc4 --out gpurun_out/${tag}_pmc_lora_gemm.json | tail -20 ;;
    pmc:*)
      # pmc:<kernel regex>:<tools script + args, ',' for spaces> -> FETCH / WRITE / L2 hit passes
      spec=${st#pmc:}; rx=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
      i=0
      for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
        i=$((i+1)); say "pmc $rx pass $i: $grp"
        timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$rx" -d gpurun_out/${tag}_kpmc$i -o run \
            --output-format csv -- python3 tools/$args > gpurun_out/${tag}_kpmc$i.log 2>&1 \
            || { tail -20 gpurun_out/${tag}_kpmc$i.log; exit 1; }
      done
      python3 tools/pmc_kernels.py gpurun_out/${tag}_kpmc1 gpurun_out/${tag}_kpmc2 gpurun_out/${tag}_kpmc3 | tail -30 ;;
    sq:*)
      # sq:<kernel regex>:<tools script + args> -> one SQ counter pass (instruction mix, wave cycles, waits)
      spec=${st#sq:}; rx=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
      say "sq $rx"
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES \
          SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-include-regex "$rx" -d gpurun_out/${tag}_sq \
          -o run --output-format csv -- python3 tools/$args > gpurun_out/${tag}_sq.log 2>&1 \
          || { tail -20 gpurun_out/${tag}_sq.log; exit 1; } ;;
    counters)
      say counters
      timeout -k 10 120 rocprofv3 -L > gpurun_out/${tag}_counters.txt 2>&1 || { tail -20 gpurun_out/${tag}_counters.txt; exit 1; }
      grep -o -E "TCC_[A-Z0-9_]*(DRAM|MALL|EA0_RD|EA_RD|BUBBLE|PROBE)[A-Z0-9_]*" gpurun_out/${tag}_counters.txt | sort -u | head -40 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
say done
