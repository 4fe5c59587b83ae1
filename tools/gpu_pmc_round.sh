set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=r02c
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_lora_gemm" -d gpurun_out/${tag}_pmc_$c -o run \
      --output-format csv -- python3 tools/lora_epoch_driver.py 2 > gpurun_out/${tag}_pmc_$c.log 2>&1 \
      || { tail -20 gpurun_out/${tag}_pmc_$c.log; exit 1; }
done
timeout -k 10 300 bash tools/pmc_gemm.sh 8 > gpurun_out/${tag}_pmc_sq.txt 2>&1 || { tail -20 gpurun_out/${tag}_pmc_sq.txt; exit 1; }
cat gpurun_out/${tag}_pmc_sq.txt
