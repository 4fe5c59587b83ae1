#!/bin/bash
# 8 identical member-eval processes sharing cuda:0, each checking its own repeats bitwise
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export OMP_NUM_THREADS=2
pids=()
for i in 0 1 2 3 4 5 6 7; do
  timeout -k 20 700 python -u tools/contention_determinism_probe.py self p$i 6 > gpurun_out/r13u_self_p$i.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
grep -h "rows_differ" gpurun_out/r13u_self_p*.log | grep -v '"rows_differ": \[\], "img_differ": \[\], "lib_differ": \[\]' | head -20
grep -c rows_differ gpurun_out/r13u_self_p*.log
exit $rc
