#!/bin/bash
# A/B of the update kernel's rank-1 load grouping (EGG_UPD_PGRP1 = 8 / 16): builds each variant
# into its own library (EGGROLL_LIB) and profiles tools/es_kernel_probe.py with rocprofv3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for g in 8 16; do
  d=/tmp/egg_pg$g; mkdir -p $d
  for s in eggroll_es eggroll_lora eggroll_model; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -DEGG_UPD_PGRP1=$g -Iinclude \
      hyperscalees_t2i_amd/csrc/$s.hip -o $d/$s.o || exit 1
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/*.o -o $d/libeggroll.so || exit 1
  EGGROLL_LIB=$d/libeggroll.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/upd_pg$g -o run \
     --output-format csv -- python3 -u tools/es_kernel_probe.py 20 > gpurun_out/upd_pg$g.log 2>&1 || { tail gpurun_out/upd_pg$g.log; exit 1; }
  t=$(find gpurun_out/upd_pg$g -name "*kernel_trace.csv" | head -1)
  echo "PGRP1=$g"; python3 tools/es_prof_summary.py "$t" 20
done
