#!/bin/bash
# round 6 call h: GROUP_M sweep on the product GEMM shapes (automatic kernel choice)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for g in 4 16 32; do
  echo "== g8 (A) vs g$g (B)"
  timeout -k 10 300 python -u tools/lib_ab.py hyperscalees_t2i_amd/_build/libeggroll.so tools/_ab/g$g.so 0 > gpurun_out/r13h_g$g.log 2>&1 || { tail -20 gpurun_out/r13h_g$g.log; exit 1; }
  tail -1 gpurun_out/r13h_g$g.log
done
