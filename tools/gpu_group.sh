#!/bin/bash
# Rasterisation-group A/B of the LoRA GEMM: one process per prebuilt library (EGG_GROUP_M variants,
# hyperscalees_t2i_amd/_build/libeggroll_g*.so) plus the default build, each under its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=hyperscalees_t2i_amd/_build
for rep in 1 2; do
  for g in 8 1 2 4 16; do
    lib=$B/libeggroll_g$g.so; [ $g = 8 ] && lib=$B/libeggroll.so
    EGGROLL_LIB=$PWD/$lib timeout -k 10 120 python -u tools/group_probe.py g$g >> gpurun_out/group_probe.log 2>&1 || { tail -20 gpurun_out/group_probe.log; exit 1; }
    tail -1 gpurun_out/group_probe.log
  done
done
