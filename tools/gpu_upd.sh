#!/bin/bash
# Update-kernel load-group A/B (EGG_UPD_GROUP 8 / 16 / 32): update parity tests on each library, then
# tools/aux_probe.py per library, twice, each step under its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=$PWD/hyperscalees_t2i_amd/_build
for g in 16 32; do
  EGGROLL_LIB=$B/libeggroll_u$g.so timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "update or full_size" --timeout 120 --timeout-method thread > gpurun_out/upd_t$g.log 2>&1 || { tail -20 gpurun_out/upd_t$g.log; exit 1; }
  tail -1 gpurun_out/upd_t$g.log
done
for rep in 1 2; do
  for g in 8 16 32; do
    lib=$B/libeggroll_u$g.so; [ $g = 8 ] && lib=$B/libeggroll.so
    echo "u$g" >> gpurun_out/upd_probe.log
    EGGROLL_LIB=$lib timeout -k 10 120 python -u tools/aux_probe.py >> gpurun_out/upd_probe.log 2>&1 || { tail -20 gpurun_out/upd_probe.log; exit 1; }
  done
done
python - <<'PY'
import json
cur = None
for line in open("gpurun_out/upd_probe.log"):
    line = line.strip()
    if line.startswith("u") and len(line) < 4:
        cur = line; continue
    if line.startswith("{"):
        d = json.loads(line); u = d["update"]
        print(cur, "pop", d.get("sizes", {}).get("pop"), "update us", round(u["us"], 2), "GBps", round(u["GBps"]))
PY
