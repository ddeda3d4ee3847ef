#!/bin/bash
# The gated projection armed only at likely-converging reads: bit comparison against the known hash, the PCG / production
# tests, then the driver command (launches per step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/bitcmp.py 7 40 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_production.py \
  tests/test_gpu_boundary.py 2>&1 | tail -2
tools/gpu_env_ab.sh "${1:-arm}" "" "PUCFEM_GP_GATE=0" "" "PUCFEM_GP_GATE=0"
for i in 0 1 2 3; do python -c "import json; r=json.loads(open('gpurun_out/${1:-arm}/bench$i.out').read().strip().splitlines()[-1]); print($i, r['value'], r['launches_per_step'])"; done
