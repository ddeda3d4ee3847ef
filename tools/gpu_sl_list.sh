#!/bin/bash
# The semilagrangian second pass as one numbered list (PUCFEM_SL_WAVE=2, default) against k_sl_slow (0) and
# k_sl_wave (1): locator tests, bit comparison of production steps, then alternating driver-command benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sl_list}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "semilagrange or mixing" > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -3 "$OUT/pytest.out"
for m in 2 0; do
  PUCFEM_SL_WAVE=$m timeout -k 10 300 python tools/bitcmp.py 7 30 || exit 1
done
BARGS="--warmup 5 --steps 20" tools/gpu_env_ab.sh "$TAG" "" "PUCFEM_SL_WAVE=0" "" "PUCFEM_SL_WAVE=0" "PUCFEM_SL_WAVE=1"
