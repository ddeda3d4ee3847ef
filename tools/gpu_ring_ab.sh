#!/bin/bash
# mesh_fine: the step record appended by k_mix2's reducing block (PUCFEM_RING_FOLD, default) vs k_stats_ring: bit
# comparison (fields + records), the small-mesh tests, then the rate per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in "PUCFEM_RING_FOLD=0" "PUCFEM_RING_FOLD=1"; do
  echo "$e"; env $e timeout -k 10 120 python tools/bitcmp_fine.py 1100 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_long.py \
  tests/test_gpu_boundary.py tests/test_gpu_parity.py 2>&1 | tail -3
for r in 1 2; do
  for e in "PUCFEM_RING_FOLD=0" "PUCFEM_RING_FOLD=1"; do
    echo "$e"; env $e timeout -k 10 120 python tools/fine_probe.py 3000 | cut -c1-80 || exit 1
  done
done
