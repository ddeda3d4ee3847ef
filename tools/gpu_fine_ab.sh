#!/bin/bash
# mesh_fine small-mesh path: bit comparison against libpucfem.prev.so (the previous commit) and the knob, the graph
# tests, then the rate (tools/fine_probe.py) per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in "PUCFEM_LIB_VARIANT=prev" "PUCFEM_DENSE_BC=0" "PUCFEM_DENSE_BC=1"; do
  echo "$e"; env $e timeout -k 10 120 python tools/bitcmp_fine.py 300 || exit 1
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_long.py \
  -k "graph_of_k or mesh_fine" 2>&1 | tail -3
for r in 1 2; do
  for e in "PUCFEM_LIB_VARIANT=prev" "PUCFEM_DENSE_BC=0" "PUCFEM_DENSE_BC=1"; do
    echo "$e"; env $e timeout -k 10 120 python tools/fine_probe.py 3000 | cut -c1-80 || exit 1
  done
done
