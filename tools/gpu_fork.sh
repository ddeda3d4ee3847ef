#!/bin/bash
# Small meshes: the final-divergence record on a forked branch of the captured step (PUCFEM_GRAPH_FORK, default) vs one
# chain: bit comparison (fields + records), the small-mesh tests, then the rate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in "PUCFEM_GRAPH_FORK=0" "PUCFEM_GRAPH_FORK=1"; do
  echo "$e"; env $e timeout -k 10 120 python tools/bitcmp_fine.py 1100 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_boundary.py \
  tests/test_gpu_long.py 2>&1 | tail -2
for r in 1 2 3; do
  for e in "PUCFEM_GRAPH_FORK=0" "PUCFEM_GRAPH_FORK=1"; do
    echo "$e"; env $e timeout -k 10 120 python tools/fine_probe.py 3000 | cut -c1-80 || exit 1
  done
done
