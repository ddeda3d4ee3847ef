#!/bin/bash
# Small meshes: the first projection with its BCs in one launch (k_grad_proj_bc; PUCFEM_DENSE_BC=0 turns both dense
# folds off): bit comparison (fields + records), the production / boundary / small-mesh tests, then the rate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in "PUCFEM_DENSE_BC=0" "PUCFEM_DENSE_BC=1"; do
  echo "$e"; env $e timeout -k 10 120 python tools/bitcmp_fine.py 1100 || exit 1
done
timeout -k 10 700 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_production.py \
  tests/test_gpu_boundary.py tests/test_gpu_long.py > gpurun_out/gpbc_pytest.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpbc_pytest.txt | tail -30; [ $rc -ne 0 ] && { tail -40 gpurun_out/gpbc_pytest.txt; exit $rc; }
for r in 1 2; do
  for e in "PUCFEM_DENSE_BC=0" "PUCFEM_DENSE_BC=1"; do
    echo "$e"; env $e timeout -k 10 120 python tools/fine_probe.py 3000 | cut -c1-80 || exit 1
  done
done
