#!/bin/bash
# k_mdot2 on virtual blocks (PUCFEM_FIT_GRID, default on) vs the plain grid: bit comparison, then driver-command A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in "PUCFEM_FIT_GRID=1" "PUCFEM_FIT_GRID=0"; do
  echo "$e"; env $e timeout -k 10 300 python tools/bitcmp.py 7 130 || exit 1
done
tools/gpu_env_ab.sh "${1:-vblocks}" "" "PUCFEM_FIT_GRID=0" "" "PUCFEM_FIT_GRID=0"
