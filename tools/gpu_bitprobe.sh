#!/bin/bash
# Which setting changes the long / tight L7 trajectories: bitcmp hashes per environment setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for args in "7 130" "7 40 1e-12"; do
  for e in "PUCFEM_SL_WAVE=2" "PUCFEM_SL_WAVE=0" "PUCFEM_SL_WAVE=1" "PUCFEM_GP_GATE=0" "PUCFEM_FIT_GRID=0"; do
    echo "$e $args"; env $e timeout -k 10 300 python tools/bitcmp.py $args || exit 1
  done
done
BARGS="--warmup 5 --steps 20" tools/gpu_env_ab.sh "${1:-bitprobe}" "" "PUCFEM_FIT_GRID=0" "PUCFEM_DYE_SL_FIRST=1" "" "PUCFEM_FIT_GRID=0" "PUCFEM_DYE_SL_FIRST=1"
