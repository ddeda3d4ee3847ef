#!/bin/bash
# The dye tail's semi-Lagrangian part released after the next viscous pair's first SELL launch (PUCFEM_DYE_GATE=3) or
# after its face kernel (4), against the end of the step (0): bit comparison, then alternating driver-command benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in "PUCFEM_DYE_GATE=0" "PUCFEM_DYE_GATE=3"; do
  echo "$e"; env $e timeout -k 10 300 python tools/bitcmp.py 7 40 || exit 1
done
tools/gpu_env_ab.sh "${1:-gate34}" "" "PUCFEM_DYE_GATE=3" "PUCFEM_DYE_GATE=4" "" "PUCFEM_DYE_GATE=3" "PUCFEM_DYE_GATE=4"
