#!/bin/bash
# The dye stream on k of every 8 CUs (PUCFEM_SL_CUMASK), with the tail released at the end of the step or at the next
# step's first V-cycle (PUCFEM_DYE_GATE=1): alternating driver-command benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_env_ab.sh "${1:-cumask}" "" "PUCFEM_DYE_GATE=1 PUCFEM_SL_CUMASK=6" "PUCFEM_DYE_GATE=1 PUCFEM_SL_CUMASK=4" \
  "PUCFEM_SL_CUMASK=6" "" "PUCFEM_DYE_GATE=1 PUCFEM_SL_CUMASK=6" "PUCFEM_DYE_GATE=1 PUCFEM_SL_CUMASK=4" "PUCFEM_SL_CUMASK=6"
