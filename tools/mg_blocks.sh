#!/bin/bash
# V-cycle grid-size sweep (PUCFEM_MG_BLOCKS) at L7, fp32 cycle
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for nb in 1024 2048 4096 8192 16384; do
  PUCFEM_MG_BLOCKS=$nb timeout -k 10 300 python tools/mg_sweep.py 7 single > gpurun_out/mgb_$nb.out 2>&1 || exit $?
  echo "nb=$nb $(cat gpurun_out/mgb_$nb.out)"
done
