#!/bin/bash
# The main stream at the highest priority and the dye stream at the lowest (PUCFEM_STREAM_PRIO=1) vs default priorities:
# bit comparison, then alternating driver-command benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in "PUCFEM_STREAM_PRIO=0" "PUCFEM_STREAM_PRIO=1"; do
  echo "$e"; env $e timeout -k 10 300 python tools/bitcmp.py 7 40 || exit 1
done
tools/gpu_env_ab.sh "${1:-prio}" "" "PUCFEM_STREAM_PRIO=1" "" "PUCFEM_STREAM_PRIO=1" "" "PUCFEM_STREAM_PRIO=1"
