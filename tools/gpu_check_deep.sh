#!/bin/bash
# deep-halo bisect probe (W=2/3, L3) -> the whole GPU suite -> W=8 L7 exchange counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-chk}
timeout -k 10 300 python -u tools/deep_probe.py 3 3 color > gpurun_out/${TAG}_deep_probe.txt 2>&1; rc=$?
cat gpurun_out/${TAG}_deep_probe.txt >&2; [ $rc -ne 0 ] && exit $rc
TAG=$TAG bash tools/gpu_full.sh
