#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/deep_probe.py 3 2 food > gpurun_out/deep_probe_food.txt 2>&1; rc=$?
cat gpurun_out/deep_probe_food.txt >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/deep_probe.py 3 3 color > gpurun_out/deep_probe_color.txt 2>&1; rc=$?
cat gpurun_out/deep_probe_color.txt >&2; [ $rc -ne 0 ] && exit $rc
TAG=r13c bash tools/gpu_full.sh
