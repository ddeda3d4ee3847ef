#!/bin/bash
# lmax per level (device vs host) at L5/L7 and the L7 per-step margin test with device / host lmax
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-lmax}; mkdir -p "$OUT"
timeout -k 10 300 python -u tools/lmax_probe.py 5 7 > "$OUT/lmax_probe.txt" 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale_parity.py -k per_step -x -v -rP --timeout 380 --timeout-method thread > "$OUT/per_step_dev.txt" 2>&1 || exit $?
PUCFEM_LMAX_HOST=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_scale_parity.py -k per_step -x -v -rP --timeout 380 --timeout-method thread > "$OUT/per_step_host.txt" 2>&1 || exit $?
