#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-cgcg}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_scale_parity.py tests/test_gpu_configs.py tests/test_gpu_rccl.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "single_reduction or multirank or partitioned or rank or rccl" > $OUT/pytest.txt 2>&1; rc=$?; echo "pytest rc=$rc" >&2; tail -n 4 $OUT/pytest.txt >&2; [ $rc -ne 0 ] && exit $rc
PUCFEM_CGCG=0 timeout -k 10 300 python -u tools/comm_probe.py 5 8 6 > $OUT/comm_probe_l5_w8_standard.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/comm_probe.py 5 8 6 > $OUT/comm_probe_l5_w8_cgcg.txt 2>&1 || exit 1
tail -n 2 $OUT/comm_probe_l5_w8_*.txt >&2
