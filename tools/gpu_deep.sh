#!/bin/bash
# SL second pass + multi-rank checks of the deep halos: SL locator tests, the partitioned-run tests (LocalComm),
# the W=8 exchange counts at L7 (tools/comm_probe.py), then the W=8 value tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-deep}
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_gpu_parity.py -k "semilagrange or knn or step_pairs or single_reduction" \
  > gpurun_out/${T}_sl.out 2>&1
rc=$?; echo "sl rc=$rc" >&2; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/${T}_sl.out | tail -20 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_gpu_multirank.py \
  "tests/test_gpu_scale_parity.py::test_production_partitioned_L3_vs_oracle" tests/test_gpu_rccl.py \
  > gpurun_out/${T}_multirank.out 2>&1
rc=$?; echo "multirank rc=$rc" >&2; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/${T}_multirank.out | tail -20 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/comm_probe.py 7 8 5 > gpurun_out/${T}_comm_probe_l7_w8.txt 2>&1
rc=$?; echo "probe rc=$rc" >&2; tail -14 gpurun_out/${T}_comm_probe_l7_w8.txt >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_multirank8.py \
  > gpurun_out/${T}_w8.out 2>&1
rc=$?; echo "w8 rc=$rc" >&2; grep -E "PASSED|FAILED|ERROR|passed|failed|W=8|Error" gpurun_out/${T}_w8.out | tail -40 >&2
exit $rc
