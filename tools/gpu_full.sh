#!/bin/bash
# The whole GPU suite (one process), then the W=8 exchange counts at L7
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread --durations=25 \
  > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >&2; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${T}_pytest_gpu.txt | tail -8 >&2
grep -E "W=8|L6 W=8|L5 W=8" gpurun_out/${T}_pytest_gpu.txt | tail -20 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -u tools/comm_probe.py 7 8 5 > gpurun_out/${T}_comm_probe_l7_w8.txt 2>&1
rc=$?; echo "probe rc=$rc" >&2; tail -4 gpurun_out/${T}_comm_probe_l7_w8.txt >&2
exit $rc
