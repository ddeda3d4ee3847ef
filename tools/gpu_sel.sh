#!/bin/bash
# Selected GPU tests: PYTEST_SEL (pytest node ids / -k expression), output tag TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-sel}
timeout -k 10 ${TLIM:-1100} python -u -m pytest -x -v -s --timeout 1100 --timeout-method thread ${PYTEST_SEL} > gpurun_out/${TAG}.out 2> gpurun_out/${TAG}.err
rc=$?; echo "pytest rc=$rc" >&2; grep -E "PASSED|FAILED|ERROR|passed|failed|W=8|step" gpurun_out/${TAG}.out | tail -60 >&2
exit $rc
