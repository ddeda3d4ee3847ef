#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.out 2> gpurun_out/pytest_gpu.err
rc=$?; echo "pytest rc=$rc" >&2; tail -40 gpurun_out/pytest_gpu.out >&2; tail -5 gpurun_out/pytest_gpu.err >&2
exit $rc
