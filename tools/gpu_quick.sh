#!/bin/bash
# Quick GPU iteration: full GPU parity suite, then the L7 bench line without the CPU legs.
# Usage: tools/gpu_quick.sh TAG [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.out" 2>&1
rc=$?; echo "pytest rc=$rc" >&2; grep -E "passed|failed|Error|error" "$OUT/pytest_gpu.out" | tail -15 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline --no-secondary "$@" > "$OUT/bench.out" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" >&2; tail -3 "$OUT/bench.err" >&2; tail -1 "$OUT/bench.out" >&2
exit $rc
